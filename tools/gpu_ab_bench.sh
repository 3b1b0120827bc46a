# Bench A/B of library builds: headline step, K1 and north-star kernel per build, alternating.
# usage: bash tools/gpu_ab_bench.sh lib1 lib2 [rounds]
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/abb
A=$1; B=$2; R=${3:-2}
for i in $(seq $R); do for L in $A $B; do
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python3 bench.py --steps 200 --no-config3 --no-superpoint --no-lsd --no-cpu-baseline > gpurun_out/abb/b.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/abb/b.json'));print('$L', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['north_star']['kernel_ms'], d['north_star']['ms_per_step'])"
done; done
