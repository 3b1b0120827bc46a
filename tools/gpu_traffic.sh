# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) for the calibration kernel and the
# per-pixel kernels at the bench and north-star shapes. usage: bash tools/gpu_traffic.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-traffic}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/$TAG/raw -o ${name}_$ctr -- "$@" > gpurun_out/$TAG/${name}_$ctr.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/$TAG/raw/${name}_${ctr}_counter_collection.csv $ctr >> gpurun_out/$TAG/summary.csv
}
for ctr in FETCH_SIZE WRITE_SIZE; do
  run calib $ctr tools/calib/fetch_calib
  run bench $ctr python3 tools/k1_batch1.py detect
  run northstar $ctr python3 tools/profile_kernels.py --shape northstar --kind shi_tomasi --calls 3
done
rm -rf gpurun_out/$TAG/raw
echo ok
