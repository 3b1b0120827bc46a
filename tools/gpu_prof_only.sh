# kernel-trace profile of one profile_kernels.py shape. usage: bash tools/gpu_prof_only.sh <tag> <shape> [kind]
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=${1:-p}; SHAPE=${2:-fast720}; KIND=${3:-}
ARGS="--shape $SHAPE"; [ -n "$KIND" ] && ARGS="$ARGS --kind $KIND"
mkdir -p gpurun_out/$TAG
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 tools/profile_kernels.py $ARGS > gpurun_out/$TAG/prof.log 2>&1
python3 - <<PY
import csv,glob
for f in glob.glob("gpurun_out/$TAG/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Name"].startswith("void fdk"): print(r["Name"][:70], r["Calls"], r["AverageNs"])
PY
