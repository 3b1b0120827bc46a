# GPU tests (stop at first failure), then a kernel-trace profile of one profile_kernels.py shape.
# usage: bash tools/gpu_check_prof.sh <tag> <shape> [kind]
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-chk}; SHAPE=${2:-fast720}; KIND=${3:-}
ARGS="--shape $SHAPE"; [ -n "$KIND" ] && ARGS="$ARGS --kind $KIND"
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -60 gpurun_out/$TAG/tests.log; exit 1; }
tail -3 gpurun_out/$TAG/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 tools/profile_kernels.py $ARGS > gpurun_out/$TAG/prof.log 2>&1
python3 - <<PY
import csv,glob
for f in glob.glob("gpurun_out/$TAG/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:90], r["Calls"], r["AverageNs"])
PY
