# SQ counters + HBM traffic of one profile_kernels.py shape (separate --pmc passes, kernel trace only).
# usage: bash tools/gpu_pmc.sh <tag> <shape> [kind] [calls]
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-pmc}; SHAPE=${2:-northstar}; KIND=${3:-}; CALLS=${4:-3}
ARGS="--shape $SHAPE --calls $CALLS"; [ -n "$KIND" ] && ARGS="$ARGS --kind $KIND"
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/$TAG/raw -o $name -- python3 tools/profile_kernels.py $ARGS > gpurun_out/$TAG/$name.log 2>&1
  for c in "$@"; do python3 tools/pmc_summary.py gpurun_out/$TAG/raw/${name}_counter_collection.csv $c >> gpurun_out/$TAG/summary.csv; done
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass sq2 SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_COUNT
pass fetch FETCH_SIZE
pass write WRITE_SIZE
rm -rf gpurun_out/$TAG/raw
cat gpurun_out/$TAG/summary.csv
