# SQ/GRBM counters for the north-star per-pixel kernel (separate --pmc passes, kernel trace only).
# usage: bash tools/gpu_pmc.sh <tag> <kind>
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-pmc}; KIND=${2:-shi_tomasi}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/sq -o sq -- python3 tools/profile_kernels.py --shape northstar --kind $KIND --calls 3 > gpurun_out/$TAG/sq.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_COUNT --output-format csv -d gpurun_out/$TAG/sq2 -o sq2 -- python3 tools/profile_kernels.py --shape northstar --kind $KIND --calls 3 > gpurun_out/$TAG/sq2.log 2>&1
find gpurun_out/$TAG -name "*.csv" | head
echo ok
