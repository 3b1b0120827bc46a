# K10 counters at the conv1b and conv2a shapes (tools/sp_k10_probe.py): the probe's own timing, then one
# rocprofv3 --pmc pass per counter set (separate runs). usage: bash tools/sp_k10_pmc.sh [TAG]
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-k10}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for L in conv1b conv2a; do
  timeout -k 10 120 python3 tools/sp_k10_probe.py --layer $L --calls 10 | tee -a $O/timing.txt
done
run() {  # name layer counters...
  local name=$1 layer=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/raw -o $name \
      -- python3 tools/sp_k10_probe.py --layer $layer --calls 3 > $O/$name.log 2>&1
  for c in "$@"; do python3 tools/pmc_summary.py $O/raw/${name}_counter_collection.csv $c | grep c64 | sed "s/^/$name,/" >> $O/summary.csv; done
}
for L in conv1b conv2a; do
  run ${L}_a $L SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES
  run ${L}_b $L SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
  run ${L}_c $L SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE || echo "pass c failed"
done
rm -rf $O/raw
cat $O/summary.csv
