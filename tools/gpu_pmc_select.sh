# SQ / SQC counters of k_select at the headline shape (Harris 640x480 batch 1), one pass per group.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcs
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmcs/$1 -o $1 -- python3 tools/k1_batch1.py detect > gpurun_out/pmcs/$1.log 2>&1
  f=$(find gpurun_out/pmcs/$1 -name '*counter_collection.csv' | head -1)
  for c in $2; do python3 tools/pmc_summary.py "$f" $c | grep -i select || true; done
}
run a "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
run b "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH"
run c "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE"
echo ok
