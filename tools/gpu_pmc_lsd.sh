# SQ / TCC counters of the LSD kernels (lsd_probe.py: 1920x1080 x 256 checker frames), one pass per group.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcl
run() {
  timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmcl/$1 -o $1 -- python3 tools/lsd_probe.py A=0 > gpurun_out/pmcl/$1.log 2>&1
  f=$(find gpurun_out/pmcl/$1 -name '*counter_collection.csv' | head -1)
  for c in $2; do python3 tools/pmc_summary.py "$f" $c | grep -i lsd || true; done
}
run a "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
run b "FETCH_SIZE"
run c "WRITE_SIZE"
run d "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
echo ok
