# k_select at the headline shape: instruction-cache and wave-state counters (one rocprofv3 --pmc pass per
# set; a set rocprofv3 rejects is reported and skipped). usage: bash tools/ksel_icache.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/icache
mkdir -p $O
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -iE "icache|ifetch|SQC_INST|INST_LEVEL" $O/avail.txt | head -40 > $O/avail_icache.txt || true
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/raw -o $name -- python3 tools/ksel_icache_probe.py > $O/$name.log 2>&1 || { echo "$name failed"; return 0; }
  for c in "$@"; do python3 tools/pmc_summary.py $O/raw/${name}_counter_collection.csv $c | grep k_select | sed "s/^/$name,/" >> $O/summary.csv; done
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU
run sqc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ
rm -rf $O/raw
cat $O/summary.csv; cat $O/avail_icache.txt
