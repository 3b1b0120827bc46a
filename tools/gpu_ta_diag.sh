# TA (vector-memory address unit) and SQ memory-instruction counters of k_fast (configs[2] detect) and the
# north-star K1 (fd_points_response): is either bound by its memory instructions rather than VALU?
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/ta_diag; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_ties.py tests/test_cpp_api.py tests/test_gpu_select_custom.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 $O/tests.log
pmc() {  # name shape counters...
  local name=$1 shape=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/raw -o $name -- python3 tools/profile_kernels.py --shape $shape --calls 2 > $O/$name.log 2>&1
  for c in "$@"; do python3 tools/pmc_summary.py $O/raw/${name}_counter_collection.csv $c | sed "s/^/$name,/" >> $O/summary.csv; done
}
pmc fast_ta fast720 TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
pmc fast_sq fast720 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
pmc ns_ta northstar TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE
pmc brief_ta fastbrief TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
rm -rf $O/raw
grep -E "k_fast|k_corner|k_brief|k_select" $O/summary.csv
