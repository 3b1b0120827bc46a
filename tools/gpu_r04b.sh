# Round 4 measurement call: plain bench line, the rocprofv3 kernel summary of the bench by leg, the PMC
# traffic / SQ passes (tools/gpu_round_pmc.sh), and diagnostic SQ / TA passes of the north-star kernel and
# the LSD map (padded vs unpadded rows). usage: bash tools/gpu_r04b.sh
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 900 python3 bench.py > $O/bench_plain.json 2> $O/bench_plain.err
tail -c 600 $O/bench_plain.json
bash tools/gpu_round_bench.sh r04
bash tools/gpu_round_pmc.sh r04
D=$O/diag; mkdir -p $D
pmc() {  # name shape-args -- counters...
  local name=$1; local shape=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $D/raw -o $name -- python3 tools/profile_kernels.py $shape --calls 2 > $D/$name.log 2>&1
  for c in "$@"; do python3 tools/pmc_summary.py $D/raw/${name}_counter_collection.csv $c | sed "s/^/$name,/" >> $D/summary.csv; done
}
pmc ns1 "--shape northstar --kind shi_tomasi" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
pmc ns2 "--shape northstar --kind shi_tomasi" SQ_ACTIVE_INST_VALU2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc lsdu_ta "--shape lsd --kind dense_unpitched" TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE
pmc lsdp_ta "--shape lsd --kind dense" TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE
pmc lsdu_sq "--shape lsd --kind dense_unpitched" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc lsdp_sq "--shape lsd --kind dense" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc lsdu_f "--shape lsd --kind dense_unpitched" FETCH_SIZE
pmc lsdu_w "--shape lsd --kind dense_unpitched" WRITE_SIZE
rm -rf $D/raw
grep -E "k_corner_lp|k_lsd_map" $D/summary.csv
echo done
