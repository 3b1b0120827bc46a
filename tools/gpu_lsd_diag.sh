# LSD map diagnostics: counters available on this GPU, SQ issue/wait and TA counters of k_lsd_map
# (dense, 1080p x256), and the map's wave-count A/B. usage: bash tools/gpu_lsd_diag.sh [suffix] [noab]
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/lsd_diag${1:-}; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "TA_[A-Z_]*\|TD_[A-Z_]*\|TCP_[A-Z_]*" $O/avail.txt | sort -u > $O/avail_ta.txt || true
pmc() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/raw -o $name -- python3 tools/profile_kernels.py --shape lsd --kind dense --calls 2 > $O/$name.log 2>&1
  for c in "$@"; do python3 tools/pmc_summary.py $O/raw/${name}_counter_collection.csv $c | sed "s/^/$name,/" >> $O/summary.csv; done
}
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_WAIT_ANY GRBM_GUI_ACTIVE
pmc ta TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum GRBM_GUI_ACTIVE
rm -rf $O/raw
grep k_lsd_map $O/summary.csv
[ "${2:-}" = noab ] || bash tools/gpu_env_ab.sh lsdw "lsd --kind dense --calls 3" "FD_LSD_WAVES=16384" "FD_LSD_WAVES=8192" "FD_LSD_WAVES=32768" "FD_LSD_WAVES=4096" "FD_LSD_WAVES=16384"
