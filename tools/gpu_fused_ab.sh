set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fab
for v in "1 0" "1 1" "1 2" "0 0"; do set -- $v
  FD_FUSED_GATHER=$1 FD_FUSED_DBG=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fab/r$1$2 -o r -- python3 tools/k1_batch1.py detect > gpurun_out/fab/r$1$2.log 2>&1
  echo "== fused=$1 dbg=$2"; python3 tools/rocpd_summary.py $(find gpurun_out/fab/r$1$2 -name '*.db' | head -1) | grep -i "corner\|select" | cut -c1-20,80-200
done
