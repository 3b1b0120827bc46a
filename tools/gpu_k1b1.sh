set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/k1b1
for tw in 10240 1024 256; do
  for mode in detect response; do
    FD_TARGET_WAVES=$tw timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/k1b1/raw -o ${mode}_$tw -- python3 tools/k1_batch1.py $mode > /dev/null 2>&1
    python3 tools/rocpd_summary.py gpurun_out/k1b1/raw/${mode}_${tw}_results.db | grep -E "k_corner|k_select" | sed "s/^/$mode tw=$tw /" >> gpurun_out/k1b1/summary.txt
  done
done
rm -rf gpurun_out/k1b1/raw
echo ok
