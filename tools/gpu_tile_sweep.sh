set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ts
for h in 6 4 3 2 1; do
  FD_TILE_H=$h timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ts/h$h -o r -- python3 tools/k1_batch1.py detect > /dev/null 2>&1
  echo "== tile_h=$h"; python3 tools/rocpd_summary.py $(find gpurun_out/ts/h$h -name '*.db' | head -1) | grep -i "corner\|select" | cut -c1-30,70-200
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_points.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tp.log 2>&1
FD_TILE_H=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_points.py tests/test_gpu_select.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tp2.log 2>&1
