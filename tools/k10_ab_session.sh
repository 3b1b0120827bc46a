set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k10b
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k10b/tests.log 2>&1 || { tail -40 gpurun_out/k10b/tests.log; exit 1; }
tail -2 gpurun_out/k10b/tests.log
for L in base new base new; do
  for ly in conv1b conv2a conv2b conv3a; do
    FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 60 python3 tools/sp_k10_probe.py --layer $ly --calls 10 | sed "s/^/$L /"
  done
done
for L in base new base new; do
  FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 120 python3 tools/sp_forward_time.py
done
