# K10 group-tile A/B: abvar/base.so (8 x 32, XCD-aware) vs abvar/new.so (16 x 16) vs abvar/noxcd.so (8 x 32, plain
# dealing): the NN tests on new, the layer probes and the forward, alternating twice
set -e
cd $GRAFT_REPO_ROOT
FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/new.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k10s_tests.log 2>&1 || { tail -30 gpurun_out/k10s_tests.log; exit 1; }
tail -1 gpurun_out/k10s_tests.log
for r in 1 2; do
  for L in base new noxcd; do
    for ly in conv1b conv2a conv3a; do
      FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 60 python3 tools/sp_k10_probe.py --layer $ly --calls 10 | sed "s/^/$L /"
    done
    FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 120 python3 tools/sp_forward_time.py
  done
done
