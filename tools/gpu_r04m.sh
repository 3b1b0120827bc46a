# SuperPoint first layer as one HIP pass (fd_nn_conv3x3_c1): NN tests, then the network probe and the
# SuperPoint bench leg
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04m
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_nn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m/nn.log 2>&1 || { tail -40 gpurun_out/r04m/nn.log; exit 1; }
tail -1 gpurun_out/r04m/nn.log
timeout -k 10 300 python3 tools/sp_fused_ab.py > gpurun_out/r04m/sp_ab.txt 2>&1 || true
tail -12 gpurun_out/r04m/sp_ab.txt
