# SuperPoint conv3a (64 -> 128) as two 64-channel blocks of the matrix-core convolution: NN tests, forward A/B
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04q
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q/nn.log 2>&1 || { tail -30 gpurun_out/r04q/nn.log; exit 1; }
tail -1 gpurun_out/r04q/nn.log
timeout -k 10 300 python3 tools/sp_fused_ab.py > gpurun_out/r04q/sp_ab.txt 2>&1 || true
grep round gpurun_out/r04q/sp_ab.txt
