# SuperPoint first layers: layered (conv1a pass + K10) vs fused (conv1a inside K10's housekeeping phase),
# after the NN tests. usage: bash tools/k10_fused_session.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k10f
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k10f/tests.log 2>&1 || { tail -40 gpurun_out/k10f/tests.log; exit 1; }
tail -2 gpurun_out/k10f/tests.log
for r in 1 2; do
  FD_DEBUG_AB=1 timeout -k 10 120 python3 tools/sp_forward_time.py | sed "s/^/layered /"
  FD_DEBUG_AB=1 FD_SP_C1C64=1 timeout -k 10 120 python3 tools/sp_forward_time.py | sed "s/^/fused /"
done
