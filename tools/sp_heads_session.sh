# SuperPoint heads: merged convPa/convDa + GEMM 1x1 heads (default) vs the separate convolutions
# (FD_SP_HEADS_MM=0), after the NN tests; then one kernel trace of the default forward.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sph
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sph/tests.log 2>&1 || { tail -40 gpurun_out/sph/tests.log; exit 1; }
tail -1 gpurun_out/sph/tests.log
for r in 1 2; do
  FD_DEBUG_AB=1 FD_SP_HEADS_MM=0 timeout -k 10 120 python3 tools/sp_forward_time.py | sed "s/^/separate /"
  FD_DEBUG_AB=1 timeout -k 10 120 python3 tools/sp_forward_time.py | sed "s/^/merged+gemm /"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sph/trace -o run -- python3 tools/sp_layer_prof.py > gpurun_out/sph/trace.log 2>&1
