# Fused bias + ReLU (+ pool) in the SuperPoint forward: NN GPU tests, then the configs[4] forward A/B.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nn.py tests/test_capi_symbols.py -s > gpurun_out/sp_tests.log 2>&1 || { tail -30 gpurun_out/sp_tests.log; exit 1; }
grep "fused vs" gpurun_out/sp_tests.log; tail -2 gpurun_out/sp_tests.log
timeout -k 10 400 python3 -u tools/sp_fused_ab.py 2>&1 | grep -v amdgpu.ids
