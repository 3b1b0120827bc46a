# Tie-order radix pre-sort and LSD map rows stored as contiguous dwords through LDS: GPU tests, LSD A/B of
# two builds, then the TA / SQ memory-instruction diagnostics (tools/gpu_ta_diag.sh without its tests).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_ties.py tests/test_cpp_api.py tests/test_gpu_select_custom.py tests/test_gpu_lsd.py tests/test_gpu_lines.py > gpurun_out/r3b_tests.log 2>&1 || { tail -30 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
bash tools/gpu_ab_libs.sh "lsd --kind dense --calls 3" abvar/base.so abvar/new.so abvar/base.so abvar/new.so
SKIP_TESTS=1 bash tools/gpu_ta_diag.sh
