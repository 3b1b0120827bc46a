# k_select A/B (abvar/base.so vs abvar/new.so): the selection / point / tie tests on new, the headline
# kernel stats alternating twice, and new's phase clocks
set -e
cd $GRAFT_REPO_ROOT
FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/new.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_select.py tests/test_gpu_select_custom.py tests/test_gpu_points.py tests/test_gpu_ties.py tests/test_gpu_fast_cut.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/selab_tests.log 2>&1 || { tail -30 gpurun_out/selab_tests.log; exit 1; }
tail -1 gpurun_out/selab_tests.log
bash tools/gpu_session.sh ab=bench stamps=abvar/new.so
