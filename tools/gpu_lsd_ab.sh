# LSD map store alignment: store-shape probe, LSD GPU tests on the new build, dense-map A/B of two
# builds (FD_LIB_PATH), then k_select phase clocks at the headline shape.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 5 120 tools/calib/store_probe > gpurun_out/store_probe.txt 2>&1
cat gpurun_out/store_probe.txt
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lsd.py tests/test_gpu_lines.py > gpurun_out/lsd_tests.log 2>&1 || { tail -30 gpurun_out/lsd_tests.log; exit 1; }
tail -2 gpurun_out/lsd_tests.log
bash tools/gpu_ab_libs.sh "lsd --kind dense --calls 3" abvar/base.so abvar/new.so abvar/new2.so abvar/base.so abvar/new.so abvar/new2.so
bash tools/gpu_ab_libs.sh "lsd --kind compact --calls 3" abvar/base.so abvar/new2.so
FD_SELECT_STAMPS=1 timeout -k 10 200 python3 tools/select_stamps.py > gpurun_out/stamps_hl.txt 2>&1
grep -A1 "cycles" gpurun_out/stamps_hl.txt | head -8
