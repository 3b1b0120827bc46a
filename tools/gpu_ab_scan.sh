# DPP wave scans (K1 sorted-segment flush, k_select suffix, k_gather) vs shuffle scans: GPU tests of the
# point/selection paths, headline-shape A/B of the two builds, then the LSD diagnostics.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_points.py tests/test_gpu_select.py tests/test_gpu_ties.py tests/test_gpu_nn.py tests/test_gpu_select_custom.py > gpurun_out/scan_tests.log 2>&1 || { tail -30 gpurun_out/scan_tests.log; exit 1; }
tail -2 gpurun_out/scan_tests.log
bash tools/gpu_ab_libs.sh bench abvar/base.so abvar/new.so abvar/base.so abvar/new.so
bash tools/gpu_ab_libs.sh "northstar --kind shi_tomasi" abvar/base.so abvar/new.so abvar/base.so abvar/new.so
bash tools/gpu_lsd_diag.sh
