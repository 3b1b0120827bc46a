# Latency-chain trims (constant-trip cross-wave sums in k_select / k_gather / k_lsd_scan, LSD scan 4 per
# thread): GPU tests, headline and LSD A/B of two builds, k_select phase clocks at the headline shape.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_points.py tests/test_gpu_select.py tests/test_gpu_ties.py tests/test_gpu_lsd.py tests/test_gpu_lines.py tests/test_gpu_nn.py > gpurun_out/hl_tests.log 2>&1 || { tail -30 gpurun_out/hl_tests.log; exit 1; }
tail -2 gpurun_out/hl_tests.log
bash tools/gpu_ab_libs.sh bench abvar/base.so abvar/new.so abvar/base.so abvar/new.so
bash tools/gpu_ab_libs.sh "lsd --kind dense --calls 3" abvar/base.so abvar/new.so
FD_SELECT_STAMPS=1 timeout -k 10 200 python3 tools/select_stamps.py > gpurun_out/stamps_hl.txt 2>&1
grep -A1 "cycles" gpurun_out/stamps_hl.txt | head -12
