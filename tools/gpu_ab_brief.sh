# LDS-staged BRIEF patches + k_select suffix totals by one read and a DPP sum: GPU tests (BRIEF, points,
# selection), configs[2] and headline A/B of two builds.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_brief.py tests/test_gpu_points.py tests/test_gpu_select.py tests/test_gpu_ties.py > gpurun_out/brief_tests.log 2>&1 || { tail -30 gpurun_out/brief_tests.log; exit 1; }
tail -2 gpurun_out/brief_tests.log
bash tools/gpu_ab_libs.sh fastbrief abvar/base.so abvar/new.so abvar/base.so abvar/new.so
bash tools/gpu_ab_libs.sh bench abvar/base.so abvar/new.so abvar/base.so abvar/new.so
