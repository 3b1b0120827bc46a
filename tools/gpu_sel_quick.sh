# Selection change check: select + points GPU tests, phase clocks, plain bench line.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_select.py tests/test_gpu_points.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
FD_SELECT_STAMPS=1 timeout -k 10 120 python3 tools/select_stamps.py > gpurun_out/stamps.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_plain.json 2>gpurun_out/bench_plain.err
