# Selection tests + phase clocks + bench (headline only).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_select.py tests/test_gpu_points.py -m gpu -x -q > gpurun_out/tests.log 2>&1
FD_SELECT_STAMPS=1 timeout -k 10 300 python3 tools/select_stamps.py > gpurun_out/stamps.log 2>&1
timeout -k 10 300 python3 bench.py --no-north-star --no-config3 --no-cpu-baseline > gpurun_out/bench_quick.json 2>gpurun_out/bench_quick.err
