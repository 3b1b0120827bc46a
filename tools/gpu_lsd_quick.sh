set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lsd.py tests/test_cpp_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lsd_tests.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_plain.json 2>gpurun_out/bench_plain.err
