set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_points.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ingest_tests.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_plain.json 2>gpurun_out/bench_plain.err
