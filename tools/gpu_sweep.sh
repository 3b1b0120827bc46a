set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/k1_tests.log 2>&1
timeout -k 10 300 python tools/sweep_tiles.py shi_tomasi 1080 1920 256 response 2560,5120,10240,20480 100 > gpurun_out/sweep_ns.log 2>&1
timeout -k 10 300 python tools/sweep_tiles.py harris 1080 1920 256 response 5120,10240 100 >> gpurun_out/sweep_ns.log 2>&1
timeout -k 10 300 python tools/sweep_tiles.py shi_tomasi 1080 1920 256 detect 5120,10240 100 >> gpurun_out/sweep_ns.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/k1_bench.log 2>&1
echo ok
