# GPU points tests, plain bench, then the rocprofv3 summary of the same bench command.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python3 -m pytest tests/test_gpu_points.py -x -q > gpurun_out/tp.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_plain.json 2>gpurun_out/bench_plain.err
bash tools/gpu_bench_prof.sh ${1:-r01}
