# Full GPU pass: the gpu test suite, smoke(), the plain bench line, then the rocprofv3 summary of it.
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_plain.json 2>gpurun_out/bench_plain.err
bash tools/gpu_bench_prof.sh $TAG
