# Whole GPU suite + smoke() (what the driver runs at round end).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
