# rocprofv3 per-phase kernel summary of a bench run restricted to the given legs (bench args).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pl
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/pl/raw -o bench -- python3 bench.py "$@" > gpurun_out/pl/bench.json 2>gpurun_out/pl/bench.err
DB=$(find gpurun_out/pl/raw -name '*.db' | head -1)
python3 tools/rocpd_summary.py --phases "$DB" > gpurun_out/pl/stats.csv
rm -rf gpurun_out/pl/raw
