# rocprofv3 kernel-trace summary of the bench command itself, per bench leg (roctx phases):
# profiles/<tag>_bench_kernel_stats.csv (by phase) and <tag>_bench_kernel_stats_total.csv.
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/bp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/bp/raw -o bench -- python3 bench.py > gpurun_out/bp/bench.json 2>gpurun_out/bp/bench.err
DB=$(find gpurun_out/bp/raw -name '*.db' | head -1)
python3 tools/rocpd_summary.py --phases "$DB" > gpurun_out/bp/${TAG}_bench_kernel_stats.csv
python3 tools/rocpd_summary.py "$DB" > gpurun_out/bp/${TAG}_bench_kernel_stats_total.csv
rm -rf gpurun_out/bp/raw
echo ok
