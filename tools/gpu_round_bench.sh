# Round profile pass, part 1: rocprofv3 kernel-trace summary of the bench command itself, per bench
# leg (roctx phases). usage: bash tools/gpu_round_bench.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
export TMPDIR=/tmp
O=gpurun_out/$TAG/bench
mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace --stats -d $O/raw -o bench -- python3 bench.py > $O/bench.json 2>$O/bench.err
DB=$(find $O/raw -name '*.db' | head -1)
python3 tools/rocpd_summary.py --phases "$DB" > $O/${TAG}_bench_kernel_stats.csv
python3 tools/rocpd_summary.py "$DB" > $O/${TAG}_bench_kernel_stats_total.csv
rm -rf $O/raw
echo ok
