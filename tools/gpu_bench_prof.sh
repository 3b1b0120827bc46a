# rocprofv3 kernel-trace summary of the bench command itself (profiles/<tag>_bench_kernel_stats.csv)
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out/bp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/bp/raw -o bench -- python3 bench.py > gpurun_out/bp/bench.json 2>gpurun_out/bp/bench.err
python3 tools/rocpd_summary.py gpurun_out/bp/raw/bench_results.db > gpurun_out/bp/${TAG}_bench_kernel_stats.csv
rm -rf gpurun_out/bp/raw
echo ok
