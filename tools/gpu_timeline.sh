set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl/raw -o bench -- python3 bench.py --steps 32 --warmup 16 --cpu-seconds 0 --no-north-star > gpurun_out/tl/bench.log 2>&1
python3 tools/timeline.py gpurun_out/tl/raw/bench_results.db 100000 > gpurun_out/tl/timeline.txt
FD_GATHER_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl/raw -o slow -- python3 bench.py --steps 32 --warmup 16 --cpu-seconds 0 --no-north-star > gpurun_out/tl/slow.log 2>&1
python3 tools/timeline.py gpurun_out/tl/raw/slow_results.db 100000 > gpurun_out/tl/timeline_slow.txt

echo ok
