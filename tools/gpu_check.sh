set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
FD_SELECT_STAMPS=1 timeout -k 10 200 python tools/select_stamps.py > gpurun_out/stamps.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/k1_bench.log 2>&1
bash tools/gpu_prof.sh p2 > /dev/null 2>&1
echo ok
