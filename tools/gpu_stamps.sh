set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FD_SELECT_STAMPS=1 timeout -k 10 300 python3 tools/select_stamps.py > gpurun_out/stamps.log 2>&1
