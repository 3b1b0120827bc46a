set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 60 python3 tools/sp_k10_probe.py --layer conv1b --calls 10
  timeout -k 10 60 python3 tools/sp_k10_probe.py --layer conv1b --calls 10 --zero
done
timeout -k 10 120 python3 -c "
import sys, torch; sys.path.insert(0, '.')
import bench
print(bench.copy_bandwidth(torch, torch.device('cuda')))
"
