set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_points.py tests/test_gpu_select.py tests/test_gpu_ties.py tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
FD_SELECT_STAMPS=1 timeout -k 10 100 python3 tools/select_stamps_fast.py 2>&1 | grep -A2 "k_select cycles" | tail -3
timeout -k 10 300 python3 bench.py --steps 50 --no-config3 --no-superpoint --no-lsd --no-cpu-baseline > gpurun_out/b.json 2>/dev/null
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['value'],d['ms_per_step'],d['north_star']['ms_per_step'],d['north_star']['kernel_ms'])"
