set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nn.log 2>&1 || { tail -30 gpurun_out/nn.log; exit 1; }
tail -2 gpurun_out/nn.log
timeout -k 10 500 python3 bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
python3 -c "
import json;d=json.load(open('gpurun_out/bench_full.json'))
print(d['value'], d['ms_per_step']); print(json.dumps(d['config4_lsd_map']['lines'])); print(d['config3_fast_brief']['ms_per_step'])"
