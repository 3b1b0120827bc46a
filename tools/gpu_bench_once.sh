set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
tail -c 3000 gpurun_out/bench_full.json
MIOPEN_FIND_MODE=FAST timeout -k 10 300 python3 bench.py --steps 20 --no-north-star --no-config3 --no-lsd --no-cpu-baseline > gpurun_out/bench_fast.json 2> gpurun_out/bench_fast.err
python3 -c "import json;d=json.load(open('gpurun_out/bench_fast.json'));print(d['config5_superpoint'])"
