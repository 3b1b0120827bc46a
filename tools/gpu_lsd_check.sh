# LSD: GPU parity tests, then the bench LSD leg alone.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lsd.py tests/test_gpu_lines.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lsdt.log 2>&1 || { tail -30 gpurun_out/lsdt.log; exit 1; }
tail -1 gpurun_out/lsdt.log
timeout -k 10 300 python3 bench.py --steps 10 --no-config3 --no-superpoint --no-cpu-baseline > gpurun_out/lsdb.json 2>/dev/null
python3 -c "import json;d=json.load(open('gpurun_out/lsdb.json'))['config4_lsd_map'];print(d['ms_per_batch'], d['roofline']['frac'], d['lines']['ms_per_batch'])"
