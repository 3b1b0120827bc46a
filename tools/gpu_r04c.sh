# Round 4 session C: tie tests + a bench-shape timing of the reference tie order (k_select_reference with
# pipelined partition passes), the raw v_sqrt_f32 accuracy probe, then the GPU suite.
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04c
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ties.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c/ties.log 2>&1 || { tail -30 gpurun_out/r04c/ties.log; exit 1; }
tail -2 gpurun_out/r04c/ties.log
timeout -k 10 300 python3 bench.py --steps 50 --no-config3 --no-lsd --no-superpoint --no-cpu-baseline > gpurun_out/r04c/bench_ties.json 2> gpurun_out/r04c/bench_ties.err
python3 -c "
import json; d=json.load(open('gpurun_out/r04c/bench_ties.json'))
print('headline', d['value'], d['ms_per_step'], d['ties'])
print('north_star', d['north_star']['kernel_ms'], d['north_star']['ms_per_step'], d['north_star']['ties'])"
timeout -k 10 300 tools/calib/sqrt_raw > gpurun_out/r04c/sqrt_raw.txt 2>&1; cat gpurun_out/r04c/sqrt_raw.txt
bash tools/gpu_tests_smoke.sh
