# wide prelude on a compact frame list: tie tests, FD_REF_WIDE A/B on the north-star tie batch, bench tie legs
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04j
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ties.py tests/test_gpu_select_custom.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j/ties.log 2>&1 || { tail -40 gpurun_out/r04j/ties.log; exit 1; }
tail -1 gpurun_out/r04j/ties.log
bash tools/gpu_env_ab.sh refwide2 "nsties" "FD_REF_WIDE=0" "FD_REF_WIDE=1" > gpurun_out/r04j/ab.txt 2>&1
grep -E "k_select_ref|k_refw" gpurun_out/r04j/ab.txt | head -40
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04j/bench.json 2> gpurun_out/r04j/bench.err
python3 -c "
import json; d=json.loads(open('gpurun_out/r04j/bench.json').read().strip().splitlines()[-1])
def walk(o,p=''):
    if isinstance(o,dict):
        for k,v in o.items(): walk(v,p+'.'+k)
    elif 'ties' in p and ('ms' in p or 'vs' in p or 'resolved' in p) or p in ('.value','.ms_per_step'): print(p,o)
walk(d)"
