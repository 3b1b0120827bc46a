# k_select_reference: tie tests, then phase clocks on the bench tie frames (tools/ref_stamps.py)
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04d
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ties.py tests/test_gpu_select_custom.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d/ties.log 2>&1 || { tail -30 gpurun_out/r04d/ties.log; exit 1; }
tail -1 gpurun_out/r04d/ties.log
FD_SELECT_STAMPS=1 timeout -k 10 300 python3 tools/ref_stamps.py > gpurun_out/r04d/stamps.txt 2>&1
grep "k_select_reference" gpurun_out/r04d/stamps.txt | tail -30
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04d/bench.json 2> gpurun_out/r04d/bench.err
python3 -c "
import json; d=json.loads(open('gpurun_out/r04d/bench.json').read().strip().splitlines()[-1])
def walk(o,p=''):
    if isinstance(o,dict):
        for k,v in o.items(): walk(v,p+'.'+k)
    elif 'ties' in p or p in ('.value','.ms_per_step'): print(p,o)
walk(d)"
