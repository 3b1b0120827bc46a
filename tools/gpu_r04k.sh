# k_select_reference with the register-resident sort of 17..64-element ranges: tie tests, phase clocks,
# wave-local cutoff A/B (FD_REF_WL builds in abvar/) on the headline and north-star tie shapes
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04k
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ties.py tests/test_gpu_select_custom.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k/ties.log 2>&1 || { tail -40 gpurun_out/r04k/ties.log; exit 1; }
tail -1 gpurun_out/r04k/ties.log
FD_SELECT_STAMPS=1 timeout -k 10 300 python3 tools/ref_stamps.py > gpurun_out/r04k/stamps.txt 2>&1
grep "k_select_reference" gpurun_out/r04k/stamps.txt | tail -6
bash tools/gpu_ab_libs.sh ties abvar/wl128.so feature_detector_amd/lib/libfdhip.so abvar/wl512.so > gpurun_out/r04k/ab_ties.txt 2>&1
bash tools/gpu_ab_libs.sh nsties abvar/wl128.so feature_detector_amd/lib/libfdhip.so abvar/wl512.so > gpurun_out/r04k/ab_nsties.txt 2>&1
grep k_select_ref gpurun_out/r04k/ab_ties.txt gpurun_out/r04k/ab_nsties.txt
for W in 0 1; do
FD_REF_WIDE=$W timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04k/bench_w$W.json 2> gpurun_out/r04k/bench_w$W.err
python3 -c "
import json; d=json.loads(open('gpurun_out/r04k/bench_w$W.json').read().strip().splitlines()[-1])
print('FD_REF_WIDE=$W headline', d['ms_per_step'], d['ties'].get('reference_order_ms_per_step'), d['ties'].get('reference_vs_raster_step'),
      'north_star', d['north_star']['ties'].get('reference_order_ms_per_step'), d['north_star']['ties'].get('reference_vs_raster_step'))"
done
