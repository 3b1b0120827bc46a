# 64 -> 64 matrix-core convolution A/B: the working build (libfdhip) vs the previous build (abvar/head.so)
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04p
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04p/nn.log 2>&1 || { tail -30 gpurun_out/r04p/nn.log; exit 1; }
tail -1 gpurun_out/r04p/nn.log
for L in feature_detector_amd/lib/libfdhip.so abvar/head.so; do
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04p/prof -o run -- python3 tools/sp_layer_prof.py > gpurun_out/r04p/prof.log 2>&1
  f=$(find gpurun_out/r04p/prof -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'conv3x3' in r['Name']: print('$L', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
  rm -rf gpurun_out/r04p/prof
done
timeout -k 10 300 python3 tools/sp_fused_ab.py > gpurun_out/r04p/sp_ab.txt 2>&1 || true
grep round gpurun_out/r04p/sp_ab.txt
