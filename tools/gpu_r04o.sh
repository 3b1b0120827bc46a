# 64 -> 64 matrix-core convolution: 8-row tiles (abvar/c64rows8.so) vs the 4-row default -- NN tests on the
# 8-row build, kernel summaries of both, and the SuperPoint forward A/B on the default build
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04o
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o/nn.log 2>&1 || { tail -30 gpurun_out/r04o/nn.log; exit 1; }
tail -1 gpurun_out/r04o/nn.log
FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/c64rows8.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_nn.py -x -q --timeout 120 --timeout-method thread -k "conv64 or bias_relu" > gpurun_out/r04o/nn8.log 2>&1 || { tail -30 gpurun_out/r04o/nn8.log; exit 1; }
tail -1 gpurun_out/r04o/nn8.log
for L in feature_detector_amd/lib/libfdhip.so abvar/c64rows8.so; do
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o/prof -o run -- python3 tools/sp_layer_prof.py > gpurun_out/r04o/prof.log 2>&1
  f=$(find gpurun_out/r04o/prof -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'conv3x3' in r['Name']: print('$L', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
"
  rm -rf gpurun_out/r04o/prof
done
timeout -k 10 300 python3 tools/sp_fused_ab.py > gpurun_out/r04o/sp_ab.txt 2>&1 || true
grep round gpurun_out/r04o/sp_ab.txt
