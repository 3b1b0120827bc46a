# A/B of library builds (FD_LIB_PATH) on one profile_kernels.py shape, each under rocprofv3
# --kernel-trace --stats. usage: bash tools/gpu_ab_libs.sh "<shape> [profile_kernels args]" lib1 lib2 ...
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/abl
SHAPE=$1; shift
for L in "$@"; do
  n=$(basename $L .so)_$RANDOM
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$n -o run -- python3 tools/profile_kernels.py --shape $SHAPE > gpurun_out/abl/$n.log 2>&1
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/abl/$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fdk::' in r['Name']: print('$L', r['Name'].replace('void ','')[:45], r['Calls'], r['AverageNs'], r['MinNs'])
"
  rm -rf gpurun_out/abl/$n
done
