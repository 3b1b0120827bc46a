# Headline tile-height sweep on one library build (FD_TILE_H overrides choose_tile_h), rocprofv3 kernel
# stats of 200 fd_points_detect calls each. usage: bash tools/gpu_tile_sweep.sh lib.so h1 h2 ...
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/abl
LIB=$1; shift
for H in "$@"; do
  n=tile$H_$RANDOM
  FD_TILE_H=$H FD_LIB_PATH=$GRAFT_REPO_ROOT/$LIB timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$n -o run -- python3 tools/profile_kernels.py --shape bench > gpurun_out/abl/$n.log 2>&1
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/abl/$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fdk::' in r['Name']: print('tile_h=$H', r['Name'].replace('void ','')[:45], r['Calls'], r['AverageNs'], r['MinNs'])
"
  rm -rf gpurun_out/abl/$n
done
