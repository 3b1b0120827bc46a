# Timing-only knockout A/B (profiles/r03_k1_hist_ko.txt): abvar/base.so = HEAD, abvar/kohist.so = HEAD with
# hist_flush (fd_corner_common.h) adding only when (logical_block() & 7) == 0; both under rocprofv3 kernel stats.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/abl
for L in abvar/base.so abvar/kohist.so abvar/base.so abvar/kohist.so; do
  n=$(basename $L .so)_$RANDOM
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$n -o run -- python3 tools/k1_ko_timing.py > gpurun_out/abl/$n.log 2>&1 || exit 1
  tail -1 gpurun_out/abl/$n.log
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/abl/$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fdk::' in r['Name']: print('$L', r['Name'].replace('void ','')[:45], r['Calls'], r['AverageNs'], r['MinNs'])
"
  rm -rf gpurun_out/abl/$n
done
