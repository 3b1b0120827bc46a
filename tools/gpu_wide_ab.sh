set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
FD_SELECT_STAMPS=1 timeout -k 10 100 python3 tools/select_stamps_fast.py 2>&1 | grep "k_select cycles" | tail -1
for sh in fast720 northstar; do
for w in 0 1; do
  if [ $w = 1 ]; then export FD_NO_WIDE=1; else unset FD_NO_WIDE; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w/$sh$w -o run -- python3 tools/profile_kernels.py --shape $sh > /dev/null 2>&1
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/w/$sh$w/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_select' in r['Name'] or 'k_gather' in r['Name']: print('$sh nowide=$w', r['Name'][:40], r['Calls'], r['AverageNs'])
"
done; done
