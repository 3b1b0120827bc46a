# A/B of environment settings (e.g. FD_PX=4) on profile_kernels.py shapes, each under rocprofv3
# --kernel-trace --stats, all in one GPU call; optional GPU test files first.
# usage: bash tools/gpu_env_ab.sh [-t "test files"] <tag> "<shape> [profile_kernels args]" "ENV=V ..." ["ENV=V ..." ...]
# A failing test run (exit 1) does not stop the timings; a crash, abort or time-out stops everything.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TESTS=""
if [ "$1" = "-t" ]; then TESTS=$2; shift 2; fi
TAG=$1; SHAPE=$2; shift 2
O=gpurun_out/envab/$TAG; mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread $TESTS > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; ok $rc || { echo "tests rc=$rc: stop"; exit $rc; }
fi
i=0
for ENVS in "$@"; do
  i=$((i+1)); n=v$i
  env $ENVS timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 tools/profile_kernels.py --shape $SHAPE > $O/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$ENVS: rc=$rc: stop"; tail -5 $O/$n.log; exit $rc; }
  python3 -c "
import csv,glob
for f in glob.glob('$O/$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fdk::' in r['Name']: print('[$ENVS]', r['Name'].replace('void ','')[:52], r['Calls'], r['AverageNs'], r['MinNs'])
"
done
