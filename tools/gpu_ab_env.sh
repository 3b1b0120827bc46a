# A/B of an environment variable on one profile_kernels.py shape. usage: bash tools/gpu_ab_env.sh <shape> <kind|-> VAR v1 v2 ...
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/abe
SHAPE=$1; KIND=$2; VAR=$3; shift 3
KA=""; [ "$KIND" != "-" ] && KA="--kind $KIND"
for v in "$@"; do
  env $VAR=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abe/$VAR$v -o run -- python3 tools/profile_kernels.py --shape $SHAPE $KA > /dev/null 2>&1
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/abe/$VAR$v/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fdk::' in r['Name']: print('$VAR=$v', r['Name'].replace('void ','')[:45], r['Calls'], r['AverageNs'])
"
done
