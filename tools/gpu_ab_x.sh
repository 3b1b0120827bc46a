# A/B of FD_XFLAGS experiment variants on one profile_kernels.py shape. usage: bash tools/gpu_ab_x.sh <shape> <kind> v1 v2 ...
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/abx
SHAPE=$1; KIND=$2; shift 2
for v in "$@"; do
FD_XFLAGS=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abx/p$v -o run -- python3 tools/profile_kernels.py --shape $SHAPE --kind $KIND > /dev/null 2>&1
python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/abx/p$v/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if r['Name'].startswith('void fdk'): print('x=$v', r['Name'][:45], r['Calls'], r['AverageNs'])
"
done
