set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
for v in 0 1 2 3; do
FD_XFLAGS=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/p$v -o run -- python3 tools/profile_kernels.py --shape fast720 > /dev/null 2>&1
python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/ab/p$v/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_fast' in r['Name'] or 'k_select<' in r['Name']: print('x=$v', r['Name'][:40], r['Calls'], r['AverageNs'])
"
done
