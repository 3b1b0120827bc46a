# Headline K1 (640x480 batch 1): product, no candidates (thr 1e30), load-free build, both.
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/k1b; mkdir -p $O
one() {
  local n=$1 lib=$2; shift 2
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 tools/profile_kernels.py --shape bench "$@" > $O/$n.log 2>&1
  python3 -c "
import csv,glob
for f in glob.glob('$O/$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_corner' in r['Name'] or 'k_select' in r['Name']: print('$n', r['Name'][30:60], r['Calls'], r['AverageNs'])
"
}
one product feature_detector_amd/lib/libfdhip.so
one noemit feature_detector_amd/lib/libfdhip.so --thr 1e30
one noload abl/noload/libfdhip.so
one noload_noemit abl/noload/libfdhip.so --thr 1e30
