# North-star K1: what bounds it. Kernel time of the product build, of the same build with no candidates
# (threshold 1e30: emission code never runs), and of the load-free diagnostic build (FD_NOLOAD: the
# frame reads replaced by an ALU hash, same instruction stream otherwise).
# usage: bash tools/gpu_k1_decisive.sh   (needs abl/noload/libfdhip.so: make OUT=../../abl/noload XFLAGS=-DFD_NOLOAD)
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/k1d; mkdir -p $O
one() {  # name lib args...
  local n=$1 lib=$2; shift 2
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 tools/profile_kernels.py --shape northstar "$@" > $O/$n.log 2>&1
  python3 -c "
import csv,glob
for f in glob.glob('$O/$n/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if r['Name'].startswith('void fdk'): print('$n', r['Name'][:60], r['Calls'], r['AverageNs'])
"
}
one product feature_detector_amd/lib/libfdhip.so
one noemit feature_detector_amd/lib/libfdhip.so --thr 1e30
one noload abl/noload/libfdhip.so
one noload_noemit abl/noload/libfdhip.so --thr 1e30
