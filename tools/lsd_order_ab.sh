# k_lsd_map wave order (FD_LSD_ORDER 1 = chunk fastest) x chunk height (FD_LSD_CH; default 67 at 1080p x256):
# rocprofv3 kernel stats of profile_kernels --shape lsd --kind dense
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lord
for cfg in "0 0" "1 0" "0 64" "1 64" "0 32" "1 32" "1 16" "0 0"; do
  set -- $cfg
  d=gpurun_out/lord/o$1_c$2
  rm -rf $d
  if [ "$2" = 0 ]; then ch=""; else ch="FD_LSD_CH=$2"; fi
  env FD_DEBUG_AB=1 FD_LSD_ORDER=$1 $ch timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/profile_kernels.py --shape lsd --kind dense --calls 6 > $d.log 2>&1 || exit 1
  python3 -c '
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_lsd" in r["Name"]:
            print(sys.argv[2], r["Name"].replace("void ", "")[27:52], r["Calls"], r["AverageNs"], r["MinNs"])
' $d "order=$1 ch=$2"
  rm -rf $d
done
