# k_lsd_scatter columns per wave (FD_LSD_SC 16 / 32 / 64): rocprofv3 kernel stats, dense maps and compact lists
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lsc
for sc in 16 64 32 16; do
  for kind in dense compact; do
    d=gpurun_out/lsc/s${sc}_$kind
    rm -rf $d
    FD_DEBUG_AB=1 FD_LSD_SC=$sc timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/profile_kernels.py --shape lsd --kind $kind --calls 4 > $d.log 2>&1 || exit 1
    python3 -c '
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_lsd" in r["Name"]:
            print(sys.argv[2], r["Name"].replace("void ", "")[27:52], r["Calls"], r["AverageNs"], r["MinNs"])
' $d "sc=$sc $kind"
    rm -rf $d
  done
done
