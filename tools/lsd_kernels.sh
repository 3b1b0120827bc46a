# LSD dense map kernel stats (rocprofv3, profile_kernels --shape lsd --kind dense), three passes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lrows
for L in 1 2 3; do
  d=gpurun_out/lrows/p$L
  rm -rf $d
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/profile_kernels.py --shape lsd --kind dense --calls 6 > $d.log 2>&1 || exit 1
  python3 -c '
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_lsd" in r["Name"]:
            print(sys.argv[2], r["Name"].replace("void ", "")[27:52], r["Calls"], r["AverageNs"], r["MinNs"])
' $d "pass $L"
  rm -rf $d
done
