# Kernel-argument placement A/B at the headline (HIP_FORCE_DEV_KERNARG=0/1), rocprofv3 kernel stats of
# tools/profile_kernels.py --shape bench, alternating twice.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kargs
for r in 1 2; do
  for v in 0 1; do
    d=gpurun_out/kargs/k${v}_$r
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/profile_kernels.py --shape bench > $d.log 2>&1
    python3 -c '
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fdk::" in r["Name"]:
            print(sys.argv[2], r["Name"].replace("void ", "")[:40], r["Calls"], r["AverageNs"], r["MinNs"])
' $d "DEV_KERNARG=$v"
  done
done
