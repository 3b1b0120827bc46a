# LSD map: waves per launch (FD_LSD_WAVES) x store policy (abvar/base.so nontemporal, abvar/aux0.so default),
# rocprofv3 kernel stats of profile_kernels --shape lsd --kind dense
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lw
for L in base aux0; do
  for wv in 32768 65536 131072; do
    d=gpurun_out/lw/${L}_$wv
    FD_DEBUG_AB=1 FD_LSD_WAVES=$wv FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/profile_kernels.py --shape lsd --kind dense --calls 4 > $d.log 2>&1
    python3 -c '
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_lsd" in r["Name"]:
            print(sys.argv[2], r["Name"].replace("void ", "")[27:48], r["Calls"], r["AverageNs"], r["MinNs"])
' $d "$L waves=$wv"
    rm -rf $d
  done
done
