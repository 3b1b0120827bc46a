# SQ counter pass (one rocprofv3 --pmc run of 8 SQ + 1 GRBM counter) per environment setting on one
# profile_kernels.py shape; prints per-kernel counter averages.
# usage: bash tools/gpu_sq_ab.sh <tag> "<shape> [args]" "ENV=V ..." ["ENV=V ..." ...]
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
TAG=$1; SHAPE=$2; shift 2
O=gpurun_out/sqab/$TAG; mkdir -p $O
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for ENVS in "$@"; do
  i=$((i+1)); n=v$i
  env $ENVS timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/$n -o run -- python3 tools/profile_kernels.py --shape $SHAPE --calls 2 > $O/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$ENVS: rc=$rc: stop"; tail -5 $O/$n.log; exit $rc; }
  python3 - "$O/$n" "$ENVS" <<'EOF'
import csv, glob, sys, collections
d, envs = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'fdk::' not in k: continue
        k = k.replace('void ', '')[:48]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
for k, c in acc.items():
    n = len(disp[k])
    print(f"[{envs}] {k} dispatches={n} " + " ".join(f"{name}={v / n:.4g}" for name, v in sorted(c.items())))
EOF
done
