# One GPU call made of named steps, run in order; the first failing step ends the call.
# usage: bash tools/gpu_session.sh STEP [STEP ...]
#   tests              the GPU test suite, then smoke()
#   tests=PATHS        a subset (comma-separated pytest paths / node ids), no smoke()
#   ab=SHAPE           A/B of abvar/base.so vs abvar/new.so (FD_LIB_PATH) on a tools/profile_kernels.py
#                      shape (comma-separated args), alternating twice, each under rocprofv3 --kernel-trace --stats
#   abx=SHAPE:L1:L2..  the same over libraries L1, L2, ... (paths under the repo), each once, in order
#   env=SHAPE:E1:E2..  A/B of environment settings (each Ek: comma-separated VAR=V) on a shape, under
#                      rocprofv3 --kernel-trace --stats; FD_DEBUG_AB=1 is set so the library honours its switches
#   bench=ARGS         one bench.py line (ARGS: comma-separated bench.py flags) -> gpurun_out/bench_<n>.json
#   stamps[=LIB,E..]   k_select phase clocks (FD_SELECT_STAMPS) at the bench shapes (LIB: FD_LIB_PATH, e.g.
#                      abvar/new.so, may be empty; E: VAR=V settings, e.g. FD_SELECT_REPEAT=1)
#   py=SCRIPT          python3 SCRIPT (comma-separated args), output to gpurun_out/py_<n>.log
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
n=0

# per-kernel rows of a rocprofv3 --stats csv directory: label, name, calls, average ns, min ns
kstats() {
  python3 -c '
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fdk::" in r["Name"]:
            print(sys.argv[2], r["Name"].replace("void ", "")[:48], r["Calls"], r["AverageNs"], r["MinNs"])
' "$1" "$2"
}

# one rocprofv3 kernel-trace run of profile_kernels.py: prof DIR SHAPE [ENV ...]
prof() {
  local d=$1 shape=$2
  shift 2
  env "$@" timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
      -- python3 tools/profile_kernels.py --shape $shape > $d.log 2>&1
}

for S in "$@"; do
  n=$((n + 1))
  key=${S%%=*}
  val=${S#*=}
  [ "$key" = "$S" ] && val=""
  echo "[session] step $n: $S"
  case $key in
    tests)
      paths=${val//,/ }
      timeout -k 10 700 python3 -u -m pytest ${paths:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
          > gpurun_out/tests_$n.log 2>&1 || { tail -60 gpurun_out/tests_$n.log; exit 1; }
      tail -3 gpurun_out/tests_$n.log
      if [ -z "$val" ]; then
        timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
        cat gpurun_out/smoke.log
      fi ;;
    ab)
      for L in abvar/base.so abvar/new.so abvar/base.so abvar/new.so; do
        d=gpurun_out/abl/$(basename $L .so)_${n}_$RANDOM
        prof $d "${val//,/ }" FD_LIB_PATH=$GRAFT_REPO_ROOT/$L
        kstats $d $L
        rm -rf $d
      done ;;
    abx)
      IFS=':' read -ra parts <<< "$val"
      for L in "${parts[@]:1}"; do
        d=gpurun_out/abl/$(basename $L .so)_${n}_$RANDOM
        prof $d "${parts[0]//,/ }" FD_LIB_PATH=$GRAFT_REPO_ROOT/$L
        kstats $d $L
        rm -rf $d
      done ;;
    env)
      IFS=':' read -ra parts <<< "$val"
      for E in "${parts[@]:1}"; do
        d=gpurun_out/abl/env_${n}_$RANDOM
        prof $d "${parts[0]//,/ }" FD_DEBUG_AB=1 ${E//,/ }
        kstats $d "[$E]"
        rm -rf $d
      done ;;
    bench)
      timeout -k 10 400 python3 bench.py ${val//,/ } > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('value', d['value'], 'ms_per_step', d['ms_per_step'])" gpurun_out/bench_$n.json ;;
    stamps)
      IFS=',' read -ra sp <<< "$val"
      lib=${sp[0]:-}
      env ${sp[@]:1} FD_LIB_PATH=${lib:+$GRAFT_REPO_ROOT/$lib} FD_DEBUG_AB=1 FD_SELECT_STAMPS=1 timeout -k 10 120 \
          python3 tools/select_stamps.py > gpurun_out/stamps_$n.txt 2>&1
      grep -v "^  levels\|k_select_reference" gpurun_out/stamps_$n.txt | head -12 ;;
    py)
      timeout -k 10 300 python3 ${val//,/ } > gpurun_out/py_$n.log 2>&1 || { tail -30 gpurun_out/py_$n.log; exit 1; }
      tail -20 gpurun_out/py_$n.log ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "[session] done"
