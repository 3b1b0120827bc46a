# Round profile pass, part 2: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the bench
# shapes' kernels and SQ counters of the north-star kernel. usage: bash tools/gpu_round_pmc.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
export TMPDIR=/tmp
O=gpurun_out/$TAG/pmc
mkdir -p $O
run() {  # name counters... -- cmd
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  timeout -s KILL 150 rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d $O/raw -o $name -- "$@" > $O/$name.log 2>&1
  for c in "${ctrs[@]}"; do python3 tools/pmc_summary.py $O/raw/${name}_counter_collection.csv $c | sed "s/^/$name,/" >> $O/summary.csv; done
}
for ctr in FETCH_SIZE WRITE_SIZE; do
  run calib_$ctr $ctr -- tools/calib/fetch_calib
  run bench_$ctr $ctr -- python3 tools/k1_batch1.py detect
  run northstar_$ctr $ctr -- python3 tools/profile_kernels.py --shape northstar --kind shi_tomasi --calls 3
  run fast720_$ctr $ctr -- python3 tools/profile_kernels.py --shape fast720 --calls 4
  run lsdd_$ctr $ctr -- python3 tools/profile_kernels.py --shape lsd --kind dense --calls 2
  run lsdc_$ctr $ctr -- python3 tools/profile_kernels.py --shape lsd --kind compact --calls 2
done
run ns_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -- python3 tools/profile_kernels.py --shape northstar --kind shi_tomasi --calls 3
run fast_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -- python3 tools/profile_kernels.py --shape fast720 --calls 4
rm -rf $O/raw
python3 tools/make_round_profiles.py $O/summary.csv $TAG > $O/sq_summary.json
echo ok
