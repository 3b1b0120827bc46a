# VALU issue mixes (valu_probe classes 70-75 beside their single-class references), FAST selection
# gather-spread A/B, then the round PMC pass. usage: bash tools/gpu_probe_mix.sh
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in 4 27 28 36 9 41 70 71 72 73 74 75; do timeout -k 5 60 tools/calib/valu_probe $c; done > gpurun_out/probe_mix.txt 2>&1
cat gpurun_out/probe_mix.txt | grep "waves/SIMD [48]"
bash tools/gpu_env_ab.sh fastg fast720 "FD_GATHER_GROUPS=1" "FD_GATHER_GROUPS=4" "FD_GATHER_GROUPS=8" "FD_GATHER_GROUPS=1"
FD_SELECT_STAMPS=1 timeout -k 10 120 python3 tools/select_stamps_fast.py > gpurun_out/stamps_fast.txt 2>&1
grep -E "cycles|frames" gpurun_out/stamps_fast.txt | tail -4
bash tools/gpu_round_pmc.sh r03
