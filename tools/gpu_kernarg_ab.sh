# Kernel-argument placement A/B (HIP_FORCE_DEV_KERNARG=0/1): per-workgroup K1 clocks on the
# instrumented build (abvar/clk.so: `make -C feature_detector_amd/csrc OUT=/tmp/clk XFLAGS=-DFD_K1_CLOCKS`,
# copied there) and the headline bench step, alternating, one GPU call.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
HB="--no-north-star --no-config3 --no-lsd --no-superpoint --no-cpu-baseline"
for v in 0 1 0 1; do
  echo "== HIP_FORCE_DEV_KERNARG=$v"
  HIP_FORCE_DEV_KERNARG=$v FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/clk.so timeout -k 10 120 python3 tools/k1_wg_clock.py 2>/dev/null
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python3 bench.py $HB 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('bench value', d['value'], 'ms_per_step', d['ms_per_step'])"
done
