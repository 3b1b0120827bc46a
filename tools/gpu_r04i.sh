# wide prelude of k_select_reference: tie tests (auto / forced wide / forced single-workgroup), then the
# bench tie frames' kernel times with the prelude off and on (FD_REF_WIDE)
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04i
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ties.py tests/test_gpu_select_custom.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i/ties.log 2>&1 || { tail -40 gpurun_out/r04i/ties.log; exit 1; }
tail -1 gpurun_out/r04i/ties.log
bash tools/gpu_env_ab.sh refwide "nsties" "FD_REF_WIDE=0" "FD_REF_WIDE=1" "FD_REF_WIDE=0" "FD_REF_WIDE=1" > gpurun_out/r04i/ab.txt 2>&1 || true
grep -E "k_select_ref|k_refw" gpurun_out/r04i/ab.txt | head -60
