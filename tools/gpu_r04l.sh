# wave-local ranges in size order to free waves: tie tests, then A/B against the previous build (abvar/head.so)
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04l
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ties.py tests/test_gpu_select_custom.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l/ties.log 2>&1 || { tail -40 gpurun_out/r04l/ties.log; exit 1; }
tail -1 gpurun_out/r04l/ties.log
for i in 1 2; do
bash tools/gpu_ab_libs.sh ties abvar/head.so feature_detector_amd/lib/libfdhip.so >> gpurun_out/r04l/ab.txt 2>&1
bash tools/gpu_ab_libs.sh nsties abvar/head.so feature_detector_amd/lib/libfdhip.so >> gpurun_out/r04l/ab.txt 2>&1
done
grep k_select_ref gpurun_out/r04l/ab.txt
