# LSD valid-list scatter: the working build (libfdhip) vs abvar/head.so: LSD and line
# tests, then the dense and compact 1080p x256 kernels of both builds, twice
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04r
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lsd.py tests/test_gpu_lines.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r/lsd.log 2>&1 || { tail -30 gpurun_out/r04r/lsd.log; exit 1; }
tail -1 gpurun_out/r04r/lsd.log
for i in 1 2; do
bash tools/gpu_ab_libs.sh "lsd --kind dense" abvar/head.so feature_detector_amd/lib/libfdhip.so >> gpurun_out/r04r/ab.txt 2>&1
bash tools/gpu_ab_libs.sh "lsd --kind compact" abvar/head.so feature_detector_amd/lib/libfdhip.so >> gpurun_out/r04r/ab.txt 2>&1
done
grep -E "scatter|scan|values" gpurun_out/r04r/ab.txt
