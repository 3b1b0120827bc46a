# k_select_reference wave-local cutoff re-checked after the register sort and the merged swap pass:
# FD_REF_WL 128 / 256 (libfdhip) / 512 on the headline and north-star tie shapes, two rounds
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r04s
for i in 1 2; do
bash tools/gpu_ab_libs.sh ties abvar/wl128.so feature_detector_amd/lib/libfdhip.so abvar/wl512.so >> gpurun_out/r04s/ab.txt 2>&1
bash tools/gpu_ab_libs.sh nsties abvar/wl128.so feature_detector_amd/lib/libfdhip.so abvar/wl512.so >> gpurun_out/r04s/ab.txt 2>&1
done
grep k_select_ref gpurun_out/r04s/ab.txt
