# LSD map store cache-policy A/B (FD_LSD_STORE_AUX builds in abvar/), dense maps 1080p x256, two rounds
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
bash tools/gpu_ab_libs.sh "lsd --kind dense" feature_detector_amd/lib/libfdhip.so abvar/lsdaux2.so abvar/lsdaux3.so >> gpurun_out/ab_lsd.txt 2>&1
done
grep k_lsd_map gpurun_out/ab_lsd.txt
