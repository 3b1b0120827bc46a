set -e
cd $GRAFT_REPO_ROOT
for sh in northstar fast720 bench; do
bash tools/gpu_ab_libs.sh $sh feature_detector_amd/lib/libfdhip_c512_f1024.so feature_detector_amd/lib/libfdhip.so feature_detector_amd/lib/libfdhip_c508_f744.so feature_detector_amd/lib/libfdhip_c508_f320.so
done
