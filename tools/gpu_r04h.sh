# candidate-list store cache-policy A/B (FD_LIST_NT build in abvar/): FAST configs[2] shape, north-star detect, headline
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
bash tools/gpu_ab_libs.sh fast720 feature_detector_amd/lib/libfdhip.so abvar/listnt.so >> gpurun_out/ab_listnt.txt 2>&1
bash tools/gpu_ab_libs.sh nsdetect feature_detector_amd/lib/libfdhip.so abvar/listnt.so >> gpurun_out/ab_listnt.txt 2>&1
bash tools/gpu_ab_libs.sh bench feature_detector_amd/lib/libfdhip.so abvar/listnt.so >> gpurun_out/ab_listnt.txt 2>&1
done
cat gpurun_out/ab_listnt.txt
