# k_select phase costs by knockout builds (abl/ko<n>: FD_KO=n stops the selection early; timing only).
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_libs.sh bench abl/old/libfdhip.so feature_detector_amd/lib/libfdhip.so abl/ko2/libfdhip.so abl/ko9/libfdhip.so abl/ko8/libfdhip.so abl/ko7/libfdhip.so abl/ko6/libfdhip.so abl/ko3/libfdhip.so 2>&1 | grep k_select
