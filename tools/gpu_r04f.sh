# k_select_reference wave-local cutoff A/B (FD_REF_WL builds in abvar/), headline tie frames then north star
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_libs.sh ties abvar/wl0.so abvar/wl256.so abvar/wl256u4ni.so abvar/wl256u8ni.so abvar/wl0u8ni.so > gpurun_out/ab_ties.txt 2>&1
grep k_select_ref gpurun_out/ab_ties.txt
bash tools/gpu_ab_libs.sh nsties abvar/wl0.so abvar/wl256.so abvar/wl256u4ni.so abvar/wl256u8ni.so abvar/wl0u8ni.so > gpurun_out/ab_nsties.txt 2>&1
grep k_select_ref gpurun_out/ab_nsties.txt
