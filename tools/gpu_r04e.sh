# Round 4: wave-count sweep of K1 now that it can hold 5 (response) / 4 (detect) waves per SIMD
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_env_ab.sh ns "northstar --kind shi_tomasi" "FD_TARGET_WAVES=10240" "FD_TARGET_WAVES=5120" "FD_TARGET_WAVES=15360" "FD_TARGET_WAVES=20480" "FD_TARGET_WAVES=40960" "FD_TARGET_WAVES=10240" > gpurun_out/r04e_ns.txt 2>&1
cat gpurun_out/r04e_ns.txt
bash tools/gpu_env_ab.sh nsd "nsdetect --kind shi_tomasi" "FD_TARGET_WAVES=10240" "FD_TARGET_WAVES=8192" "FD_TARGET_WAVES=20480" "FD_TARGET_WAVES=10240" > gpurun_out/r04e_nsd.txt 2>&1
cat gpurun_out/r04e_nsd.txt
