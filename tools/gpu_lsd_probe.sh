set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lsd.py tests/test_cpp_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lsd_tests.log 2>&1
timeout -k 10 200 python3 tools/lsd_probe.py FD_LSD_WAVES=16384 FD_LSD_WAVES=8192 FD_LSD_WAVES=32768 FD_LSD_WAVES=65536 FD_LSD_WAVES=16384
FD_LIB_PATH=$PWD/feature_detector_amd/lib/old/libfdhip.so timeout -k 10 200 python3 tools/lsd_probe.py A=0
