set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_points.py tests/test_gpu_select.py > gpurun_out/ab1_tests.log 2>&1 || { tail -30 gpurun_out/ab1_tests.log; exit 1; }
tail -2 gpurun_out/ab1_tests.log
bash tools/gpu_ab_libs.sh "northstar --kind shi_tomasi" abvar/base.so abvar/new.so abvar/slots12.so abvar/slots10.so abvar/base.so abvar/new.so
bash tools/gpu_ab_libs.sh "nsdetect --kind shi_tomasi" abvar/base.so abvar/new.so
bash tools/gpu_env_ab.sh hl bench "FD_PX=0" "FD_PX=2" "FD_PX=4" "FD_PX=2 FD_TILE_H=6" "FD_PX=2 FD_TILE_H=2" "FD_PX=0"
