# Host-frame call A/B (tools/e2e_probe.py) of abvar/base.so vs abvar/new.so, after the point / selection tests
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_points.py tests/test_gpu_select.py tests/test_gpu_select_custom.py tests/test_gpu_fast_cut.py tests/test_gpu_context.py tests/test_cpp_api.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e2e/tests.log 2>&1 || { tail -40 gpurun_out/e2e/tests.log; exit 1; }
tail -2 gpurun_out/e2e/tests.log
for L in base new base new; do
  echo "== $L"
  FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 100 python3 tools/e2e_probe.py 2>&1 | grep -v amdgpu.ids
done
