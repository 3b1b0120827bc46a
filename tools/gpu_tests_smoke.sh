# GPU test suite (optionally a subset: pass pytest paths/-k args) then smoke(); stops at the first failure.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 700 python3 -u -m pytest ${@:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests.log 2>&1 || rc=$?
tail -40 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
cat gpurun_out/smoke.log
