# Run the given GPU test files (default: the whole -m gpu suite) under a time limit.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${FD_TEST_TIMEOUT:-900} python3 -m pytest ${@:-tests} -m gpu -x -q > gpurun_out/tests.log 2>&1
