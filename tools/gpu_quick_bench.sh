# GPU tests for the given files, then the bench with only the requested legs (args after --).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS=""
while [ $# -gt 0 ] && [ "$1" != "--" ]; do TESTS="$TESTS $1"; shift; done
[ "$1" = "--" ] && shift
if [ -n "$TESTS" ]; then timeout -k 10 600 python3 -m pytest $TESTS -m gpu -x -q > gpurun_out/tests.log 2>&1; fi
timeout -k 10 400 python3 bench.py "$@" > gpurun_out/bench_quick.json 2>gpurun_out/bench_quick.err
