# One GPU call of an optimisation step: the GPU tests + smoke() on the working tree's library, then an
# A/B of two library builds (abvar/base.so = HEAD, abvar/new.so = the change) on profile_kernels.py
# shapes, alternating, each under rocprofv3 --kernel-trace --stats; then a plain bench line.
# usage: bash tools/gpu_ab_session.sh "<shape args>" ["<shape args>" ...]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests_smoke.sh
for S in "$@"; do
  bash tools/gpu_ab_libs.sh "$S" abvar/base.so abvar/new.so abvar/base.so abvar/new.so
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_plain.json 2> gpurun_out/bench_plain.err
cat gpurun_out/bench_plain.json | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('value', d['value'], 'ms_per_step', d['ms_per_step'])"
