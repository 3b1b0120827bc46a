# Round 4 final measurement, part 1: the GPU test suite + smoke, a plain bench line, the rocprofv3 kernel
# summary of the bench by leg. usage: bash tools/gpu_r04z.sh   (part 2: bash tools/gpu_round_pmc.sh r04)
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
bash tools/gpu_tests_smoke.sh > $O/tests_smoke.txt 2>&1 || { tail -30 $O/tests_smoke.txt; exit 1; }
tail -3 $O/tests_smoke.txt
timeout -k 10 900 python3 bench.py > $O/bench_plain.json 2> $O/bench_plain.err
tail -c 400 $O/bench_plain.json
bash tools/gpu_round_bench.sh r04
echo done
