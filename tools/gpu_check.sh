set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/k1_tests.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/k1_bench.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/k1_prof -o ns -- python3 tools/profile_kernels.py --shape northstar > gpurun_out/k1_prof.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/k1_prof -o fast -- python3 tools/profile_kernels.py --shape fast720 >> gpurun_out/k1_prof.log 2>&1
echo ok
