# Kernel-duration profiles of the bench shapes (rocprofv3 kernel trace), summarised to CSV.
# usage: bash tools/gpu_prof.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-prof}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for spec in "northstar shi_tomasi" "northstar harris" "bench harris" "fast720 fast"; do
  set -- $spec
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/raw -o $1_$2 -- python3 tools/profile_kernels.py --shape $1 --kind $2 > gpurun_out/$TAG/$1_$2.log 2>&1
  python3 tools/rocpd_summary.py gpurun_out/$TAG/raw/$1_$2_results.db > gpurun_out/$TAG/$1_$2.csv
done
rm -rf gpurun_out/$TAG/raw
echo ok
