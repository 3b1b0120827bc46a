# GPU tests on the current build, then the scheduling-strategy A/B on the LSD shape (whole-library builds
# abl/fd_<variant>.so; only the k_lsd_* rows matter) and the per-pixel shapes against the new default.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
tail -1 gpurun_out/tests.log
for r in 1 2; do
  echo "## round $r shape lsd"
  bash tools/gpu_ab_libs.sh lsd abl/fd_new.so abl/fd_iterative-ilp.so abl/fd_max-ilp.so
  for shape in bench northstar fast720; do
    echo "## round $r shape $shape"
    bash tools/gpu_ab_libs.sh $shape abl/fd_base.so abl/fd_new.so
  done
done
