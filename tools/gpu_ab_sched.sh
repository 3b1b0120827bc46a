# A/B of compiler scheduling strategies (-mllvm -amdgpu-sched-strategy=...) on the bench, north-star and FAST
# shapes: library builds abl/fd_<variant>.so made on the CPU side, two interleaved rounds in one call.
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do for shape in bench northstar fast720; do
  echo "## round $r shape $shape"
  bash tools/gpu_ab_libs.sh $shape abl/fd_base.so abl/fd_max-ilp.so abl/fd_iterative-ilp.so abl/fd_max-memory-clause.so
done; done
