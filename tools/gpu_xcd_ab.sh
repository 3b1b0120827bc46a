# XCD-aware tile mapping A/B: GPU point tests, kernel times (bench, northstar, fast720) and FETCH_SIZE at the
# headline shape for abl/old vs the current build.
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/xcd; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_points.py tests/test_gpu_select.py tests/test_gpu_ties.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for sh in bench northstar fast720; do bash tools/gpu_ab_libs.sh $sh abl/old/libfdhip.so feature_detector_amd/lib/libfdhip.so | grep -v "k_select\|k_gather\|k_mask"; done
for L in abl/old/libfdhip.so feature_detector_amd/lib/libfdhip.so; do
  FD_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o f -- python3 tools/k1_batch1.py detect > /dev/null 2>&1
  python3 tools/pmc_summary.py $O/pmc/f_counter_collection.csv FETCH_SIZE | grep k_corner | sed "s|^|$L |"
  rm -rf $O/pmc
done
