# Round 4 session A: GPU tests + smoke on the in-tree library, then A/B of library builds under rocprofv3
# (north-star response kernel, north-star detect) and the LSD dense map with padded vs unpadded rows.
set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
rc=0; bash tools/gpu_tests_smoke.sh || rc=$?
echo "tests rc=$rc"
# plain test failures (pytest rc 1) still let the timing run; a crash, abort or timeout ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if grep -q "Timeout" gpurun_out/tests.log; then echo "a test timed out: stopping"; exit 3; fi
bash tools/gpu_ab_libs.sh "northstar --kind shi_tomasi" abvar/base.so abvar/occ.so abvar/pkq.so feature_detector_amd/lib/libfdhip.so abvar/base.so abvar/occ.so abvar/pkq.so feature_detector_amd/lib/libfdhip.so > gpurun_out/ab_ns.txt 2>&1
cat gpurun_out/ab_ns.txt
bash tools/gpu_ab_libs.sh "nsdetect --kind shi_tomasi" abvar/base.so abvar/occ.so abvar/pkq.so feature_detector_amd/lib/libfdhip.so > gpurun_out/ab_nsd.txt 2>&1
cat gpurun_out/ab_nsd.txt
bash tools/gpu_ab_libs.sh "bench --kind harris" abvar/occ.so feature_detector_amd/lib/libfdhip.so abvar/occ.so feature_detector_amd/lib/libfdhip.so > gpurun_out/ab_hl.txt 2>&1
cat gpurun_out/ab_hl.txt
bash tools/gpu_ab_libs.sh "fast720" abvar/occ.so feature_detector_amd/lib/libfdhip.so abvar/occ.so feature_detector_amd/lib/libfdhip.so > gpurun_out/ab_fast.txt 2>&1
cat gpurun_out/ab_fast.txt
bash tools/gpu_ab_libs.sh "lsd --kind dense_unpitched" feature_detector_amd/lib/libfdhip.so > gpurun_out/ab_lsd.txt 2>&1
bash tools/gpu_ab_libs.sh "lsd --kind dense" feature_detector_amd/lib/libfdhip.so >> gpurun_out/ab_lsd.txt 2>&1
bash tools/gpu_ab_libs.sh "lsd --kind dense_unpitched" feature_detector_amd/lib/libfdhip.so >> gpurun_out/ab_lsd.txt 2>&1
bash tools/gpu_ab_libs.sh "lsd --kind dense" feature_detector_amd/lib/libfdhip.so >> gpurun_out/ab_lsd.txt 2>&1
cat gpurun_out/ab_lsd.txt
