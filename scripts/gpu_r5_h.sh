# Round 5, call h: 128-B triangle records (the shading's vertex attributes in the record's second half,
# written once per scene): the GPU suite, then certified trace and C4 build A/B against the 64-B layout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_h}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; fi
AB_SET=certbase AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_tcs4.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -E "ms_med|frame_sha1" gpurun_out/${T}_trace_ab.log | cut -c1-330
AB_SCRIPT=ab_build.py ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_tcs4.so raytracebvh_amd/librtbvh.so > gpurun_out/${T}_build_ab.log 2>&1 || { echo "BUILD AB FAILED"; tail -5 gpurun_out/${T}_build_ab.log; exit 1; }
cut -c1-330 gpurun_out/${T}_build_ab.log
echo "call ok"
