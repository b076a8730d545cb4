# Round 5, call k: the GPU suite (certified walks end at nodes without a grid), and the certified trace A/B
# against the previous commit's walk.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_k}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; fi


AB_SET=certbase AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_head.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -E "ms_med" gpurun_out/${T}_trace_ab.log | cut -c1-330
echo "call ok"
