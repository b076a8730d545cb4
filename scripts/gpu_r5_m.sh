# Round 5, call l: 8-B LDS stack entries, one LDS op per push and pop (RTBVH_STACK8, 10 rows) -- the certified trace A/B
# against the product library, then the GPU suite on the A/B library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_m}
AB_SET=certbase AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_s8.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -E "ms_med|frame_sha1" gpurun_out/${T}_trace_ab.log | cut -c1-330
grep packet_steps gpurun_out/${T}_trace_ab.log | cut -c1-200
RTBVH_LIB=$(realpath ablib/librtbvh_s8.so) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
echo "call ok (tests rc=$rc)"
