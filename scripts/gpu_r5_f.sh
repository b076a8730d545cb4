# Round 5, call f: the next QNode fetched while the step's leaf test is in flight (RTBVH_PF), at 6, 7 and 8
# waves per SIMD, against the product library, on the certified bench mode (frames compared bit for bit).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_f}
AB_SET=certbase AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_pf6.so ablib/librtbvh_pf7.so ablib/librtbvh_pf8.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -E "ms_med|frame_sha1" gpurun_out/${T}_trace_ab.log | cut -c1-330
grep packet_steps gpurun_out/${T}_trace_ab.log | cut -c1-200
echo "call ok"
