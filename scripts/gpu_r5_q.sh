# Round 5, call q: k_primary_binned's launch bounds (the fused shading spills 37 VGPRs at 8 waves per SIMD):
# 8 / 6 / 5 waves, certified one-frame traces, libraries interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_q}
AB_SET=certbase AB_ROUNDS=3 ROUNDS=3 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_pbw6.so ablib/librtbvh_pbw5.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -E "ms_med" gpurun_out/${T}_trace_ab.log | cut -c1-200
echo "call ok"
