# Round 5, call i: the certified walk's pre-bound margin per node (rho_n at the node grid's exit distance,
# folded into the near planes) and without the dead exact-decode branch, against the product library;
# then the certified GPU tests with the new library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_i}
AB_SET=certbase AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_nx.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -E "ms_med|frame_sha1" gpurun_out/${T}_trace_ab.log | cut -c1-330
grep packet_steps gpurun_out/${T}_trace_ab.log | cut -c1-260
RTBVH_LIB=$(realpath ablib/librtbvh_nx.so) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "certif or auto or contain or margin" --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
echo "call ok (tests rc=$rc)"
