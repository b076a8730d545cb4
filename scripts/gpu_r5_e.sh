# Round 5, call e: the GPU suite; certified trace A/B (the cheaper pre-bound key, the shading out of line
# in the fused binned kernel); C4 build stages against round 4 (margin codes only for the QNodes
# written, division-free); the per-rank certified trace times of the N-GPU split (scripts/rank_sim_cert.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit 1; fi
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; fi
AB_SET=certbase AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh raytracebvh_amd/librtbvh.so ablib/librtbvh_ckey.so ablib/librtbvh_noinl.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep ms_med gpurun_out/${T}_trace_ab.log | cut -c1-330
grep packet_steps gpurun_out/${T}_trace_ab.log | cut -c1-200
AB_SCRIPT=ab_build.py ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_r4.so raytracebvh_amd/librtbvh.so > gpurun_out/${T}_build_ab.log 2>&1 || { echo "BUILD AB FAILED"; tail -5 gpurun_out/${T}_build_ab.log; exit 1; }
cut -c1-330 gpurun_out/${T}_build_ab.log
timeout -k 10 600 python scripts/rank_sim_cert.py 20 > gpurun_out/${T}_rank_sim_cert.json 2> gpurun_out/${T}_rank_sim_cert.err || { echo "RANK SIM FAILED"; tail -5 gpurun_out/${T}_rank_sim_cert.err; exit 1; }
cat gpurun_out/${T}_rank_sim_cert.json
echo "call ok (tests rc=$rc)"
