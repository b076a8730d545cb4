# Round 5, call a: the GPU suite on the per-node margin code (+ the LDS top table), then the certified
# walk A/B on C5 against round 4's library: top-table sizes 0 (per-node margins only), 96, 192 (default),
# 256, 341 QNodes, with the walk census (trav_max_steps, visits).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit 1; fi
AB_SET=certified AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_r4.so ablib/librtbvh_top0.so raytracebvh_amd/librtbvh.so ablib/librtbvh_top96.so ablib/librtbvh_top256.so ablib/librtbvh_top341.so > gpurun_out/${T}_cert_ab.log 2>&1 || { echo "AB FAILED"; tail -5 gpurun_out/${T}_cert_ab.log; exit 1; }
cut -c1-700 gpurun_out/${T}_cert_ab.log
echo "call ok (tests rc=$rc)"
