# Round 5, call c: the GPU suite (QNodes the walk never reads no longer written, slack-free rays certified
# on the exact decode, the fused binned shading, the linear node margin); the certified trace A/B against
# round 4 and the two options off; the C4 build stages against round 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit 1; fi
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; fi
AB_SET=certified AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_r4.so raytracebvh_amd/librtbvh.so ablib/librtbvh_noexact.so ablib/librtbvh_nofuse.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -v packet_steps gpurun_out/${T}_trace_ab.log | cut -c1-330
grep packet_steps gpurun_out/${T}_trace_ab.log | python3 -c "
import sys, json
for l in sys.stdin:
    lib, _, js = l.partition(' {') if l.startswith('lib') else ('', '', l)
    d = json.loads('{' + js if lib else l)
    print(lib[:22], d['variant'], 'redo', d['redo_rays'], 'int', d['internal_visits'][1], 'max', d['trav_max_steps'])
"
AB_SCRIPT=ab_build.py ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_r4.so raytracebvh_amd/librtbvh.so > gpurun_out/${T}_build_ab.log 2>&1 || { echo "BUILD AB FAILED"; tail -5 gpurun_out/${T}_build_ab.log; exit 1; }
cat gpurun_out/${T}_build_ab.log | cut -c1-400
echo "call ok (tests rc=$rc)"
