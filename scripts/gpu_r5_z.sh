# Round 5, call z: the 8-wide certified bounce walk (RTBVH_WIDE8 build, ablib/librtbvh_w8.so): the certified
# tests on it, then the C5 A/B against the 4-wide build (bounce walk times, frame hashes, visit counts)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_z}
RTBVH_LIB=$PWD/ablib/librtbvh_w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cert or auto_walk or containment or c5_frame or qnodes" > gpurun_out/${T}_w8_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_w8_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_w8_tests.log | head -20; exit 1; fi
AB_SET=certbase ROUNDS=2 AB_ROUNDS=3 timeout -k 10 600 bash scripts/ab_libs.sh ablib/librtbvh_w4.so ablib/librtbvh_w8.so > gpurun_out/${T}_w8_ab.log 2>&1 || { tail -5 gpurun_out/${T}_w8_ab.log; exit 1; }
cut -c1-300 gpurun_out/${T}_w8_ab.log
AB_COUNTS=1 AB_SET=certbase ROUNDS=1 AB_ROUNDS=1 timeout -k 10 600 bash scripts/ab_libs.sh ablib/librtbvh_w4.so ablib/librtbvh_w8.so > gpurun_out/${T}_w8_counts.log 2>&1 || { tail -5 gpurun_out/${T}_w8_counts.log; exit 1; }
cut -c1-600 gpurun_out/${T}_w8_counts.log
echo "call ok"
