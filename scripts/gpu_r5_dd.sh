# Round 5, call dd: parked long certified walks (k_bounce_tail): the certified GPU tests on the default build
# (park after 128 steps), then one-frame trace stages (ab_libs) and per-rank frames at N = 1 / 8 (one frame,
# four in flight) for park 0 (off) / 64 / 128 / 256 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_dd}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cert or auto_walk or containment or c5_frame or band or flight" > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_tests.log | head -20; exit 1; fi
AB_SET=certbase ROUNDS=2 AB_ROUNDS=3 timeout -k 10 600 bash scripts/ab_libs.sh ablib/librtbvh_park0.so ablib/librtbvh_park64.so ablib/librtbvh_park128.so ablib/librtbvh_park256.so > gpurun_out/${T}_ab.log 2>&1 || { tail -5 gpurun_out/${T}_ab.log; exit 1; }
grep -o 'librtbvh_park[0-9]*.so\|"bounce_trav_ms_med": [0-9.]*\|"trace_ms_med": [0-9.]*\|frame_sha1": "[0-9a-f]*"' gpurun_out/${T}_ab.log | paste -sd' ' | sed 's/librtbvh/\nlibrtbvh/g'
echo
for L in park0 park128 park64 park256; do
  for NR in "1 0" "8 1"; do
    set -- $NR
    RTBVH_LIB=$PWD/ablib/librtbvh_$L.so timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 20 > gpurun_out/${T}_${L}_n$1_one.json 2>> gpurun_out/${T}_rank.err || { tail -5 gpurun_out/${T}_rank.err; exit 1; }
    RTBVH_LIB=$PWD/ablib/librtbvh_$L.so timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 40 inflight 4 > gpurun_out/${T}_${L}_n$1_inflight.json 2>> gpurun_out/${T}_rank.err || { tail -5 gpurun_out/${T}_rank.err; exit 1; }
    echo "$L N$1 one $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_${L}_n$1_one.json) inflight $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_${L}_n$1_inflight.json)"
  done
done
echo "call ok"
