# Round 5, call jj: k_primary_binned with 512 threads per tile (8 waves share a tile's bins) against 256:
# binned tests on it, per-rank frames at N = 8 / 1 (four in flight, one frame), and the C5 stage times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_jj}
RTBVH_LIB=$PWD/ablib/librtbvh_rb512.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "binned or band or cert or c5_frame" > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_tests.log | head -20; exit 1; fi
for rnd in 1 2; do
for L in rb256 rb512; do
  for NR in "8 1" "1 0"; do
    set -- $NR
    RTBVH_LIB=$PWD/ablib/librtbvh_$L.so timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 40 inflight 4 > gpurun_out/${T}_${L}_n$1_inflight_$rnd.json 2>> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
    RTBVH_LIB=$PWD/ablib/librtbvh_$L.so timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 20 > gpurun_out/${T}_${L}_n$1_one_$rnd.json 2>> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
    echo "r$rnd $L N$1 inflight $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_${L}_n$1_inflight_$rnd.json) one $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_${L}_n$1_one_$rnd.json) primary_one $(python3 -c "import json;print(round(json.load(open('gpurun_out/${T}_${L}_n$1_one_$rnd.json'))['ms_stage'][5],4))")"
  done
done
done
echo "call ok"
