# Round 5, call ii: the 512-block bounce grid for small in-flight shards (api.hip): band / in-flight tests, then
# per-rank frames at N = 8 / 4 / 2 / 1 (four in flight, one frame)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_ii}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "band or flight" > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_tests.log | head -20; exit 1; fi
for NR in "8 1" "4 1" "2 1" "1 0"; do
  set -- $NR
  timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 40 inflight 4 > gpurun_out/${T}_n$1_inflight.json 2>> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
  timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 20 > gpurun_out/${T}_n$1_one.json 2>> gpurun_out/${T}.err || { tail -5 gpurun_out/${T}.err; exit 1; }
  echo "N$1 inflight $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_n$1_inflight.json) one $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_n$1_one.json)"
done
echo "call ok"
