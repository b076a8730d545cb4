# Round 5, call ee: the N > 1 bin passes over the rank's leaves only (TraceArgs::pb_list): the band / in-flight /
# binned GPU tests on it, then per-rank frames at N = 1 / 4 / 8 (one frame, four in flight) against HEAD's build,
# and the N = 8 rank's kernels under rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_ee}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "band or flight or binned or cert" > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_tests.log | head -20; exit 1; fi
for rnd in 1 2; do
for L in base list; do
  for NR in "8 1" "4 1" "1 0"; do
    set -- $NR
    RTBVH_LIB=$PWD/ablib/librtbvh_$L.so timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 20 > gpurun_out/${T}_${L}_n$1_one_$rnd.json 2>> gpurun_out/${T}_rank.err || { tail -5 gpurun_out/${T}_rank.err; exit 1; }
    RTBVH_LIB=$PWD/ablib/librtbvh_$L.so timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 40 inflight 4 > gpurun_out/${T}_${L}_n$1_inflight_$rnd.json 2>> gpurun_out/${T}_rank.err || { tail -5 gpurun_out/${T}_rank.err; exit 1; }
    echo "r$rnd $L N$1 one $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_${L}_n$1_one_$rnd.json) inflight $(grep -o '"ms_per_frame_host": [0-9.]*' gpurun_out/${T}_${L}_n$1_inflight_$rnd.json)"
  done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_n8 -o run -- python3 scripts/rank_prof.py 8 1 10 > gpurun_out/${T}_n8_prof.json 2>> gpurun_out/${T}_rank.err || { tail -5 gpurun_out/${T}_rank.err; exit 1; }
grep -E "k_pb_bin|k_primary_binned|k_bounce_trav" gpurun_out/${T}_n8/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
echo "call ok"
