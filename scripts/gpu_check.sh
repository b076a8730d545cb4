# One GPU call: the GPU parity suite, the N=3 gloo rehearsal of bench.py's multi-rank path
# (uneven band deal) and the default bench; outputs under gpurun_out/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
if [ -z "$SKIP_REHEARSE" ]; then
  RANKS=${RANKS:-3} bash scripts/gpu_rehearse_ranks.sh > gpurun_out/rehearse.log 2>&1 || { echo "REHEARSE FAILED"; tail -30 gpurun_out/rehearse.log; exit 1; }
  echo "rehearse ok"
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
