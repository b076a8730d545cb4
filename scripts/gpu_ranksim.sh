# GPU tests -> bench -> per-rank simulation of the N-GPU split (scripts/rank_sim.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python scripts/rank_sim.py 10 > gpurun_out/rank_sim.json 2> gpurun_out/rank_sim.err || { echo "RANKSIM FAILED"; tail -20 gpurun_out/rank_sim.err; exit 1; }
cat gpurun_out/rank_sim.json
