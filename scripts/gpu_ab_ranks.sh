# GPU tests -> bench -> rank simulation at N=1,8 for kernel variants (RANK_SIM_VARIANTS).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-extras} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
RANK_SIM_VARIANTS=${VARIANTS:-0} RANK_SIM_N=1,8 timeout -k 10 300 python scripts/rank_sim.py 10 > gpurun_out/rank_sim.json 2> gpurun_out/rank_sim.err || { echo "RANKSIM FAILED"; tail -20 gpurun_out/rank_sim.err; exit 1; }
cat gpurun_out/rank_sim.json
