# tests + bench (+ rocprofv3 kernel stats of the bench) in one call; outputs under gpurun_out/<tag>_*
# usage: TAG=r04_a BENCH_ARGS="..." bash scripts/gpu_r4.sh   (PROF=1: also the rocprofv3 stats pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-run}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
  tail -2 gpurun_out/${T}_gpu_tests.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.err || { echo "PROF FAILED"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.err; exit 1; }
  echo prof ok
fi
