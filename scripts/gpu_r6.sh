# Round 6 GPU call: STEPS (comma list) of tests | oneframe | bench | pmc | benchprof, in that order, each under
# its own time limit, stopping at the first failure.  Outputs under gpurun_out/${TAG}_*.
#   TAG=r06_a STEPS=tests,oneframe,bench bash scripts/gpu_r6.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r06_x}
S=",${STEPS:-tests,oneframe,bench},"
if [[ $S == *,tests,* ]]; then
  KARGS=()
  if [ -n "${PYTEST_K:-}" ]; then KARGS=(-k "$PYTEST_K"); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KARGS[@]}" > gpurun_out/${T}_gpu_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${T}_gpu_tests.log
  if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -30; exit 1; fi
fi
if [[ $S == *,pmc,* ]]; then
  PMC_MODE=certified PMC_NAME=certified SKIP_TESTS=1 SKIP_PROF=1 SKIP_BENCH=1 bash scripts/gpu_round.sh > gpurun_out/${T}_pmc.log 2>&1 || { echo "PMC ROUND FAILED"; tail -20 gpurun_out/${T}_pmc.log; exit 1; }
  cp gpurun_out/pmc_c5_round.json gpurun_out/${T}_pmc_c5_certified.json
fi
if [[ $S == *,oneframe,* ]]; then
  PROF_MODE=${PROF_MODE:-certified} PROF_ITERS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_oneframe -o run -- python3 $R/scripts/profile_trace.py > gpurun_out/${T}_oneframe.log 2>&1 || { echo "ONE-FRAME PROF FAILED"; tail -5 gpurun_out/${T}_oneframe.log; exit 1; }
  python3 - <<EOF
import csv
rows = list(csv.DictReader(open("gpurun_out/${T}_oneframe/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f"{r['Name'][:60]:<60} {r['Calls']:>6} {float(r['AverageNs'])/1e3:10.1f} us")
EOF
fi
if [[ $S == *,bench,* ]]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
  tail -1 gpurun_out/${T}_bench.json | cut -c1-700
fi
if [[ $S == *,benchprof,* ]]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_benchprof -o run -- python3 $R/bench.py > gpurun_out/${T}_benchprof.json 2> gpurun_out/${T}_benchprof.err || { echo "BENCH PROF FAILED"; tail -5 gpurun_out/${T}_benchprof.err; exit 1; }
fi
echo "call ok"
