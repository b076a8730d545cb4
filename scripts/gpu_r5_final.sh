# Round 5, the measurement call at a commit: the GPU suite; PMC passes of the certified mode (->
# profiles/pmc_c5_certified.json, which bench.py reads; PMC_COMMIT from the caller); a one-frame-at-a-time
# rocprofv3 kernel trace of the same mode; the bench; the bench under rocprofv3 --kernel-trace --stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; fi
PMC_MODE=certified PMC_NAME=certified SKIP_TESTS=1 SKIP_PROF=1 SKIP_BENCH=1 bash scripts/gpu_round.sh > gpurun_out/${T}_pmc.log 2>&1 || { echo "PMC ROUND FAILED"; tail -20 gpurun_out/${T}_pmc.log; exit 1; }
cp gpurun_out/pmc_c5_round.json gpurun_out/${T}_pmc_c5_certified.json
PROF_MODE=certified PROF_ITERS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_oneframe -o run -- python3 $R/scripts/profile_trace.py > gpurun_out/${T}_oneframe.log 2>&1 || { echo "ONE-FRAME PROF FAILED"; tail -5 gpurun_out/${T}_oneframe.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json | cut -c1-600
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_benchprof -o run -- python3 $R/bench.py > gpurun_out/${T}_benchprof.json 2> gpurun_out/${T}_benchprof.err || { echo "BENCH PROF FAILED"; tail -5 gpurun_out/${T}_benchprof.err; exit 1; }
echo "call ok"
