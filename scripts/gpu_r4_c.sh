# Round 4, call c: kernel trace of the certified walks against the unchecked ones (the re-trace
# kernels' own durations), the refit-gather cache-policy probe (time + 64/128-B memory requests), and
# the bench's orbit extras.  Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_c}
AB_SET=certified AB_ROUNDS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_certprof -o run -- python3 scripts/ab_trace.py > gpurun_out/${T}_certprof.log 2>&1 || { echo "CERT PROF FAILED"; tail -20 gpurun_out/${T}_certprof.log; exit 1; }
echo "cert prof ok"
timeout -k 10 120 ./scripts/gather_policy > gpurun_out/${T}_gather_policy.json 2>&1 || { echo "GATHER POLICY FAILED"; cat gpurun_out/${T}_gather_policy.json; exit 1; }
cat gpurun_out/${T}_gather_policy.json
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_gp_pmc -o run -- ./scripts/gather_policy > gpurun_out/${T}_gp_pmc.log 2>&1 || { echo "GATHER PMC FAILED"; tail -20 gpurun_out/${T}_gp_pmc.log; exit 1; }
echo "gather pmc ok"
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
  cat gpurun_out/${T}_bench.json
fi
echo "call ok"
