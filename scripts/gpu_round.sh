# One GPU call: parity tests -> PMC passes of the bench's traversal mode (HBM request counters,
# instruction mix; written to profiles/pmc_c5_nearest-first-wide.json, which bench.py reads) ->
# bench -> rocprofv3 kernel-trace/stats of the same bench command.
# Everything lands under gpurun_out/; every GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_MODE=${PMC_MODE:-nearest+packet+refill+wide+binned}
PMC_NAME=${PMC_NAME:-nearest-first-wide-binned}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
if [ -z "$SKIP_PMC" ]; then
  PROF_MODE=$PMC_MODE PROF_ITERS=1 PROF_COUNTS=$R/gpurun_out/counts_round.json timeout -k 10 300 python3 scripts/profile_trace.py > gpurun_out/counts_round.log 2>&1 || { echo "COUNTS FAILED"; tail -5 gpurun_out/counts_round.log; exit 1; }
  PMC_OUT=pmc_round MODES="$PMC_MODE" SETS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum;TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" bash scripts/gpu_pmc.sh || exit 1
  cd $R
  python3 scripts/make_pmc_json.py gpurun_out/pmc_round "$PMC_MODE" c5 gpurun_out/pmc_c5_round.json gpurun_out/counts_round.json || exit 1
  cp gpurun_out/pmc_c5_round.json profiles/pmc_c5_$PMC_NAME.json
  echo "pmc ok"
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py ${BENCH_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || { echo "PROF FAILED"; tail -20 gpurun_out/prof_bench.err; exit 1; }
  echo "prof ok"
fi
echo "round ok"
