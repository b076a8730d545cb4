# Round 4, call bb (final): the bench on the committed code, then rocprofv3 kernel stats of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_bb}
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err || { echo "PROF FAILED"; tail -20 gpurun_out/${T}_prof_bench.err; exit 1; }
echo "call ok"
