# Round 4, call r: the C3 frame (Test.obj, 1080p, the metric's own config) -- wall time per rebuilt frame
# (graph and not), stage times, and a rocprofv3 kernel trace of the non-graph frames.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_r}
C3_GRAPH=1 timeout -k 10 120 python -u scripts/c3_profile.py > gpurun_out/${T}_c3_graph.log 2>&1 || { echo "C3 FAILED"; tail -5 gpurun_out/${T}_c3_graph.log; exit 1; }
C3_GRAPH=0 timeout -k 10 120 python -u scripts/c3_profile.py > gpurun_out/${T}_c3_nograph.log 2>&1 || { echo "C3 FAILED"; tail -5 gpurun_out/${T}_c3_nograph.log; exit 1; }
tail -1 gpurun_out/${T}_c3_graph.log; tail -1 gpurun_out/${T}_c3_nograph.log
cd /tmp
C3_GRAPH=0 C3_FRAMES=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_c3prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/c3_profile.py > $GRAFT_REPO_ROOT/gpurun_out/${T}_c3prof.log 2>&1 || { echo "C3 PROF FAILED"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/${T}_c3prof.log; exit 1; }
echo "call ok"
