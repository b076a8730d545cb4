# fused refit tail: GPU tests touching compute_bvh / binned / trees, then the rebuilt-frame timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "overlap or graph or binned or compute or auto or pseudo or grid or c5 or in_flight" --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -1 gpurun_out/tail_tests.log
cd /tmp && export TMPDIR=/tmp
FRAMES=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tail -o run -- python3 $R/scripts/frame_rebuild.py > $R/gpurun_out/prof_tail.log 2>&1 || { echo "PROF FAILED"; exit 1; }
python3 $R/scripts/frame_timeline.py $R/gpurun_out/prof_tail/run_kernel_trace.csv $R/gpurun_out/frame_timeline_tail.json
