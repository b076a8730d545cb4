# the overlapped rebuilt frame: GPU parity suite, then the frame timeline (plain and graph)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} --timeout 120 --timeout-method thread > gpurun_out/ov_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ov_tests.log; exit 1; }
tail -2 gpurun_out/ov_tests.log
bash scripts/gpu_frame_timeline.sh || exit 1
cd /tmp && export TMPDIR=/tmp
FRAME_FLAGS=0x100000 FRAMES=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_frame_g -o run -- python3 $R/scripts/frame_rebuild.py > $R/gpurun_out/prof_frame_g.log 2>&1 || { echo "GRAPH PROF FAILED"; tail -5 $R/gpurun_out/prof_frame_g.log; exit 1; }
python3 $R/scripts/frame_timeline.py $R/gpurun_out/prof_frame_g/run_kernel_trace.csv $R/gpurun_out/frame_timeline_graph.json
