# rocprofv3 kernel trace of the rebuilt C5 frame (build + binned primary + 1 bounce every frame),
# plain and as a hipGraph; summarised by scripts/frame_timeline.py into gpurun_out/frame_timeline*.json
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
FRAMES=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_frame -o run -- python3 $R/scripts/frame_rebuild.py > $R/gpurun_out/prof_frame.log 2>&1 || { echo "PROF FAILED"; tail -5 $R/gpurun_out/prof_frame.log; exit 1; }
python3 $R/scripts/frame_timeline.py $R/gpurun_out/prof_frame/run_kernel_trace.csv $R/gpurun_out/frame_timeline.json
