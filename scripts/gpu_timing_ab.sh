# rebuilt C5 frame timelines: plain vs RTBVH_FLAG_TIMING (A/B of the timing events' cost)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for F in 0 1; do
  FRAME_FLAGS=$F FRAMES=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_t$F -o run -- python3 $R/scripts/frame_rebuild.py > $R/gpurun_out/prof_t$F.log 2>&1 || { echo "PROF FAILED"; tail -5 $R/gpurun_out/prof_t$F.log; exit 1; }
  python3 $R/scripts/frame_timeline.py $R/gpurun_out/prof_t$F/run_kernel_trace.csv $R/gpurun_out/frame_timeline_t$F.json
done
