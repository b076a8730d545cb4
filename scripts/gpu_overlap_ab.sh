# the rebuilt C5 frame (rocprof span) and bench.py's c5_frame_rebuild, with and without RTBVH_OVERLAP
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "overlap or pseudo or grid" --timeout 120 --timeout-method thread > gpurun_out/ovab_tests.log 2>&1 || { tail -20 gpurun_out/ovab_tests.log; exit 1; }
tail -1 gpurun_out/ovab_tests.log
cd /tmp && export TMPDIR=/tmp
for O in 0 1; do
  RTBVH_OVERLAP=$O FRAMES=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_o$O -o run -- python3 $R/scripts/frame_rebuild.py > $R/gpurun_out/prof_o$O.log 2>&1 || { echo "PROF FAILED"; exit 1; }
  python3 $R/scripts/frame_timeline.py $R/gpurun_out/prof_o$O/run_kernel_trace.csv $R/gpurun_out/frame_timeline_o$O.json
done
