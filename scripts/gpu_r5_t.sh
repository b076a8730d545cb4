# Round 5, call t: the kernel timeline of rtbvh_compute_bvh frames (the rebuilt frame, AUTO_WALK), plain and
# as one hipGraph, for the gaps between kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_t}
PROF_COMPUTE=1 PROF_MODE=auto PROF_ITERS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_compute -o run -- python3 $GRAFT_REPO_ROOT/scripts/profile_trace.py > gpurun_out/${T}_compute.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${T}_compute.log; exit 1; }
echo "call ok"
