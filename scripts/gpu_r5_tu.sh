# Round 5, calls t + u in one box: the compute_bvh kernel timeline, then frames in flight x hardware queues.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r5_t.sh && bash scripts/gpu_r5_u.sh
