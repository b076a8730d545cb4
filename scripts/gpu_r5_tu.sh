# Round 5, calls t + u + v in one box: the compute_bvh kernel timeline, frames in flight x hardware queues,
# C3 under several walk configurations (scripts/c3_modes.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r5_t.sh && bash scripts/gpu_r5_u.sh && timeout -k 10 300 python scripts/c3_modes.py > gpurun_out/r05_v_c3_modes.log 2>&1 && cat gpurun_out/r05_v_c3_modes.log
