set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RTBVH_LIB=$GRAFT_REPO_ROOT/raytracebvh_amd/librtbvh_prof.so timeout -k 10 300 python -u scripts/pb_phases.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pb_phases.log
AB_SET=binned AB_ROUNDS=3 timeout -k 10 300 python -u scripts/ab_trace.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_binned.log
