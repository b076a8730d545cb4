# Round 4, call e: cost probes of k_primary_binned's fine phase (RTBVH_PB_PROBE builds: wrong frames,
# timing only) against the library, binned mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04_e} CERT_AB=1 AB_ROUNDS=2 AB_LIBS="${AB_LIBS:-raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_pbp1.so raytracebvh_amd/librtbvh_pbp2.so}" LIB_SET=${LIB_SET:-binnedbase} ROUNDS=2 bash scripts/gpu_ab_r4.sh || exit 1
echo "call ok"
