# Round 4, call h: tail splitting A/B on the certified mode (trigger at 4 / 8 / 16 rays left in a wave,
# off), with the certified-vs-unchecked counts and walk-length census of the library build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_h}
TAG=$T CERT_AB=1 AB_ROUNDS=2 AB_LIBS="raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_notail.so raytracebvh_amd/librtbvh_tail4.so raytracebvh_amd/librtbvh_tail16.so" LIB_SET=certbase ROUNDS=2 bash scripts/gpu_ab_r4.sh || exit 1
echo "call ok"
