# Round 4, call d: why the certified bounce walk is slower than the unchecked one -- library A/B on the
# certified mode (base; RTBVH_CERT_AB=1 no margin; =2 margin range unbounded), then the certified vs
# unchecked A/B in one process (stage and walk-kernel times, visit counts).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04_d} AB_ROUNDS=3 AB_LIBS="raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_cab1.so raytracebvh_amd/librtbvh_cab2.so" LIB_SET=certbase ROUNDS=2 bash scripts/gpu_ab_r4.sh || exit 1
echo "call ok"
