# Round 4, call g: the certified walk's tail splitting -- GPU parity tests of the certified walks, then
# the library A/B on the certified mode (tail splitting on / off) with the walk-length census, then the
# binned pass's load/test probes (wrong frames, timing only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "certified or auto_walk or orbit or containment" > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
TAG=$T CERT_AB=1 AB_ROUNDS=2 AB_LIBS="raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_notail.so" LIB_SET=certbase ROUNDS=2 bash scripts/gpu_ab_r4.sh || exit 1
TAG=${T}_pb CERT_AB=0 AB_ROUNDS=2 AB_LIBS="raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_pbp2.so raytracebvh_amd/librtbvh_pbp3.so raytracebvh_amd/librtbvh_pbp4.so" LIB_SET=binnedbase ROUNDS=1 bash scripts/gpu_ab_r4.sh || exit 1
echo "call ok"
