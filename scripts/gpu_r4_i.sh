# Round 4, call i: the binned pass with 1/det per triangle (RTBVH_PB_HOIST) and the packed fine-phase
# rectangle -- parity tests of the binned / certified modes, then the library A/B (binned mode) against
# the same library without the hoist and the previous commit's.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_i}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "binned or certified or auto_walk" > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
TAG=$T CERT_AB=0 AB_ROUNDS=3 AB_LIBS="raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_nohoist.so raytracebvh_amd/librtbvh_head.so" LIB_SET=binnedbase ROUNDS=2 bash scripts/gpu_ab_r4.sh || exit 1
echo "call ok"
