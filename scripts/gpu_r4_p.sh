# Round 4, call p: the certified walk's pre-bound stack keys -- each box's key the entry of the box grown
# by rho(its own entry) (perbox), against the keys lowered by rho max|1/d| at the first bound (maxinv) and
# neither (nofix) -- certified-mode library A/B with the walk census, then the certified parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_p}
TAG=$T CERT_AB=0 AB_ROUNDS=3 AB_LIBS="raytracebvh_amd/librtbvh_perbox.so raytracebvh_amd/librtbvh_maxinv.so raytracebvh_amd/librtbvh_nofix.so" LIB_SET=certbase ROUNDS=2 bash scripts/gpu_ab_r4.sh || exit 1
for lib in perbox maxinv; do
  RTBVH_LIB=$(realpath raytracebvh_amd/librtbvh_$lib.so) AB_SET=certbase AB_COUNTS=1 AB_ROUNDS=1 timeout -k 10 300 python -u scripts/ab_trace.py > gpurun_out/${T}_census_$lib.log 2>&1 || { echo "CENSUS FAILED"; tail -5 gpurun_out/${T}_census_$lib.log; exit 1; }
  echo "$lib $(grep trav_max gpurun_out/${T}_census_$lib.log)"
done
RTBVH_LIB=$(realpath raytracebvh_amd/librtbvh_perbox.so) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "certified or auto_walk or orbit or containment" > gpurun_out/${T}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
echo "call ok"
