# Round 4, call w: small scenes with the node records resident in LDS (k_primary_lds, k_bounce_lds)
# beside the previous library, the new build alone (lds0) and the bounce pass alone (lds1): full GPU
# suite, then C3 frames (graph, AUTO) interleaved, frames compared by hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_w}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for r in 1 2; do
  for lib in librtbvh_old.so librtbvh_lds0.so librtbvh_lds1.so new; do
    L=$PWD/ablib/$lib; [ $lib = new ] && L=$PWD/raytracebvh_amd/librtbvh.so
    echo -n "$lib " >> gpurun_out/${T}_small_ab.log
    RTBVH_LIB=$L timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_small_ab.log || { echo "C3 $lib FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_small_ab.log

RTBVH_LIB=$PWD/ablib/librtbvh_sprobe.so C3_FRAMES=5 timeout -k 10 120 python -u scripts/c3_profile.py > gpurun_out/${T}_small_probe.log 2>&1 || { echo "probe FAILED"; exit 1; }
grep SMALLPROBE gpurun_out/${T}_small_probe.log | tail -3
echo "call ok"
