# Round 4, call y: the GPU suite on the committed one-workgroup build, the C3 frame beside the previous
# library, its phase probe, then PMC passes over the C3 frame (scripts/gpu_r4_v.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_y}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for r in 1 2; do
  for lib in librtbvh_old.so new; do
    L=$PWD/ablib/$lib; [ $lib = new ] && L=$PWD/raytracebvh_amd/librtbvh.so
    echo -n "$lib " >> gpurun_out/${T}_small_ab.log
    RTBVH_LIB=$L timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_small_ab.log || { echo "C3 $lib FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_small_ab.log
RTBVH_LIB=$PWD/ablib/librtbvh_sprobe.so C3_FRAMES=5 timeout -k 10 120 python -u scripts/c3_profile.py > gpurun_out/${T}_small_probe.log 2>&1 || { echo "probe FAILED"; exit 1; }
grep SMALLPROBE gpurun_out/${T}_small_probe.log | tail -3
TAG=${T} bash scripts/gpu_r4_v.sh
