# Round 4, call dd: the lane walks' LDS stack entries read with ds_read (a module-scope array, the LDS
# and scratch loads kept apart) against the committed form (a generic pointer: flat loads): GPU suite,
# C3 and C2 frames.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_dd}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for r in 1 2; do
  for lib in librtbvh_flat.so new; do
    L=$PWD/ablib/$lib; [ $lib = new ] && L=$PWD/raytracebvh_amd/librtbvh.so
    echo -n "$lib " >> gpurun_out/${T}_lsb_ab.log
    RTBVH_LIB=$L timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_lsb_ab.log || { echo "C3 $lib FAILED"; exit 1; }
    echo -n "$lib C2 " >> gpurun_out/${T}_lsb_ab.log
    RTBVH_LIB=$L C3_SCENE=Image_Test C3_BOUNCES=0 timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_lsb_ab.log || { echo "C2 $lib FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_lsb_ab.log
echo "call ok"
