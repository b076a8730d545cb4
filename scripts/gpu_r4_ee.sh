# Round 4, call ee: the small scenes' bounce pass on LDS-resident node records (boxes + child ids,
# 112 KB) with 8 LDS stack entries per lane (k_bounce_lds) against the committed k_bounce: GPU suite,
# C3 / C2 frames.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_ee}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for r in 1 2; do
  for lib in librtbvh_flat.so new; do
    L=$PWD/ablib/$lib; [ $lib = new ] && L=$PWD/raytracebvh_amd/librtbvh.so
    echo -n "$lib " >> gpurun_out/${T}_lds_ab.log
    RTBVH_LIB=$L timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_lds_ab.log || { echo "C3 $lib FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_lds_ab.log
echo "call ok"
