# Round 4, call t: AUTO on small scenes with the packet primary pass (C3, C2) beside the plain
# reference-order kernels; the one-workgroup build's phase times (probe build); the AUTO/packet tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_t}
for r in 1 2; do
  for m in auto plain; do
    C3_MODE=$m timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_small_modes.log || { echo "C3 $m FAILED"; exit 1; }
    C3_SCENE=Image_Test C3_BOUNCES=0 C3_MODE=$m timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_small_modes.log || { echo "C2 $m FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_small_modes.log
RTBVH_LIB=$PWD/ablib/librtbvh_sprobe.so C3_FRAMES=5 timeout -k 10 120 python -u scripts/c3_profile.py > gpurun_out/${T}_small_probe.log 2>&1 || { echo "probe FAILED"; tail -5 gpurun_out/${T}_small_probe.log; exit 1; }
grep SMALLPROBE gpurun_out/${T}_small_probe.log | tail -6
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "auto or packet or verify" > gpurun_out/${T}_tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
echo "call ok"
