# Round 5, call n: the rays a certified walk cannot take at all re-traced beside the walk (k_bounce_redo_early,
# its own stream) -- the GPU suite, then one-frame certified traces with RTBVH_EARLY_REDO=1 / 0 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_n}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; fi
for r in 1 2; do
  for e in 1 0; do
    out=$(RTBVH_EARLY_REDO=$e AB_SET=certbase AB_ROUNDS=3 timeout -k 10 300 python scripts/ab_trace.py 2>&1) || { echo "$out" | tail -5; exit 1; }
    echo "early=$e $(echo "$out" | grep -E "ms_med|frame_sha1" | tr '\n' ' ' | cut -c1-420)" | tee -a gpurun_out/${T}_early_ab.log
  done
done
echo "call ok"
