# Round 4, call s: the C3 frame (the metric's own config) under each exact walk set -- AUTO's plain
# reference-order kernels, the reference order's packet + refill kernels, the certified fast walks --
# rebuilt per frame as one hipGraph; frames compared by hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04_s}
for r in 1 2; do
  for m in auto fast certified; do
    C3_MODE=$m C3_GRAPH=1 timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_c3_modes.log || { echo "C3 $m FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_c3_modes.log
echo "call ok"
