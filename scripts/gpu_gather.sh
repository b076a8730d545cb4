# Memory-system roofline for the traversal's access pattern (scripts/gather_roofline.hip).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in "8 256 1280" "4 256 1280" "2 256 1280" "8 256 128" "8 256 2"; do
  timeout -k 10 60 ./scripts/gather_roofline $cfg >> gpurun_out/gather.jsonl || { echo "FAIL $cfg"; exit 1; }
done
cat gpurun_out/gather.jsonl
