# Round 5, call w: the packet primary pass (reference-order wave packets) against AUTO's lane kernels on C3
# (Test.obj, primary + 1 bounce) and C2 (Image_Test.obj, primary only), rebuilt frames as one hipGraph.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CONFIGS=auto,packet timeout -k 10 300 python scripts/c3_modes.py > gpurun_out/r05_w_c3.log 2>&1 || { tail -5 gpurun_out/r05_w_c3.log; exit 1; }
SCENE=Image_Test BOUNCES=0 CONFIGS=auto,packet timeout -k 10 300 python scripts/c3_modes.py > gpurun_out/r05_w_c2.log 2>&1 || { tail -5 gpurun_out/r05_w_c2.log; exit 1; }
grep -h config gpurun_out/r05_w_c3.log gpurun_out/r05_w_c2.log | cut -c1-260
echo "call ok"
