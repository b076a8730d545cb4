# Round 5, call x: AUTO_WALK's timed choice of the small-scene primary kind (lanes or wave packets): the GPU
# suite, then C3 / C2 rebuilt frames (AUTO, as one hipGraph) and which kind each kept.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; grep -E "^(FAILED|E  )" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; fi
CONFIGS=auto,packet timeout -k 10 300 python scripts/c3_modes.py > gpurun_out/${T}_c3.log 2>&1 || { tail -5 gpurun_out/${T}_c3.log; exit 1; }
SCENE=Image_Test BOUNCES=0 CONFIGS=auto,packet timeout -k 10 300 python scripts/c3_modes.py > gpurun_out/${T}_c2.log 2>&1 || { tail -5 gpurun_out/${T}_c2.log; exit 1; }
grep -h config gpurun_out/${T}_c3.log gpurun_out/${T}_c2.log | cut -c1-200
echo "call ok"
