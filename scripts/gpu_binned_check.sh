set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "binned" > gpurun_out/binned_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/binned_tests.log; exit 1; }
tail -3 gpurun_out/binned_tests.log
AB_SET=binned AB_COUNTS=1 AB_ROUNDS=3 timeout -k 10 300 python -u scripts/ab_trace.py > gpurun_out/ab_binned.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/ab_binned.log; exit 1; }
cat gpurun_out/ab_binned.log
