# GPU tests (optional) + A/B of library builds: AB_LIBS="a.so b.so", AB_SCRIPT (ab_trace.py | ab_build.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
bash scripts/ab_libs.sh $AB_LIBS 2>&1 | tee gpurun_out/ab.log
