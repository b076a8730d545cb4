# Round 4, call x (final): GPU suite; the C3 frame with the one-workgroup build's new sort / climb beside
# the previous library (+ its phase probe); the bench; rocprofv3 kernel stats of the same bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_x}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
for r in 1 2; do
  for lib in librtbvh_old.so new; do
    L=$PWD/ablib/$lib; [ $lib = new ] && L=$PWD/raytracebvh_amd/librtbvh.so
    echo -n "$lib " >> gpurun_out/${T}_small_ab.log
    RTBVH_LIB=$L timeout -k 10 120 python -u scripts/c3_profile.py 2>/dev/null | tail -1 >> gpurun_out/${T}_small_ab.log || { echo "C3 $lib FAILED"; exit 1; }
  done
done
cat gpurun_out/${T}_small_ab.log
RTBVH_LIB=$PWD/ablib/librtbvh_sprobe.so C3_FRAMES=5 timeout -k 10 120 python -u scripts/c3_profile.py > gpurun_out/${T}_small_probe.log 2>&1 || { echo "probe FAILED"; exit 1; }
grep SMALLPROBE gpurun_out/${T}_small_probe.log | tail -3
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','certified_mrays_s','c5_orbit_ms_per_frame','c5_frame_rebuild_ms')}); print('c3', d.get('extras',{}).get('c3_frame') or d.get('c3_1080p'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err || { echo "PROF FAILED"; tail -20 gpurun_out/${T}_prof_bench.err; exit 1; }
echo "call ok"
