# Round 5, call p: hardware queues per process (GPU_MAX_HW_QUEUES 4 = HIP's default, 8) against the bench's
# frames in flight (four caller streams + the context's), bench without extras / CPU baseline, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r05_p}
for r in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 600 python bench.py --no-extras --no-cpu-baseline > gpurun_out/${T}_hwq${q}_${r}.json 2> gpurun_out/${T}_hwq${q}_${r}.err || { echo "BENCH FAILED"; tail -5 gpurun_out/${T}_hwq${q}_${r}.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); t=d['traversal']; print(sys.argv[2], d['value'], d['ms_per_step'], t.get('fastest_identical_ms'), t.get('runs_ms',{}).get('certified'))" gpurun_out/${T}_hwq${q}_${r}.json hwq$q
  done
done
echo "call ok"
