# Headline A/B of two library builds on one box: bench.py (frames in flight, certified) with RTBVH_LIB, interleaved
# ROUNDS times; then scripts/ab_trace.py AB_SET=certbase (one frame at a time) over both.  Outputs gpurun_out/${TAG}_*.
#   TAG=r06_hab bash scripts/gpu_r6_headline_ab.sh ablib/a.so ablib/b.so
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${TAG:-r06_hab}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    RTBVH_LIB=$(realpath $lib) timeout -k 10 300 python bench.py > gpurun_out/${T}_$(basename $lib .so)_$r.json 2> gpurun_out/${T}_err.log || { tail -5 gpurun_out/${T}_err.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_ms'], d['c5_frame_rebuild']['ms_per_frame_graph'])" gpurun_out/${T}_$(basename $lib .so)_$r.json $(basename $lib)
  done
done
AB_SET=certbase ROUNDS=2 bash scripts/ab_libs.sh "$@"
