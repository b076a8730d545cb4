# Frames in flight x bounce grid sweep of the C5 headline (bench.py --no-cpu-baseline --no-extras).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in ${CFGS:-"3 2048" "4 2048" "3 1536" "4 1536" "3 1024" "4 1024" "3 2048"}; do
  set -- $cfg
  RTBVH_BOUNCE_BLOCKS=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --inflight $1 --steps 30 > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err || { echo "BENCH $cfg FAILED"; tail -20 gpurun_out/sw_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw_$1_$2.json'));print('inflight $1 blocks $2', 'value', d['value'], 'ms', d['ms_per_step'], 'lat', d['traversal']['one_frame_latency_ms'], 'ident', d['traversal']['inflight_frame_identical'])"
done
