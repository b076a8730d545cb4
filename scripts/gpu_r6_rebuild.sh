# Round 6: rebuilt-frame timelines (AUTO_WALK | GRAPH, scripts/frame_rebuild.py under rocprofv3 --kernel-trace) for
# (RTBVH_FLAT_CLIMB existed until round 6's r06_o measurement: deleted after it)
# the env settings in VARIANTS (';'-separated, e.g. "RTBVH_FLAT_CLIMB=0;RTBVH_FLAT_CLIMB=1"), interleaved ROUNDS times
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
T=${TAG:-r06_rb}
IFS=';' read -ra VS <<< "${VARIANTS:-RTBVH_FLAT_CLIMB=0}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "${VS[@]}"; do
    i=$((i+1))
    d=$R/gpurun_out/${T}_v${i}_r$r
    env $v FRAME_FLAGS=$(( (1<<8) | (1<<20) )) FRAMES=10 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 $R/scripts/frame_rebuild.py > $d.log 2>&1 || { echo "FAILED $v"; tail -5 $d.log; exit 1; }
    python3 $R/scripts/frame_timeline.py $d/run_kernel_trace.csv $d.json || exit 1
    python3 -c "
import json; d=json.load(open('$d.json'))
ks={}
for k in d['kernels']: ks[k['kernel']]=ks.get(k['kernel'],0)+k['ms']
top=sorted(ks.items(), key=lambda x:-x[1])[:12]
print('$v', 'frame_ms_median', d['frame_ms_median'], 'min', d['frame_ms_min'], {a: round(b,4) for a,b in top})"
  done
done
echo "call ok"
