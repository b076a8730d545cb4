# bench c5_frame_rebuild under three side-stream settings (A/B)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 > gpurun_out/ab_hi.json 2> gpurun_out/ab_hi.err || { tail -5 gpurun_out/ab_hi.err; exit 1; }
RTBVH_SIDE_PRIORITY=0 timeout -k 10 400 python bench.py --steps 10 > gpurun_out/ab_lo.json 2> gpurun_out/ab_lo.err || { tail -5 gpurun_out/ab_lo.err; exit 1; }
RTBVH_NO_OVERLAP=1 timeout -k 10 400 python bench.py --steps 10 > gpurun_out/ab_no.json 2> gpurun_out/ab_no.err || { tail -5 gpurun_out/ab_no.err; exit 1; }
for f in hi lo no; do python3 -c "import json,sys; b=json.loads(open('gpurun_out/ab_$f.json').read().strip().splitlines()[-1]); r=b['c5_frame_rebuild']; print('$f', b['value'], r['ms_per_frame'], r['ms_per_frame_graph'], r['ms_per_frame_pipelined2'])"; done
