cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 0 1 2; do timeout -k 10 250 python scripts/inflight_check.py 10 > gpurun_out/ifc$i.json 2>gpurun_out/ifc$i.err & done
wait
cat gpurun_out/ifc0.json gpurun_out/ifc1.json gpurun_out/ifc2.json
