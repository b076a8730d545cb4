# Rehearsal of bench.py's N-rank path on ONE GPU: N processes on cuda:0 over gloo (the
# driver's N-GPU runs use RCCL, one GPU per rank).  N = 2 and 3 (ragged band split).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for N in ${RANKS:-2 3}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29400 + N)) bench.py --gpus $N --backend gloo --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/rehearse_n$N.json 2> gpurun_out/rehearse_n$N.err || { echo "N=$N FAILED"; tail -30 gpurun_out/rehearse_n$N.err; exit 1; }
  cat gpurun_out/rehearse_n$N.json
done
