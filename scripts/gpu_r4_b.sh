# round 4, call b: PMC passes of the certified mode (profiles/pmc_c5_certified.json comes back under
# gpurun_out/), then the A/B runs (certified vs unchecked walks, row-major fine phase, phase split)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PMC_MODE=certified PMC_NAME=certified SKIP_TESTS=1 SKIP_PROF=1 BENCH_ARGS="--no-cpu-baseline --no-extras --steps 10 --warmup 2" bash scripts/gpu_round.sh > gpurun_out/r04_b_pmc.log 2>&1 || { echo "PMC ROUND FAILED"; tail -20 gpurun_out/r04_b_pmc.log; exit 1; }
tail -3 gpurun_out/r04_b_pmc.log
cp gpurun_out/bench.json gpurun_out/r04_b_bench_short.json
TAG=r04_b AB_LIBS="raytracebvh_amd/librtbvh.so raytracebvh_amd/librtbvh_rm.so" PB_PHASES=1 bash scripts/gpu_ab_r4.sh
