set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RANK_SIM_SPLITS=0,2,3 RANK_SIM_N=1,8 timeout -k 10 300 python scripts/rank_sim.py 10 > gpurun_out/rank_sim_split.json 2> gpurun_out/rank_sim_split.err || { echo FAIL1; tail gpurun_out/rank_sim_split.err; exit 1; }
cat gpurun_out/rank_sim_split.json
timeout -k 10 300 python scripts/walk_census.py > gpurun_out/census.json 2> gpurun_out/census.err || { echo FAIL2; tail gpurun_out/census.err; exit 1; }
cat gpurun_out/census.json
