# PMC passes of scripts/rank_sim.py restricted to one rank's bands (RANK_SIM_ONLY=N,r):
# counters of the trace kernels for the whole frame (1,0) vs a rank of N=8 (8,0).
# CFGS: space-separated N,r pairs; SETS: ';'-separated counter sets (one rocprofv3 run each).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PMC_OUT:-rs_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
DEFAULT_SETS="TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
IFS=';' read -ra SETARR <<< "${SETS:-$DEFAULT_SETS}"
for cfg in ${CFGS:-1,0 8,0}; do
  i=0
  for set in "${SETARR[@]}"; do
    i=$((i+1))
    tag=p${i}_${cfg/,/_}
    RANK_SIM_ONLY=$cfg timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$tag -o run -- python3 $R/scripts/rank_sim.py 3 > $OUT/$tag.log 2>&1 || { echo "fail $cfg $i"; tail -5 $OUT/$tag.log; exit 1; }
  done
done
echo ok
