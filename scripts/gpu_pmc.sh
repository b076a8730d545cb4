# PMC passes (separate rocprofv3 runs, --kernel-trace only besides --pmc).
# MODES: space-separated PROF_MODE values; SETS: ';'-separated counter sets.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${PMC_OUT:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
DEFAULT_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum;FETCH_SIZE;WRITE_SIZE;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum;TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
IFS=';' read -ra SETARR <<< "${SETS:-$DEFAULT_SETS}"
i=0
for set in "${SETARR[@]}"; do
  i=$((i+1))
  for mode in ${MODES:-nearest reference+sort}; do
    PROF_MODE=$mode PROF_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p${i}_$mode -o run -- python3 $R/scripts/profile_trace.py > $OUT/p${i}_$mode.log 2>&1 || { echo "pass $i $mode failed"; tail -5 $OUT/p${i}_$mode.log; exit 1; }
  done
done
echo pmc done
