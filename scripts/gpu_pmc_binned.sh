# PMC passes of the binned primary kernels (C5): wave-time split, instruction mix, LDS
set -o pipefail
R=$GRAFT_REPO_ROOT
MODES="nearest+packet+refill+wide+binned" PMC_OUT=pmc_binned SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT;TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE" bash $R/scripts/gpu_pmc.sh || exit 1
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_binned nearest+packet+refill+wide+binned > gpurun_out/pmc_binned.json
