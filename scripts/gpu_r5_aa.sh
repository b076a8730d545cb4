# Round 5, call aa: PMC of the certified bounce walk, 4-wide (ablib/librtbvh_w4.so) against 8-wide (librtbvh_w8.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum;TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum;SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for L in w4 w8; do
  RTBVH_LIB=$GRAFT_REPO_ROOT/ablib/librtbvh_$L.so PMC_OUT=r05_aa_pmc_$L MODES=certified SETS="$SETS" timeout -k 10 600 bash scripts/gpu_pmc.sh || exit 1
  python3 scripts/pmc_summary.py gpurun_out/r05_aa_pmc_$L certified > gpurun_out/r05_aa_pmc_$L.json || exit 1
done
python3 - <<'PY'
import json
for L in ("w4", "w8"):
    d = json.load(open(f"gpurun_out/r05_aa_pmc_{L}.json"))
    for k, v in d.items():
        if "bounce_trav" in k:
            print(L, k, json.dumps({c: round(x) for c, x in sorted(v.items())}))
PY
echo "call ok"
