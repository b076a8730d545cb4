# Round 4, call v: PMC passes over the C3 frame (AUTO: the reference-order lane walks), to see what
# bounds k_primary / k_bounce at 1,952 triangles (issue vs latency).
set -o pipefail
R=$GRAFT_REPO_ROOT
export T=${TAG:-r04_v}
OUT=$R/gpurun_out/${T}_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
IFS=';' read -ra SETARR <<< "$SETS"
i=0
for set in "${SETARR[@]}"; do
  i=$((i+1))
  C3_FRAMES=5 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/scripts/c3_profile.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os, collections
out = os.environ.get("GRAFT_REPO_ROOT") + "/gpurun_out/" + os.environ.get("T", "r04_v") + "_pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("rtbvh::(anonymous namespace)::", "")[:60]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "k_primary" in k or "k_bounce" in k or "build_small" in k:
        print(k, {c: round(sum(v) / max(1, len(v)) / (1 if True else 1), 1) for c, v in sorted(d.items())})
PY
echo "call ok"
