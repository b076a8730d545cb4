# Round 6: PMC of the certified bounce walk on the six-wide tree (RTBVH_W6=1) against the 4-wide one
# (RTBVH_W6 existed at commit 2b9ee26 only: deleted after this measurement)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-r06_w6pmc}
mkdir -p $O
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  for w in 0 1; do
    RTBVH_W6=$w PROF_MODE=certified PROF_ITERS=2 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/p${i}_w$w -o run -- python3 $R/scripts/profile_trace.py > $O/p${i}_w$w.log 2>&1 || { echo "pass $i w$w failed"; tail -5 $O/p${i}_w$w.log; exit 1; }
  done
done
python3 - <<PY
import csv, glob, collections, os
for w in (0, 1):
    acc = collections.defaultdict(list)
    for f in glob.glob("$O/p*_w%d/run_counter_collection.csv" % w):
        for r in csv.DictReader(open(f)):
            if "k_bounce_trav" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("W6=%d" % w, {k: round(sum(v) / len(v) / 1e6, 2) for k, v in sorted(acc.items())})
PY
echo "call ok"
