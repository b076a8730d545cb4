# Round 5, call d: the certified trace against round 4 (exact-decode certification off by default);
# the C4 build stages: round 4, this code (only the walk's QNodes written), every QNode written; the
# PMC write/read requests of the build kernels with and without the skipped QNodes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_d}
AB_SET=certified AB_COUNTS=1 AB_ROUNDS=3 ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_r4.so raytracebvh_amd/librtbvh.so > gpurun_out/${T}_trace_ab.log 2>&1 || { echo "TRACE AB FAILED"; tail -5 gpurun_out/${T}_trace_ab.log; exit 1; }
grep -v packet_steps gpurun_out/${T}_trace_ab.log | grep ms_med | cut -c1-330
AB_SCRIPT=ab_build.py ROUNDS=2 scripts/ab_libs.sh ablib/librtbvh_r4.so raytracebvh_amd/librtbvh.so ablib/librtbvh_noskip.so > gpurun_out/${T}_build_ab.log 2>&1 || { echo "BUILD AB FAILED"; tail -5 gpurun_out/${T}_build_ab.log; exit 1; }
cut -c1-330 gpurun_out/${T}_build_ab.log
for lib in raytracebvh_amd/librtbvh.so ablib/librtbvh_noskip.so; do
  n=$(basename $lib .so)
  for set in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum"; do
    tag=$(echo $set | cut -c9-13)
    (cd /tmp && RTBVH_LIB=$R/$lib PROF_MODE=certified PROF_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/${T}_pmc_${n}_$tag -o run -- python3 $R/scripts/profile_trace.py > $R/gpurun_out/${T}_pmc_${n}_$tag.log 2>&1) || { echo "PMC $n FAILED"; tail -5 gpurun_out/${T}_pmc_${n}_$tag.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
for d in sorted(glob.glob("gpurun_out/r05_d_pmc_*")):
    if not os.path.isdir(d): continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("rtbvh::(anonymous namespace)::", "")
            if "refit" in k or "qnodes" in k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(os.path.basename(d), k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in cs.items()})
PY
echo "call ok"
