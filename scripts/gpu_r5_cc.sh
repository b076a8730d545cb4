# Round 5, call cc: where a rank's frame goes at N = 8 (certified, rank 1) against N = 1: per-kernel
# rocprofv3 stats one frame at a time, and the host time per frame with four in flight
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for NR in "1 0" "8 1"; do
  set -- $NR
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05_cc_n$1 -o run -- python3 scripts/rank_prof.py $1 $2 10 > gpurun_out/r05_cc_n$1_one.json 2> gpurun_out/r05_cc_n$1.err || { tail -5 gpurun_out/r05_cc_n$1.err; exit 1; }
  timeout -k 10 300 python3 scripts/rank_prof.py $1 $2 40 inflight 4 > gpurun_out/r05_cc_n$1_inflight.json 2>> gpurun_out/r05_cc_n$1.err || { tail -5 gpurun_out/r05_cc_n$1.err; exit 1; }
  cat gpurun_out/r05_cc_n$1_one.json gpurun_out/r05_cc_n$1_inflight.json | cut -c1-400
  python3 - "$1" <<'PY'
import csv, sys
n = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/r05_cc_n{n}/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    name = r["Name"].replace("rtbvh::(anonymous namespace)::", "").split("(")[0][:60]
    print(f"N{n} {name:60s} calls {r['Calls']:>4} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
done
echo "call ok"
