"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV (median / mean / min per
kernel name and grid), the form of profiles/r02_kernel_trace_summary.json.

usage: python scripts/trace_summary.py gpurun_out/prof_bench/run_kernel_trace.csv out.json
"""
import csv
import json
import statistics
import sys


def main(src, dst):
    groups = {}
    with open(src) as f:
        for row in csv.DictReader(f):
            ms = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
            name = row["Kernel_Name"].replace("void rtbvh::(anonymous namespace)::", "")
            name = name.split("(")[0] if not name.startswith("(") else name
            key = f'{name} grid={row["Grid_Size_X"]}'
            groups.setdefault(key, []).append(ms)
    out = {k: {"n": len(v), "median_ms": round(statistics.median(v), 4), "mean_ms": round(statistics.mean(v), 4),
               "min_ms": round(min(v), 4)} for k, v in sorted(groups.items(), key=lambda kv: -sum(kv[1]))}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
