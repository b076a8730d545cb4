#!/usr/bin/env python3
"""One rebuilt frame's kernel timeline from a rocprofv3 --kernel-trace CSV of
scripts/frame_rebuild.py: frames split at k_morton (the build's first kernel), and for each
kernel of the median frame its start / end relative to the frame start and the idle gap before
it (the GPU idle between launches; with two streams, idle while neither runs).  Writes JSON.

A trace frame (scripts/rank_prof.py) splits at k_zero, its first kernel: pass it as the third argument.

usage: python scripts/frame_timeline.py run_kernel_trace.csv out.json [first kernel, default k_morton]"""
import csv
import json
import statistics
import sys


def short(name):
    name = name.replace("void rtbvh::(anonymous namespace)::", "").replace("rtbvh::(anonymous namespace)::", "")
    return name.split("(")[0]


def main(src, dst, first="k_morton"):
    rows = []
    with open(src) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    frames, cur = [], None
    for s, e, n in rows:
        if n == first or n.startswith(first + "<"):
            cur = []
            frames.append(cur)
        if cur is not None:
            cur.append((s, e, n))
    frames = frames[2:] or frames   # skip the warm-ups
    spans = [(max(k[1] for k in f) - f[0][0]) / 1e6 for f in frames]   # (kernels of two streams overlap)
    med = sorted(range(len(frames)), key=lambda i: spans[i])[len(frames) // 2]
    f = frames[med]
    t0 = f[0][0]
    out = {"frames": len(frames), "frame_ms_median": round(statistics.median(spans), 4),
           "frame_ms_min": round(min(spans), 4), "kernels": []}
    prev_end = t0
    busy = 0
    for s, e, n in f:
        out["kernels"].append({"kernel": n, "start_ms": round((s - t0) / 1e6, 4), "ms": round((e - s) / 1e6, 4),
                               "gap_before_ms": round(max(0, s - prev_end) / 1e6, 4)})
        busy += e - s
        prev_end = max(prev_end, e)
    out["kernel_ms_sum"] = round(busy / 1e6, 4)
    out["gaps_ms_sum"] = round(sum(k["gap_before_ms"] for k in out["kernels"]), 4)
    # kernel time hidden under other kernels (the binned primary pass beside the build's crossing nodes)
    out["overlap_ms"] = round(out["kernel_ms_sum"] + out["gaps_ms_sum"] - (prev_end - t0) / 1e6, 4)
    stage = {}
    for k in out["kernels"]:
        stage[k["kernel"]] = round(stage.get(k["kernel"], 0) + k["ms"], 4)
    out["ms_by_kernel"] = stage
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("frames", "frame_ms_median", "kernel_ms_sum", "gaps_ms_sum", "overlap_ms")}))


if __name__ == "__main__":
    main(*sys.argv[1:4])
