#!/usr/bin/env python3
"""Turn rocprofv3 --pmc passes of scripts/profile_trace.py into profiles/pmc_<workload>.json,
the per-launch HBM traffic bench.py reports as roofline.traffic.

HBM read bytes  = 128 * TCC_EA0_RDREQ_128B + 64 * TCC_EA0_RDREQ_64B + 32 * TCC_EA0_RDREQ_32B
HBM write bytes = 64 * TCC_EA0_WRREQ_64B + 32 * (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)
Calibrated with scripts/calib_fetch.hip (profiles/r01_calib_fetch.json): a coalesced
16-B/lane stream of 4 GiB issues 33.5M 128-B requests (FETCH_SIZE reports half, as the
guide says) and a permutation gather of 64-B records (the traversal's node-record
pattern) issues one 128-B request per record, i.e. 2x the record bytes, while
FETCH_SIZE (= RDREQ x 64 B) reports exactly the record bytes.  Counters are summed
over the TCC channels and averaged over the profiled dispatches of each kernel.
records_per_launch (optional COUNTS.json: the stats of one PROF_COUNTS trace of the same mode)
is each kernel's record fetches, so bench.py can scale the bytes to another launch's fetches.
Usage: make_pmc_json.py PMC_DIR MODE WORKLOAD OUT.json [COUNTS.json]   (env PMC_COMMIT: the code's commit)"""
import collections
import csv
import glob
import json
import os
import sys

d, mode, workload, out = sys.argv[1:5]
counts = json.load(open(sys.argv[5])) if len(sys.argv) > 5 else None
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, f"p*_{mode}", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("rtbvh::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if not k.startswith("k_"):
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    g = lambda c: m.get(c, 0.0)  # noqa: E731
    rd = 128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 32 * g("TCC_EA0_RDREQ_32B_sum")
    wr = 64 * g("TCC_EA0_WRREQ_64B_sum") + 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum"))
    base = k.split("<")[0]
    e = {"instance": k, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
         "hbm_bytes_per_launch": rd + wr, "counters": m}
    if counts:
        e["records_per_launch"] = {
            "k_primary": sum(counts["packet_steps"]) or counts["internal_visits"][0] + counts["leaf_visits"][0],
            "k_bounce_trav": counts["internal_visits"][1] + counts["leaf_visits"][1],
            "k_bounce_shade": counts["bounce_rays"]}.get(base)
    if base not in kern or e["hbm_bytes_per_launch"] > kern[base]["hbm_bytes_per_launch"]:
        kern[base] = e
# the binned primary pass (RTBVH_FLAG_BINNED_PRIMARY) as one entry: every instance of its kernels
# summed per launch (the footprint/count and fill passes, the scan, the binned kernel, the shading, and
# the gated packet walk behind them), priced per bin entry
PASS = ("k_pb_bin", "k_pb_sums", "k_pb_scan", "k_primary_binned", "k_pb_shade")
inst = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    g = lambda c: m.get(c, 0.0)  # noqa: E731
    inst[k] = (128 * g("TCC_EA0_RDREQ_128B_sum") + 64 * g("TCC_EA0_RDREQ_64B_sum") + 32 * g("TCC_EA0_RDREQ_32B_sum"),
               64 * g("TCC_EA0_WRREQ_64B_sum") + 32 * (g("TCC_EA0_WRREQ_sum") - g("TCC_EA0_WRREQ_64B_sum")))
parts = [k for k in inst if k.split("<")[0] in PASS]
if parts:
    gated = [k for k in inst if k.startswith("k_primary<")]
    parts += gated
    rd = sum(inst[k][0] for k in parts)
    wr = sum(inst[k][1] for k in parts)
    kern["k_primary_pass"] = {"instance": parts, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                              "hbm_bytes_per_launch": rd + wr,
                              "records_per_launch": counts["bin_entries"][0] if counts else None}
json.dump({"workload": workload, "mode": mode, "source": d, "commit": os.environ.get("PMC_COMMIT"),
           "method": __doc__.split("Usage")[0].strip(), "kernels": kern}, open(out, "w"), indent=1)
for k, v in kern.items():
    print(k, v["instance"], "%.3f GB read, %.3f GB write" % (v["hbm_read_bytes_per_launch"] / 1e9,
                                                             v["hbm_write_bytes_per_launch"] / 1e9))
