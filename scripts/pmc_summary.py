#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*_<mode>/run_counter_collection.csv):
per kernel, the mean of each counter over its dispatches.  Usage: pmc_summary.py DIR [MODE]"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
mode = sys.argv[2] if len(sys.argv) > 2 else "nearest"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, f"p*_{mode}", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = k.replace("rtbvh::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    if not k.startswith(("k_", "rtbvh")):
        continue
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
print(json.dumps(out, indent=1))
