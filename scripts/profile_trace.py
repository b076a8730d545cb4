#!/usr/bin/env python3
"""Small driver for rocprofv3 runs: builds the C5 scene once and runs a few
builds + traces in the requested mode (PROF_COMPUTE=1: rtbvh_compute_bvh frames).  PROF_MODE is a '+'-joined list of
reference | nearest | sort | packet | refill | wide | count (e.g. "nearest+packet")."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracebvh_amd as rt  # noqa: E402

mode = os.environ.get("PROF_MODE", "nearest")
names = {"reference": 0, "nearest": rt.FLAG_NEAREST_FIRST, "sort": rt.FLAG_SORT_BOUNCE,
         "packet": rt.FLAG_PACKET_PRIMARY, "count": rt.FLAG_COUNT_VISITS, "refill": rt.FLAG_REFILL_BOUNCE,
         "wide": rt.FLAG_WIDE_BVH, "binned": rt.FLAG_BINNED_PRIMARY, "certified": rt.FLAG_CERTIFIED,
         "auto": rt.FLAG_AUTO_WALK}
flags = 0
for m in mode.split("+"):
    flags |= names[m]
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
W, H = 3840, 2160
with rt.Context(device=0, flags=flags) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    for _ in range(int(os.environ.get("PROF_ITERS", "3"))):
        if os.environ.get("PROF_COMPUTE"):   # the drop-in's frame: rtbvh_compute_bvh (build + trace, one call)
            c.compute_bvh(W, H, 1)
            continue
        c.build()
        c.trace(W, H, 1)
    if flags & rt.FLAG_COUNT_VISITS:
        print(c.stats())
    out = os.environ.get("PROF_COUNTS")   # one more trace with visit counts (run this outside rocprofv3)
    if out:
        import json
        c.set_flags(flags | rt.FLAG_COUNT_VISITS)
        c.trace(W, H, 1)
        json.dump(c.stats(), open(out, "w"))
print("done", mode)
