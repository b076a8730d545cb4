#!/usr/bin/env python3
"""The rebuilt C5 frame (rtbvh_compute_bvh: build + binned primary + 1 bounce, synchronous), wall clock
per frame over AB_FRAMES frames after 3 warm-ups, AB_ROUNDS rounds; the frame's SHA-1.  A/B of library
builds via RTBVH_LIB (scripts/ab_libs.sh AB_SCRIPT=ab_rebuild.py)."""
import hashlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import raytracebvh_amd as rt  # noqa: E402

W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
flags = (rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
         | rt.FLAG_BINNED_PRIMARY | int(os.environ.get("AB_FLAGS", "0"), 0))
n = int(os.environ.get("AB_FRAMES", "20"))
res = []
with rt.Context(device=0, flags=flags) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    for _ in range(3):
        c.compute_bvh(W, H, 1)
    for _ in range(int(os.environ.get("AB_ROUNDS", "3"))):
        t0 = time.perf_counter()
        for _ in range(n):
            c.compute_bvh(W, H, 1)
        res.append((time.perf_counter() - t0) / n * 1e3)
    sha = hashlib.sha1(c.read_framebuffer().tobytes()).hexdigest()[:16]
print(json.dumps({"lib": os.path.basename(os.environ.get("RTBVH_LIB", "librtbvh.so")), "ms_med": round(statistics.median(res), 4),
                  "ms": [round(x, 4) for x in res], "frame_sha1": sha}))
