#!/usr/bin/env python3
"""The reference's per-frame semantics at C5 (Graphics.cpp:56, 667-831): rebuild the BVH and
trace primary + 1 bounce every frame, synchronously (rtbvh_compute_bvh), in the bench's mode.
Run under `rocprofv3 --kernel-trace` for the frame's timeline (scripts/frame_timeline.py).
FRAME_FLAGS: extra RTBVH_FLAG_* bits (e.g. the graph flag); FRAMES: frames after 2 warm-ups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracebvh_amd as rt  # noqa: E402

flags = (rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH | rt.FLAG_BINNED_PRIMARY
         | int(os.environ.get("FRAME_FLAGS", "0"), 0))
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
W, H = 3840, 2160
with rt.Context(device=0, flags=flags) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    for _ in range(2 + int(os.environ.get("FRAMES", "5"))):
        c.compute_bvh(W, H, 1)
print("done")
