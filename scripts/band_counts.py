#!/usr/bin/env python3
"""Visit counts of rank 0's bands of the C5 frame for N = 1, 2, 3, 4, 8 ranks (one context, the
band trace of rtbvh_trace_band_async): a rank's share of the counts should be about 1/N."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
flags = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
out = {}
with rt.Context(device=0, flags=flags | rt.FLAG_COUNT_VISITS) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    for n in (1, 2, 3, 4, 8):
        for rank in sorted({0, n - 1}):
            c.trace_band_async(W, H, 1, rank, n, buf.data_ptr())
            st = c.stats()
            out[f"N{n}_r{rank}"] = {"packet_steps": st["packet_steps"], "internal": st["internal_visits"],
                                    "primary_rays": st["primary_rays"], "bounce_rays": st["bounce_rays"]}
print(json.dumps(out))
