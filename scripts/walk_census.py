#!/usr/bin/env python3
"""Walk-length census of the C5 bounce pass (RTBVH_FLAG_COUNT_VISITS): the longest bounce
ray's loop iterations and the log2 histogram of walk lengths, for the whole frame (N=1)
and for rank 0's bands of N=8, in the bench's traversal modes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
FAST = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST
modes = {"nearest-first-wide": FAST | rt.FLAG_WIDE_BVH, "nearest-first": FAST}
out = {}
with rt.Context(device=0, flags=FAST) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    for name, fl in modes.items():
        for N in (1, 8):
            c.set_flags(fl | rt.FLAG_COUNT_VISITS)
            c.trace_band_async(W, H, 1, 0, N, buf.data_ptr())
            c.synchronize()
            st = c.stats()
            hist = st["trav_steps_log2"]
            n = sum(hist)
            out[f"{name}_N{N}"] = {
                "bounce_rays": st["bounce_rays"], "max_steps": st["trav_max_steps"],
                "mean_steps": round((st["internal_visits"][1] + st["leaf_visits"][1]) / max(1, n), 2),
                "internal_visits": st["internal_visits"][1], "leaf_visits": st["leaf_visits"][1],
                "log2_hist": {f"{1 << k}-{(2 << k) - 1}": v for k, v in enumerate(hist) if v},
                "lane_util": round(st["trav_active_lanes"] / max(1, 64 * st["trav_wave_steps"]), 4)}
print(json.dumps(out))
