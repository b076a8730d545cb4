#!/usr/bin/env python3
"""Probe (round 6, RTBVH_TAIL_PROBE library via RTBVH_LIB): when the certified bounce walk's waves end, in 100-us
buckets from their start (one C5 frame at a time, then four frames' worth), from rtbvh_stats.trav_steps_log2."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: F401
import raytracebvh_amd as rt

s = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
W, H = 3840, 2160
with rt.Context(device=0, flags=rt.FLAG_CERTIFIED | rt.FLAG_TIMING) as c:
    c.set_scene(s)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    for it in range(3):
        c.trace(W, H, 1)
        st = c.stats()
        h = list(st["trav_steps_log2"])
        print(json.dumps({"trace": it, "bounce_trav_ms": round(st["ms_stage"][7], 4), "wave_end_100us": h}), flush=True)
