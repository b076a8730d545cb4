#!/usr/bin/env python3
"""Frames in flight, on ONE GPU: rank 0's bands of the C5 frame split over N ranks, traced K
times back to back on one context, frame i on caller stream i % F (F = 1, 2, 3 frames in
flight; the context gives each stream its own trace-buffer slot over the one BVH).  Prints
host-clock ms per frame.  Usage: python scripts/inflight_sim.py [K]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
flags = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
torch.cuda.set_device(0)
streams = [torch.cuda.Stream() for _ in range(3)]
out = {}
with rt.Context(device=0, flags=flags, stream=streams[0].cuda_stream) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(3)]
    torch.cuda.synchronize()
    for N in (1, 2, 4, 8):
        c.set_flags(flags)
        row = {}
        for F in (1, 2, 3):
            def frames(n):
                for i in range(n):
                    k = i % F
                    c.trace_band_async(W, H, 1, 0, N, bufs[k].data_ptr(), stream_ptr=streams[k].cuda_stream)
            frames(4)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            frames(K)
            torch.cuda.synchronize()
            row[f"ms_per_frame_{F}_in_flight"] = round((time.perf_counter() - t0) / K * 1e3, 4)
        out[f"N{N}_rank0"] = row
print(json.dumps(out))
