#!/usr/bin/env python3
"""Frames in flight, on ONE GPU: rank r's bands of the C5 frame split over N ranks, traced K
times back to back (a) on one context and stream, (b) alternating over two contexts (two
BVH replicas built from the same inputs) on two streams, so that frame i+1's primary pass
can start while frame i's bounce walk drains.  Prints host-clock ms per frame for each.
Usage: python scripts/inflight_sim.py [K]"""
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
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
ctxs = []
for s in streams:
    c = rt.Context(device=0, flags=flags, stream=s.cuda_stream)
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    ctxs.append(c)
torch.cuda.synchronize()
bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(2)]
out = {}
for N in (1, 2, 4, 8):
    row = {}
    for nctx in (1, 2):
        def frames(n):
            for i in range(n):
                k = i % nctx
                ctxs[k].trace_band_async(W, H, 1, 0, N, bufs[k].data_ptr())
        frames(4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frames(K)
        torch.cuda.synchronize()
        row[f"ms_per_frame_{nctx}ctx"] = round((time.perf_counter() - t0) / K * 1e3, 4)
    out[f"N{N}_rank0"] = row
same = torch.equal(bufs[0], bufs[1])
print(json.dumps({"frames": out, "buffers_identical": same}))
for c in ctxs:
    c.close()
