#!/usr/bin/env python3
"""One process, one GPU: rank r's bands of the C5 frame (N ranks) in the bench's three
traversal modes, switching modes on two contexts as bench.py does, each frame compared
with the reference-order band traced alone.  Prints differing pixel counts per mode."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
FAST = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE
modes = {"reference-order": FAST, "nearest-first": FAST | rt.FLAG_NEAREST_FIRST,
         "nearest-first-wide": FAST | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH}
torch.cuda.set_device(0)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
ctxs = []
for s in streams:
    c = rt.Context(device=0, flags=FAST, stream=s.cuda_stream)
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    ctxs.append(c)
out = {}
for N, r in ((1, 0), (2, 1), (3, 1), (3, 2)):
    ref = torch.zeros((H, W, 4), device="cuda:0")
    torch.cuda.synchronize()
    ctxs[0].set_flags(modes["reference-order"])
    ctxs[0].trace_band_async(W, H, 1, r, N, ref.data_ptr())
    ctxs[0].synchronize()
    row = {}
    for name, fl in modes.items():
        for c in ctxs:
            c.set_flags(fl)
        bufs = [torch.zeros((H, W, 4), device="cuda:0") for _ in range(K)]
        torch.cuda.synchronize()
        for i in range(K):
            ctxs[i % 2].trace_band_async(W, H, 1, r, N, bufs[i].data_ptr())
        torch.cuda.synchronize()
        row[name] = [int((b != ref).any(dim=2).sum()) for b in bufs]
    out[f"N{N}_r{r}"] = row
print(json.dumps(out))
