#!/usr/bin/env python3
"""Determinism check of back-to-back and in-flight traces, one process, one GPU: for
rank r of N, the band frame traced alone (synchronised) vs (a) K frames back to back on
one context and (b) K frames alternating over two contexts on two streams; every
frame's band buffer is compared with the alone-traced one."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
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
out = {}
for N, r in ((1, 0), (3, 1), (3, 2), (8, 5)):
    rows = len(rt.band_row_ids(H, r, N)) if hasattr(rt, "band_row_ids") else None
    ref = torch.zeros((H, W, 4), device="cuda:0")
    torch.cuda.synchronize()   # torch's zero fill runs on its current stream, not the contexts'
    ctxs[0].trace_band_async(W, H, 1, r, N, ref.data_ptr())
    ctxs[0].synchronize()
    again = torch.zeros_like(ref)
    torch.cuda.synchronize()
    ctxs[1].trace_band_async(W, H, 1, r, N, again.data_ptr())
    ctxs[1].synchronize()
    res = {"ref_vs_alone_ctx1": int((again != ref).any(dim=2).sum())}
    for name, nctx in (("serial", 1), ("inflight", 2)):
        bufs = [torch.zeros((H, W, 4), device="cuda:0") for _ in range(K)]
        torch.cuda.synchronize()
        for i in range(K):
            k = i % nctx
            ctxs[k].trace_band_async(W, H, 1, r, N, bufs[i].data_ptr())
        torch.cuda.synchronize()
        diag = []
        for b in bufs:
            m = (b != ref).any(dim=2)
            nm = int(m.sum())
            if nm:
                d = (b - ref).abs().nan_to_num(0).amax(dim=2)[m]
                diag.append({"px": nm, "zero_px": int((b == 0).all(dim=2)[m].sum()),
                             "ref_zero_px": int((ref == 0).all(dim=2)[m].sum()),
                             "bounce_like_px": int(((d > 0.05) & (d < 0.06)).sum()), "max": float(d.max())})
            else:
                diag.append(0)
        res[name] = diag
    out[f"N{N}_r{r}"] = res
print(json.dumps(out))
