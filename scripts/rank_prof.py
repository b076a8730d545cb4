#!/usr/bin/env python3
"""One rank's share of the C5 frame (certified walks, the bench's band deal) traced K times, for a per-kernel
profile under rocprofv3 --kernel-trace --stats: what a rank at N GPUs spends per frame beside its bands' rays.
Usage: python scripts/rank_prof.py N RANK K [inflight F]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

N, R, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
F = int(sys.argv[5]) if len(sys.argv) > 5 and sys.argv[4] == "inflight" else 1
W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
torch.cuda.set_device(0)
streams = [torch.cuda.Stream() for _ in range(max(F, 1))]
with rt.Context(device=0, flags=rt.FLAG_CERTIFIED | rt.FLAG_TIMING, stream=streams[0].cuda_stream) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    c.set_band_deal(16 if N <= 2 else 15 if N <= 4 else 13)
    bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(F)]
    for i in range(2 * F):
        c.trace_band_async(W, H, 1, R, N, bufs[i % F].data_ptr(), stream_ptr=streams[i % F].cuda_stream if F > 1 else 0)
    torch.cuda.synchronize()
    c.reset_stats()
    t0 = time.perf_counter()
    for i in range(K):
        c.trace_band_async(W, H, 1, R, N, bufs[i % F].data_ptr(), stream_ptr=streams[i % F].cuda_stream if F > 1 else 0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    st = c.stats()
    print(json.dumps({"N": N, "rank": R, "frames_in_flight": F, "ms_per_frame_host": round(dt * 1e3, 4),
                      "ms_trace_events": st["ms_trace"], "ms_stage": st["ms_stage"],
                      "primary_rays": st["primary_rays"], "bounce_rays": st["bounce_rays"]}))
