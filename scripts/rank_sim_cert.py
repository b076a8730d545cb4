#!/usr/bin/env python3
"""Per-rank trace time of the C5 frame split over N ranks, on ONE GPU, in the bench's configuration: the
certified walks (RTBVH_FLAG_CERTIFIED, the headline mode), the bench's band deal (root_share 16 at N <= 2,
15 at N <= 4, 13 above), F frames in flight (argv 2, default 4: frame i on caller stream i % F, a trace-buffer slot each),
and one frame at a time.  Every rank's bands are traced one rank after another with the same kernels, so
this is the compute part of bench.py's N-GPU step (the RCCL gather and rank 0's assembly are not in it:
one GPU has no xGMI peer).  Prints one JSON line: per N, each rank's ms per frame (host clock over K
frames in flight; context events one frame at a time) and the compute-only speed-up max(N=1) / max(N).
Usage: python scripts/rank_sim_cert.py [K] [F] [N list, e.g. 1,8]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
F = int(sys.argv[2]) if len(sys.argv) > 2 else 4   # frames in flight
NS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8]
W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
torch.cuda.set_device(0)
streams = [torch.cuda.Stream() for _ in range(F)]
out = {}
with rt.Context(device=0, flags=rt.FLAG_CERTIFIED | rt.FLAG_TIMING, stream=streams[0].cuda_stream) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(F)]
    torch.cuda.synchronize()
    for N in NS:
        share = 16 if N <= 2 else 15 if N <= 4 else 13
        c.set_band_deal(share)
        inflight, one = [], []
        for r in range(N):
            def frames(n, f):
                for i in range(n):
                    k = i % f
                    c.trace_band_async(W, H, 1, r, N, bufs[k].data_ptr(), stream_ptr=streams[k].cuda_stream)
            frames(2 * F, F)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            frames(K, F)
            torch.cuda.synchronize()
            inflight.append(round((time.perf_counter() - t0) / K * 1e3, 4))
            c.reset_stats()   # one frame at a time on the context stream: its HIP events
            for _ in range(K // 2):
                c.trace_band_async(W, H, 1, r, N, bufs[0].data_ptr())
            c.synchronize()
            one.append(round(c.stats()["ms_trace"], 4))
        out[f"N{N}"] = {"root_share": share, "rank_ms_in_flight": inflight, "frames_in_flight": F, "rank_ms_one_frame": one,
                        "max_ms_in_flight": max(inflight), "max_ms_one_frame": max(one)}
    for key, v in out.items():
        if "N1" in out:
            v["speedup_compute_only_in_flight"] = round(out["N1"]["max_ms_in_flight"] / v["max_ms_in_flight"], 3)
            v["speedup_compute_only_one_frame"] = round(out["N1"]["max_ms_one_frame"] / v["max_ms_one_frame"], 3)
print(json.dumps(out))
