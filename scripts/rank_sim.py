#!/usr/bin/env python3
"""Per-rank trace time of the C5 frame split over N ranks, on ONE GPU.

bench.py's N-GPU step is max over ranks of (trace of the rank's bands) + the RCCL band
gather.  The trace part does not need N devices: every rank's bands can be traced one
after another on a single GPU with the same kernels.  This prints, for N = 1, 2, 4, 8,
each rank's trace time (the context's HIP events, mean of K) and the predicted compute-only speed-up
max-rank(N=1) / max-rank(N).  The gather is not included (one GPU has no xGMI peer).
Usage: python scripts/rank_sim.py [K]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402
from raytracebvh_amd.tiles import band_row_ids  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
flags = rt.FLAG_TIMING | rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
out = {}
torch.cuda.set_device(0)
stream = torch.cuda.current_stream()
with rt.Context(device=0, flags=flags, stream=stream.cuda_stream) as ctx:
    ctx.set_scene(scene)
    ctx.set_camera(*rt.camera_reference(W, H))
    ctx.build()
    buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    only = os.environ.get("RANK_SIM_ONLY")   # "N,r": trace just that rank's bands (profiling)
    if only:
        N, r = (int(x) for x in only.split(","))
        for _ in range(K):
            ctx.trace_band_async(W, H, 1, r, N, buf.data_ptr())
        ctx.synchronize()
        print(json.dumps({"only": [N, r], "ms_trace": ctx.stats()["ms_trace"]}))
        sys.exit(0)
    splits = [int(x) for x in os.environ.get("RANK_SIM_SPLITS", "0").split(",")]
    Ns = [int(x) for x in os.environ.get("RANK_SIM_N", "1,2,4,8").split(",")]
    for N, sp in ((N, sp) for sp in splits for N in Ns):
        ctx.set_flags(flags | sp << rt.FLAG_SPLIT_SHIFT)
        per, stages = [], []
        for r in range(N):
            for _ in range(2):
                ctx.trace_band_async(W, H, 1, r, N, buf.data_ptr())
            ctx.synchronize()
            ctx.reset_stats()
            for _ in range(K):   # context HIP events: primary, bounce traversal, whole trace
                ctx.trace_band_async(W, H, 1, r, N, buf.data_ptr())
            ctx.synchronize()
            st = ctx.stats()
            per.append(round(st["ms_trace"], 4))
            stages.append([round(st["ms_stage"][5], 4), round(st["ms_stage"][7], 4),
                           round(st["ms_stage"][6] - st["ms_stage"][7], 4)])
            if r == 0:   # back-to-back frames, host clock (launch overhead included)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(K):
                    ctx.trace_band_async(W, H, 1, r, N, buf.data_ptr())
                torch.cuda.synchronize()
                wall0 = (time.perf_counter() - t0) / K * 1e3
        out[f"N{N}_split{sp}"] = {"rank_ms": per, "max_ms": max(per), "rank0_wall_ms": round(wall0, 4),
                  "stages_primary_trav_shade": stages,
                  "rows": len(band_row_ids(H, 0, N))}
    for key in out:
        k1 = "N1_split" + key.split("_split")[1]
        if k1 in out:
            out[key]["speedup_compute_only"] = round(out[k1]["max_ms"] / out[key]["max_ms"], 3)
print(json.dumps(out))
