#!/usr/bin/env python3
"""A/B traversal walk flags (or, with AB_SET=base, two library builds via RTBVH_LIB) on the C5 frame in ONE process (interleaved
rounds, cdna_hip_programming.md §5.4 rule 24).  Every variant's framebuffer must
equal the baseline's bit for bit.  Prints one JSON line per variant."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402


def main():
    ntris = int(os.environ.get("AB_TRIS", "10000000"))
    W, H = int(os.environ.get("AB_W", "3840")), int(os.environ.get("AB_H", "2160"))
    rounds = int(os.environ.get("AB_ROUNDS", "5"))
    variants = [("reference+sort", rt.FLAG_SORT_BOUNCE), ("nearest", rt.FLAG_NEAREST_FIRST),
                ("nearest+packet", rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY),
                ("refill", rt.FLAG_REFILL_BOUNCE | rt.FLAG_PACKET_PRIMARY),
                ("refill+sort", rt.FLAG_REFILL_BOUNCE | rt.FLAG_PACKET_PRIMARY | rt.FLAG_SORT_BOUNCE),
                ("nearest+refill", rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE),
                ("nearest+refill+sort", rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE
                 | rt.FLAG_SORT_BOUNCE),
                ("nearest+wide", rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_WIDE_BVH),
                ("nearest+wide+sort", rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_WIDE_BVH
                 | rt.FLAG_SORT_BOUNCE)]
    if os.environ.get("AB_SET") == "sort":
        base = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
        variants = [("wide", base), ("wide + bounce sort", base | rt.FLAG_SORT_BOUNCE)]
    if os.environ.get("AB_SET") == "base":   # the bench's mode only (A/B of two builds via RTBVH_LIB)
        variants = [("nearest-first-wide", rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST
                     | rt.FLAG_WIDE_BVH)]
    if os.environ.get("AB_SET") == "split":   # one frame over 1 / 2 / 3 primary->bounce chains
        base = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
        variants = [(f"split {k}", base | (k << rt.FLAG_SPLIT_SHIFT)) for k in (1, 2, 3, 4)]
    if os.environ.get("AB_SET") == "wide":
        base = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE
        variants = [("nearest+refill", base | rt.FLAG_NEAREST_FIRST),
                    ("nearest+wide", base | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH),
                    ("wide (left-to-right packets)", base | rt.FLAG_WIDE_BVH)]
    if os.environ.get("AB_SET") == "binnedbase":   # the binned mode only (A/B of two builds via RTBVH_LIB)
        variants = [("binned", rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
                     | rt.FLAG_BINNED_PRIMARY)]
    if os.environ.get("AB_SET") == "certified":   # the certified walks (AUTO) against the same walks unchecked
        variants = [("binned", rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
                     | rt.FLAG_BINNED_PRIMARY), ("certified", rt.FLAG_CERTIFIED)]
    if os.environ.get("AB_SET") == "certbase":   # the certified mode only (A/B of two builds via RTBVH_LIB)
        variants = [("certified", rt.FLAG_CERTIFIED)]
    if os.environ.get("AB_SET") == "binned":   # primary pass: 4-wide packets vs screen-tile bins
        base = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH
        variants = [("nearest-first-wide", base), ("binned", base | rt.FLAG_BINNED_PRIMARY)]
    scene = rt.synthetic(ntris, seed=0x5EED0005, half_extent=(100, 100, 50))
    ctx = rt.Context(device=0, flags=rt.FLAG_TIMING | rt.FLAG_WIDE_BVH)
    ctx.set_scene(scene)
    ctx.set_camera(*rt.camera_reference(W, H))
    ctx.build()
    ref = None
    res = {v: [] for v in variants}
    for r in range(rounds):
        for v, srt in variants:
            flags = rt.FLAG_TIMING | srt
            ctx.set_flags(flags)
            ctx.trace(W, H, 1)   # warm
            ctx.reset_stats()
            for _ in range(3):
                ctx.trace(W, H, 1, sync=False)
            st = ctx.stats()
            res[(v, srt)].append((st["ms_stage"][5], st["ms_stage"][6], st["ms_trace"], st["ms_stage"][7]))
            if r == 0:
                fb = ctx.read_framebuffer()
                if ref is None:
                    ref = fb
                ndiff = int((fb != ref).any(axis=-1).sum())
                sha = hashlib.sha1(fb.tobytes()).hexdigest()[:16]   # compare across RTBVH_LIB builds
                print(json.dumps({"variant": v, "pixels_differing_from_first": ndiff, "frame_sha1": sha}), flush=True)
    if os.environ.get("AB_COUNTS"):   # visit counts of each variant (one counting trace)
        for v, srt in variants:
            ctx.set_flags(srt | rt.FLAG_COUNT_VISITS)
            ctx.trace(W, H, 1)
            st = ctx.stats()
            print(json.dumps({"variant": v, "packet_steps": list(st["packet_steps"]),
                              "internal_visits": list(st["internal_visits"]), "leaf_visits": list(st["leaf_visits"]),
                              "trav_wave_steps": st["trav_wave_steps"], "bin_entries": list(st["bin_entries"]),
                              "redo_rays": list(st["redo_rays"]), "trav_max_steps": st["trav_max_steps"],
                              "trav_steps_log2": list(st["trav_steps_log2"])}))
    for (v, srt), xs in res.items():
        a = np.array(xs)
        print(json.dumps({"variant": v, "primary_ms_med": float(np.median(a[:, 0])),
                          "bounce_ms_med": float(np.median(a[:, 1])), "trace_ms_med": float(np.median(a[:, 2])),
                          "trace_ms_min": float(a[:, 2].min()), "bounce_trav_ms_med": float(np.median(a[:, 3])),
                          "bounce_trav_ms_min": float(a[:, 3].min())}))


if __name__ == "__main__":
    main()
