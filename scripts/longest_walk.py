#!/usr/bin/env python3
"""The longest bounce walk of the C5 frame in the certified and the unchecked 4-wide walks
(stats trav_longest: iterations and pixel), and that pixel's bounce ray (the reflectRay record of
a primary-only trace: origin = the primary hit, direction = the reflection).  Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402


def main():
    W, H = 3840, 2160
    scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    ctx = rt.Context(device=0, flags=rt.FLAG_WIDE_BVH)
    ctx.set_scene(scene)
    ctx.set_camera(*rt.camera_reference(W, H))
    ctx.build()
    binned = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH | \
        rt.FLAG_BINNED_PRIMARY
    pix = {}
    for name, fl in (("binned", binned), ("certified", rt.FLAG_CERTIFIED)):
        ctx.set_flags(fl | rt.FLAG_COUNT_VISITS)
        ctx.trace(W, H, 1)
        st = ctx.stats()
        v = int(st["trav_longest"])
        pix[name] = v & 0xFFFFFFFF
        print(json.dumps({"walk": name, "longest_iterations": v >> 32, "pixel": v & 0xFFFFFFFF,
                          "x": (v & 0xFFFFFFFF) % W, "y": (v & 0xFFFFFFFF) // W,
                          "trav_max_steps": st["trav_max_steps"]}), flush=True)
    # the bounce rays: reflectRay records of a primary-only trace
    ctx.set_flags(binned | rt.FLAG_REFRACT_RECORDS)
    ctx.trace(W, H, 0)
    refl, _ = ctx.read_rays()
    rec = refl.reshape(-1, 14)
    # and the bounce pass's hit distance: the certified frame's bounce hit record is not exported, so
    # report the ray and let the CPU side reason about it
    for name, p in pix.items():
        r = rec[p]
        d = r[4:7]
        print(json.dumps({"walk": name, "pixel": p, "intensity": float(r[0]), "origin": [float(x) for x in r[1:4]],
                          "direction": [float(x) for x in d], "abs_dir_min": float(np.min(np.abs(d))),
                          "dot_dd": float(np.dot(d, d))}), flush=True)


if __name__ == "__main__":
    main()
