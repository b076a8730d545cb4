#!/usr/bin/env python3
"""The C3 frame's bounce walks in the reference order, counted: the refill bounce kernel's census
(RTBVH_FLAG_REFILL_BOUNCE | RTBVH_FLAG_COUNT_VISITS: per-ray iterations as a log2 histogram, the
longest walk and its pixel) and the visits per ray of both passes.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import raytracebvh_amd as rt  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    W, H = 1920, 1080
    scene = rt.load_npz(os.path.join(REPO, "tests", "golden", "scenes", "Test.npz"))
    with rt.Context(device=0, flags=rt.FLAG_REFILL_BOUNCE | rt.FLAG_COUNT_VISITS) as ctx:
        ctx.set_scene(scene)
        ctx.set_camera(*rt.camera_reference(W, H))
        ctx.compute_bvh(W, H, 1)
        st = ctx.stats()
        v = int(st["trav_longest"])
        hist = [int(x) for x in st["trav_steps_log2"]]
        print(json.dumps({"primary_rays": st["primary_rays"], "bounce_rays": st["bounce_rays"],
                          "internal_visits": [int(x) for x in st["internal_visits"]],
                          "leaf_visits": [int(x) for x in st["leaf_visits"]],
                          "bounce_visits_per_ray": round((st["internal_visits"][1] + st["leaf_visits"][1]) / max(1, st["bounce_rays"]), 1),
                          "primary_visits_per_ray": round((st["internal_visits"][0] + st["leaf_visits"][0]) / max(1, st["primary_rays"]), 1),
                          "trav_max_steps": int(st["trav_max_steps"]), "longest_iterations": v >> 32,
                          "longest_pixel": [(v & 0xFFFFFFFF) % W, (v & 0xFFFFFFFF) // W],
                          "steps_log2_hist": hist[:16]}), flush=True)


if __name__ == "__main__":
    main()
