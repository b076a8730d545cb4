#!/usr/bin/env python3
"""C3 (Obj/Test.obj, 1920x1080, primary + 1 bounce) frames as the bench's c3_1080p line runs them --
rtbvh_compute_bvh per frame under RTBVH_FLAG_AUTO_WALK (| RTBVH_FLAG_GRAPH with C3_GRAPH=1) -- for a
rocprofv3 kernel trace of the small-scene path; prints the wall time per frame and the stage times."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import raytracebvh_amd as rt  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    W, H = 1920, 1080
    graph = os.environ.get("C3_GRAPH", "1") == "1"
    # C3_MODE: the walks (default AUTO_WALK: the reference order's plain kernels at this size); "fast": the
    # reference order's packet primary + refill bounce kernels; "certified": the certified fast walks
    walk = {"auto": rt.FLAG_AUTO_WALK, "fast": rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE,
            "certified": rt.FLAG_CERTIFIED, "plain": 0, "sort": rt.FLAG_SORT_BOUNCE,
            "packet+sort": rt.FLAG_PACKET_PRIMARY | rt.FLAG_SORT_BOUNCE}[os.environ.get("C3_MODE", "auto")]
    # C3_SCENE=Image_Test C3_BOUNCES=0: C2
    scene = rt.load_npz(os.path.join(REPO, "tests", "golden", "scenes", os.environ.get("C3_SCENE", "Test") + ".npz"))
    B = int(os.environ.get("C3_BOUNCES", "1"))
    flags = walk | (rt.FLAG_GRAPH if graph else 0)
    with rt.Context(device=0, flags=flags) as ctx:
        ctx.set_scene(scene)
        ctx.set_camera(*rt.camera_reference(W, H))
        for _ in range(3):
            ctx.compute_bvh(W, H, B)
        n = int(os.environ.get("C3_FRAMES", "50"))
        t0 = time.perf_counter()
        for _ in range(n):
            ctx.compute_bvh(W, H, B)
        dt = (time.perf_counter() - t0) / n
        st = ctx.stats()
        ctx.set_flags(walk | rt.FLAG_TIMING)
        ctx.reset_stats()
        for _ in range(10):
            ctx.compute_bvh(W, H, B)
        ts = ctx.stats()
        fb = ctx.read_framebuffer()
        print(json.dumps({"mode": os.environ.get("C3_MODE", "auto"), "scene": os.environ.get("C3_SCENE", "Test"),
                          "walk_flags": st["walk_flags"], "graph": graph, "ms_per_frame": round(dt * 1e3, 4),
                          "frame_sha1": __import__("hashlib").sha1(fb.tobytes()).hexdigest()[:16],
                          "mrays_s": round((st["primary_rays"] + st["bounce_rays"]) / dt / 1e6, 1),
                          "ms_build": round(ts["ms_build"], 4), "ms_trace": round(ts["ms_trace"], 4),
                          "ms_stage": [round(x, 4) for x in ts["ms_stage"]], "walk_state": st["walk_state"]}))


if __name__ == "__main__":
    main()
