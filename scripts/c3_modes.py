#!/usr/bin/env python3
"""C3 (Obj/Test.obj, 1952 triangles, 1920x1080, primary + 1 bounce; SCENE / BOUNCES for others) rebuilt every frame as one hipGraph under
several walk configurations, interleaved: the wall time per frame, the stage times of a timed run, and whether
the frame equals the reference order's.  Prints one JSON line per round and configuration."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
scene = rt.load_npz(os.path.join(REPO, "tests", "golden", "scenes", os.environ.get("SCENE", "Test") + ".npz"))
W, H, B = 1920, 1080, int(os.environ.get("BOUNCES", "1"))
CFG = {"auto": rt.FLAG_AUTO_WALK, "certified": rt.FLAG_CERTIFIED,
       "binned": rt.FLAG_BINNED_PRIMARY, "binned+refill": rt.FLAG_BINNED_PRIMARY | rt.FLAG_REFILL_BOUNCE,
       "packet": rt.FLAG_PACKET_PRIMARY}
if os.environ.get("CONFIGS"):
    CFG = {k: v for k, v in CFG.items() if k in os.environ["CONFIGS"].split(",")}
ref = None
with rt.Context(device=0, flags=0) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.compute_bvh(W, H, B)
    ref = c.read_framebuffer()
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for name, fl in CFG.items():
        out = {"round": rnd, "config": name}
        with rt.Context(device=0, flags=fl | rt.FLAG_GRAPH) as c:
            c.set_scene(scene)
            c.set_camera(*rt.camera_reference(W, H))
            c.compute_bvh(W, H, B)
            t0 = time.perf_counter()
            for _ in range(50):
                c.compute_bvh(W, H, B)
            out["ms_frame_graph"] = round((time.perf_counter() - t0) / 50 * 1e3, 4)
            out["frame_equal_reference"] = bool(np.array_equal(c.read_framebuffer(), ref))
        with rt.Context(device=0, flags=fl | rt.FLAG_TIMING) as c:
            c.set_scene(scene)
            c.set_camera(*rt.camera_reference(W, H))
            for _ in range(10):
                c.compute_bvh(W, H, B)
            q = c.stats()
            out["ms_build"] = round(q["ms_build"], 4)
            out["ms_trace"] = round(q["ms_trace"], 4)
            out["ms_stage"] = [round(x, 4) for x in q["ms_stage"]]
            out["walk_state"] = q["walk_state"]
            out["walk_flags"] = q["walk_flags"]
            out["redo_rays"] = q["redo_rays"]
        print(json.dumps(out), flush=True)
