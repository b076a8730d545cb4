#!/usr/bin/env python3
"""Build timing on the C4 scene (10M synthetic triangles, seed 0x5EED0004): per-stage hipEvent
averages of ITERS builds (RTBVH_FLAG_TIMING).  A/B of library builds via RTBVH_LIB."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: F401  (the HIP runtime torch loads; see raytracebvh_amd/_lib.py)
import raytracebvh_amd as rt

iters = int(os.environ.get("ITERS", "20"))
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
scene_name = os.environ.get("SCENE", "c4")   # c4 | Test | Image_Test | Rect (tests/golden/scenes)
if scene_name == "c4":
    s = rt.synthetic(10_000_000, seed=0x5EED0004, half_extent=(50.0, 50.0, 50.0))
else:
    s = rt.load_npz(os.path.join(REPO, "tests", "golden", "scenes", scene_name + ".npz"))
extra = int(os.environ.get("BUILD_FLAGS", "0"), 0)
wvp, wv = rt.camera_reference(1920, 1080)
out = []
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    with rt.Context(device=0, flags=rt.FLAG_TIMING | extra) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.build()
        c.reset_stats()
        for _ in range(iters):
            c.build(sync=False)
        c.synchronize()
        st = c.stats()
    out.append([round(x, 4) for x in st["ms_stage"][:5]])
print(json.dumps({"lib": os.path.basename(os.environ.get("RTBVH_LIB", "librtbvh.so")), "scene": scene_name,
                  "flags": extra, "stages_ms": out,
                  "total_ms": [round(sum(x), 4) for x in out]}))
