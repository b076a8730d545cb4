#!/usr/bin/env python3
"""C2 (Obj/Image_Test.obj, 3072 triangles, 1920x1080 primary rays) rebuilt every frame, as bench.py's c2_frame:
the build through the one-workgroup Morton + sort (build.hip k_morton_sort_small, the default for 2048 < T <=
8192) against the multi-kernel build (RTBVH_FLAG_MULTI_KERNEL_BUILD: the Morton launch and the radix sort's
twelve), interleaved; each with and without RTBVH_FLAG_GRAPH.  Prints one JSON line per round and variant:
the build's stage times (HIP events) and the wall time per rebuilt frame; and checks the trees are identical."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
scene = rt.load_npz(os.path.join(REPO, "tests", "golden", "scenes", "Image_Test.npz"))
W, H, B = 1920, 1080, 0
trees = {}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for name, fl in (("one_workgroup_sort", 0), ("multi_kernel", rt.FLAG_MULTI_KERNEL_BUILD)):
        out = {"round": rnd, "variant": name, "triangles": scene.num_tris}
        with rt.Context(device=0, flags=fl | rt.FLAG_TIMING) as c:
            c.set_scene(scene)
            c.set_camera(*rt.camera_reference(W, H))
            c.compute_bvh(W, H, B)
            c.reset_stats()
            t0 = time.perf_counter()
            for _ in range(50):
                c.compute_bvh(W, H, B)
            out["ms_frame"] = round((time.perf_counter() - t0) / 50 * 1e3, 4)
            q = c.stats()
            out["ms_build"] = round(q["ms_build"], 4)
            out["ms_stage"] = [round(x, 4) for x in q["ms_stage"][:5]]
            out["ms_trace"] = round(q["ms_trace"], 4)
            trees[name] = c.read_bvh()
        with rt.Context(device=0, flags=fl | rt.FLAG_GRAPH) as c:
            c.set_scene(scene)
            c.set_camera(*rt.camera_reference(W, H))
            c.compute_bvh(W, H, B)   # capture
            t0 = time.perf_counter()
            for _ in range(50):
                c.compute_bvh(W, H, B)
            out["ms_frame_graph"] = round((time.perf_counter() - t0) / 50 * 1e3, 4)
        print(json.dumps(out), flush=True)
a, b = trees["one_workgroup_sort"], trees["multi_kernel"]
print(json.dumps({"trees_identical": bool(a.tobytes() == b.tobytes())}))
