#!/usr/bin/env python3
"""Build the C5 scene's BVH BUILD_ITERS times (for rocprofv3 --kernel-trace --stats of the
build kernels alone); prints the hipEvent stage times."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracebvh_amd as rt  # noqa: E402

scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
with rt.Context(device=0, flags=rt.FLAG_TIMING) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(3840, 2160))
    c.build()
    c.reset_stats()
    for _ in range(int(os.environ.get("BUILD_ITERS", "10"))):
        c.build(sync=False)
    c.synchronize()
    st = c.stats()
    print(json.dumps({"ms_build": st["ms_build"], "stages": st["ms_stage"][:5]}))
