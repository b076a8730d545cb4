#!/usr/bin/env python3
"""Probe (round 6): the C4 build of the same scene with its triangles (and vertices, by first use) in their
Morton order against the generator's order -- the locality the refit's sorted-order gather of clip records
would get if the scene were renumbered once at rtbvh_set_scene.  Per-stage hipEvent times, interleaved."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: F401
import raytracebvh_amd as rt

iters = int(os.environ.get("ITERS", "20"))
s = rt.synthetic(10_000_000, seed=0x5EED0004, half_extent=(50.0, 50.0, 50.0))
wvp, wv = rt.camera_reference(1920, 1080)
flags = rt.FLAG_TIMING | int(os.environ.get("BUILD_FLAGS", "0"), 0)
with rt.Context(device=0, flags=flags) as c:
    c.set_scene(s)
    c.set_camera(wvp, wv)
    c.build()
    _, perm = c.read_sorted()
perm = np.asarray(perm, np.int64)
T = len(perm)
idx = s.indices.reshape(T, 3)[perm].ravel()
first = np.full(len(s.vertices), np.iinfo(np.int64).max, np.int64)
np.minimum.at(first, idx.astype(np.int64), np.arange(3 * T, dtype=np.int64))
vorder = np.argsort(first, kind="stable")
vnew = np.empty_like(vorder)
vnew[vorder] = np.arange(len(vorder))
s2 = rt.Scene(s.vertices[vorder], vnew[idx].astype(np.uint32), s.mat_indices[perm], s.materials)
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for name, sc in (("generator order", s), ("morton order", s2)):
        with rt.Context(device=0, flags=flags) as c:
            c.set_scene(sc)
            c.set_camera(wvp, wv)
            c.build()
            c.reset_stats()
            for _ in range(iters):
                c.build(sync=False)
            c.synchronize()
            st = c.stats()
            print(json.dumps({"scene": name, "flags": flags, "stages_ms": [round(x, 4) for x in st["ms_stage"][:5]],
                              "build_ms": round(sum(st["ms_stage"][:5]), 4)}), flush=True)
