#!/usr/bin/env python3
"""(Test infrastructure: it runs the oracle.) Inputs for tools/collapse_study.cpp (a CPU study: the build's greedy 4-wide collapse against an
SAH-optimal one, counted by a nearest-first walk of bounce rays): the reference tree of a synthetic scene
(oracle build), its clip-space triangles in sorted-leaf order, and the oracle's reflection rays of one row
in ROW_STEP.  Usage: python tests/collapse_study_inputs.py OUTDIR [NTRIS] [ROW_STEP]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import raytracebvh_amd as rt  # noqa: E402
from oracle import lib as orc  # noqa: E402

out = sys.argv[1]
ntris = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
step = int(sys.argv[3]) if len(sys.argv) > 3 else 32
os.makedirs(out, exist_ok=True)
W, H = 3840, 2160
s = rt.synthetic(ntris, seed=0x5EED0005, half_extent=(100.0, 100.0, 50.0))
osk = orc.Scene(s.vertices, s.indices, s.mat_indices, s.material_blob)
wvp, wv = rt.camera_reference(W, H)
orc.set_threads(os.cpu_count() or 1)
nodes = orc.build(osk, wvp, sort_mode=0)
nodes.tofile(os.path.join(out, "nodes.bin"))
T = s.num_tris
M = np.asarray(wvp, np.float32).reshape(4, 4)
pos = np.asarray(s.vertices, np.float32)[:, :3]
clip = (pos[:, 0:1] * M[0] + pos[:, 1:2] * M[1] + pos[:, 2:3] * M[2] + M[3])[:, :3].astype(np.float32)
tri_of_leaf = nodes["index"][:T].astype(np.int64) // 3   # (the leaf index field: 3 x triangle, the index-buffer offset)
idx = np.asarray(s.indices, np.int64).reshape(-1, 3)[tri_of_leaf]
np.ascontiguousarray(clip[idx].reshape(T, 9), np.float32).tofile(os.path.join(out, "tris.bin"))
_, _, st, refl, _ = orc.trace(osk, nodes, wvp, wv, W, H, 1, row_step=step, want_records=True)
r = refl.reshape(-1, 14)
live = r[:, 0] > 0
rays = np.ascontiguousarray(r[live][:, 1:7], np.float32)
rays.tofile(os.path.join(out, "rays.bin"))
print({"T": T, "rays": len(rays), "oracle": st})
