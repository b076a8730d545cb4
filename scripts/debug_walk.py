#!/usr/bin/env python3
"""One C5 bounce ray's walk, step by step (a RTBVH_DEBUG_PIXEL build prints them from the COUNT kernel),
in the certified and the unchecked 4-wide walks.  RTBVH_LIB = that build:
  make -C raytracebvh_amd/csrc OUT=../librtbvh_dbg.so OBJDIR=../../build/obj_dbg EXTRA="-DRTBVH_AB_BUILD -DRTBVH_DEBUG_PIXEL=<pixel>"
(the pixel from stats trav_longest, scripts/longest_walk.py; profiles/r04_n_longest_walk_debug.log)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import raytracebvh_amd as rt  # noqa: E402

W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
ctx = rt.Context(device=0, flags=rt.FLAG_WIDE_BVH)
ctx.set_scene(scene)
ctx.set_camera(*rt.camera_reference(W, H))
ctx.build()
binned = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH | rt.FLAG_BINNED_PRIMARY
for fl in (binned, rt.FLAG_CERTIFIED):
    ctx.set_flags(fl | rt.FLAG_COUNT_VISITS)
    ctx.trace(W, H, 1)
    print("trav_longest", ctx.stats()["trav_longest"] >> 32, flush=True)
