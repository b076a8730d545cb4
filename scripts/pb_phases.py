#!/usr/bin/env python3
"""Phase split of k_primary_binned (a RTBVH_PB_PROF build: make OUT=../librtbvh_prof.so EXTRA=-DRTBVH_PB_PROF,
loaded with RTBVH_LIB): shader-clock cycles per phase summed over the waves, C5 frame."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracebvh_amd as rt  # noqa: E402
W, H = 3840, 2160
scene = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
base = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH | rt.FLAG_BINNED_PRIMARY
with rt.Context(device=0, flags=base) as c:
    c.set_scene(scene)
    c.set_camera(*rt.camera_reference(W, H))
    c.build()
    for _ in range(3):
        c.trace(W, H, 0)
    st = c.stats()
names = ["batch loads", "coarse + survivor gather", "-", "fine", "flush (tests)", "block maxima", "epilogue", "init"]
ph = [int(x) for x in st["trav_steps_log2"][:8]]
tot = sum(ph)
print(json.dumps({n: round(v / tot, 4) for n, v in zip(names, ph)}))
print(json.dumps({"cycles_per_wave": round(tot / 32640, 1)}))
