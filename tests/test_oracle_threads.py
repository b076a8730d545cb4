"""The oracle's row-parallel trace (the all-cores CPU baseline) equals its single-thread trace."""
import numpy as np

import raytracebvh_amd as rt
from oracle import lib as orc


def test_threaded_trace_equals_single_thread():
    s = rt.synthetic(20_000, seed=5, half_extent=(30, 30, 20))
    osc = orc.Scene(s.vertices, s.indices, s.mat_indices, s.material_blob)
    wvp, wv = rt.camera_reference(160, 97)
    nodes = orc.build(osc, wvp)
    out = []
    for th in (1, 4):
        orc.set_threads(th)
        try:
            out.append(orc.trace(osc, nodes, wvp, wv, 160, 97, 2, 3, 97, 2, want_intensity=True))
        finally:
            orc.set_threads(1)
    (fb1, in1, st1), (fb4, in4, st4) = out
    assert np.array_equal(fb1, fb4) and np.array_equal(in1, in4) and st1 == st4
    assert st1["hits"] > 0
