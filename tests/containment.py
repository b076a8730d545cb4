"""A scene where the reference's left-first DFS and the fast walks disagree
(VERDICT r2 "what's missing" #3): containment of a hit in its leaf's slab interval fails.

Two triangles A (index 0) and B (index 1) lie in the plane z = C of clip space (the camera
is the identity) and both cover the primary ray of pixel PIXEL, o = (2, -0.5, 0), d = +z.
The slab test of either box enters at exactly C (RayTraceTraversal.hlsl:92-104: (C - 0) * 1),
while Moller-Trumbore (:41-86) rounds both hits BELOW the plane: t_B < t_A < C (found by
a float32 search of the kernel's arithmetic; ~29% of such coplanar hits round below).
The padding triangles sit far outside the frame and spread the mesh box, so A and B share
one Morton cell: equal codes, sorted by index, adjacent sibling leaves A then B.

 * findCollision (reference order): both boxes pass the parent's test (no hit yet), A is
   visited (best = t_A), B is popped without a box test and replaces it (t_B < t_A) -> B.
 * the 4-wide packet walk re-tests a leaf's own box at its leaf step with the current bound
   (trace.hip traverse_packet4): B's entry C > t_A prunes it -> A.
So the frames differ at PIXEL (A and B carry different materials), which is what
RTBVH_FLAG_AUTO_WALK's device check must catch.
"""
import numpy as np

from raytracebvh_amd import _lib as _L
from raytracebvh_amd.scene import Scene

C = np.float32(25.37)
A = [(-0.5961761474609375, -1.2991570234298706), (4.6817474365234375, -0.48693186044692993),
     (2.3431427478790283, 0.1366989016532898)]
B = [(4.04730749130249, 1.4174126386642456), (-0.8829755783081055, -3.043396234512329),
     (0.7036949396133423, -1.961896538734436)]
W, H = 64, 64
PIXEL = (40, 30)   # o = ((40 - 32) / 4, (30 - 32) / 4, 0) = (2, -0.5, 0)


def identity_camera():
    eye = np.eye(4, dtype=np.float32).ravel()
    return eye, eye.copy()


def containment_scene(npad: int = 70_000, seed: int = 3) -> Scene:
    """A and B (+ npad small padding triangles at x in [5e4, 1e5], y, z in [-1e5, 1e5], never
    in the 64 x 64 frame's rays: |x| <= 8, |y| <= 8).  npad > 65536 puts the scene above
    RTBVH_FLAG_AUTO_WALK's reference-order size."""
    rng = np.random.default_rng(seed)
    verts = []
    for tri in (A, B):
        for x, y in tri:
            verts.append((x, y, C, 0.0, 0.0, -1.0, 0.0, 0.0))
    cen = np.stack([rng.uniform(5e4, 1e5, npad), rng.uniform(-1e5, 1e5, npad), rng.uniform(-1e5, 1e5, npad)], 1)
    off = rng.uniform(-0.5, 0.5, (npad, 3, 3))
    pad = (cen[:, None, :] + off).astype(np.float32).reshape(-1, 3)
    v = np.zeros((6 + 3 * npad, 8), np.float32)
    v[:6] = np.array(verts, np.float32)
    v[6:, :3] = pad
    v[6:, 5] = -1.0
    idx = np.arange(6 + 3 * npad, dtype=np.uint32)
    mats = np.zeros(3, _L.MATERIAL_DTYPE)
    for k, kd in enumerate(((0.9, 0.1, 0.1, 1.0), (0.1, 0.1, 0.9, 1.0), (0.5, 0.5, 0.5, 1.0))):
        mats[k]["diffuse"] = kd
        mats[k]["specular"] = (1.0, 1.0, 1.0, 1.0)
        mats[k]["shininess"] = 100.0 * (k + 1)
        mats[k]["alpha"] = 1.0
        mats[k]["tex_num"] = -1
    midx = np.concatenate([[0, 1], np.full(npad, 2)]).astype(np.uint32)
    return Scene(v, idx, midx, mats)
