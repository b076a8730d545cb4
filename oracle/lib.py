"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY).

See oracle/rtbvh_oracle.h for what each function restates (reference file:line).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

MORTON_CPUTESTS, MORTON_HLSL = 0, 1
DELTA_CLZ64, DELTA_CPUTESTS = 0, 1

NODE_DTYPE = np.dtype([("parent", "<u4"), ("child_l", "<u4"), ("child_r", "<u4"), ("code", "<u4"),
                       ("bb_min", "<f4", (3,)), ("bb_max", "<f4", (3,)), ("index", "<u4")])
assert NODE_DTYPE.itemsize == 44


class _Texture(ctypes.Structure):   # orc_texture
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("rgba8", ctypes.c_void_p)]


class _Scene(ctypes.Structure):
    _fields_ = [("verts", ctypes.c_void_p), ("num_verts", ctypes.c_uint32),
                ("indices", ctypes.c_void_p), ("num_indices", ctypes.c_uint32),
                ("mat_indices", ctypes.c_void_p),
                ("materials", ctypes.c_void_p), ("num_materials", ctypes.c_uint32),
                ("textures", ctypes.c_void_p), ("num_textures", ctypes.c_uint32)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u32p = ctypes.c_void_p
        L.orc_expand_bits.restype = ctypes.c_uint32
        L.orc_expand_bits.argtypes = [ctypes.c_uint32]
        for f in (L.orc_morton_point_cputests, L.orc_morton_point_hlsl):
            f.restype = ctypes.c_uint32
            f.argtypes = [ctypes.c_float] * 3
        L.orc_morton_tris_cputests.argtypes = [ctypes.POINTER(_Scene), u32p]
        L.orc_morton_tris_hlsl.argtypes = [ctypes.POINTER(_Scene), u32p, u32p, u32p, u32p]
        L.orc_split_sort.argtypes = [u32p, ctypes.c_uint32, u32p]
        L.orc_lsd_sort.argtypes = [u32p, ctypes.c_uint32, u32p]
        L.orc_blelloch_scan256.argtypes = [u32p]
        L.orc_delta.restype = ctypes.c_int32
        L.orc_delta.argtypes = [ctypes.c_int, u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64]
        L.orc_karras.argtypes = [ctypes.c_int, u32p, ctypes.c_uint32, u32p, u32p, u32p]
        L.orc_refit.restype = ctypes.c_uint32
        L.orc_refit.argtypes = [ctypes.c_uint32, u32p, u32p, u32p, u32p, u32p]
        L.orc_build.restype = ctypes.c_int
        L.orc_build.argtypes = [ctypes.POINTER(_Scene), u32p, ctypes.c_int, ctypes.c_int, u32p, u32p,
                                ctypes.c_int, u32p]
        L.orc_trace.restype = ctypes.c_int
        L.orc_trace.argtypes = [ctypes.POINTER(_Scene), u32p, ctypes.c_uint32, u32p, u32p,
                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, u32p]
        L.orc_trace_ex.restype = ctypes.c_int
        L.orc_trace_ex.argtypes = L.orc_trace.argtypes + [u32p, u32p]
        L.orc_camera_reference.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u32p, u32p]
        L.orc_sample_texture.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, u32p]
        L.orc_fnv1a64.restype = ctypes.c_uint64
        L.orc_fnv1a64.argtypes = [u32p, ctypes.c_uint64]
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_set_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


class Scene:
    """Holds numpy arrays alive for the C struct view."""

    def __init__(self, vertices, indices, mat_indices, material_blob, textures=()):
        self.vertices = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 8)
        self.indices = np.ascontiguousarray(indices, dtype=np.uint32)
        self.mat_indices = np.ascontiguousarray(mat_indices, dtype=np.uint32)
        self.material_blob = np.ascontiguousarray(material_blob, dtype=np.uint8).reshape(-1, 68)
        self.textures = [np.ascontiguousarray(t, dtype=np.uint8) for t in textures]   # (H, W, 4)
        self._tex = (_Texture * max(len(self.textures), 1))()
        for k, t in enumerate(self.textures):
            self._tex[k] = _Texture(t.shape[1], t.shape[0], t.ctypes.data)
        self.c = _Scene(_p(self.vertices), len(self.vertices), _p(self.indices), len(self.indices),
                        _p(self.mat_indices), _p(self.material_blob), len(self.material_blob),
                        ctypes.cast(self._tex, ctypes.c_void_p) if self.textures else None, len(self.textures))

    @property
    def num_tris(self) -> int:
        return len(self.indices) // 3


def morton_point_cputests(x, y, z) -> int:
    return lib().orc_morton_point_cputests(x, y, z)


def morton_point_hlsl(x, y, z) -> int:
    return lib().orc_morton_point_hlsl(x, y, z)


def morton_tris(scene: Scene, mode=MORTON_CPUTESTS, wvp=None, smin=None, smax=None) -> np.ndarray:
    out = np.zeros(scene.num_tris, dtype=np.uint32)
    if mode == MORTON_CPUTESTS:
        lib().orc_morton_tris_cputests(ctypes.byref(scene.c), _p(out))
    else:
        wvp = np.ascontiguousarray(wvp, dtype=np.float32)
        smin = np.ascontiguousarray(smin, dtype=np.float32)
        smax = np.ascontiguousarray(smax, dtype=np.float32)
        lib().orc_morton_tris_hlsl(ctypes.byref(scene.c), _p(wvp), _p(smin), _p(smax), _p(out))
    return out


def split_sort(keys: np.ndarray) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.zeros(len(keys), dtype=np.uint32)
    lib().orc_split_sort(_p(keys), len(keys), _p(perm))
    return perm


def lsd_sort(keys: np.ndarray) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    perm = np.zeros(len(keys), dtype=np.uint32)
    lib().orc_lsd_sort(_p(keys), len(keys), _p(perm))
    return perm


def blelloch_scan256(data: np.ndarray) -> np.ndarray:
    d = np.ascontiguousarray(data, dtype=np.uint32).copy()
    assert d.size == 256
    lib().orc_blelloch_scan256(_p(d))
    return d


def karras(sorted_codes: np.ndarray, mode=DELTA_CLZ64):
    c = np.ascontiguousarray(sorted_codes, dtype=np.uint32)
    n = len(c)
    parent = np.zeros(2 * n - 1, dtype=np.uint32)
    cl = np.zeros(2 * n - 1, dtype=np.uint32)
    cr = np.zeros(2 * n - 1, dtype=np.uint32)
    lib().orc_karras(mode, _p(c), n, _p(parent), _p(cl), _p(cr))
    return parent, cl, cr


def refit(n, parent, cl, cr, bb_min, bb_max):
    bmin = np.ascontiguousarray(bb_min, dtype=np.float32).copy()
    bmax = np.ascontiguousarray(bb_max, dtype=np.float32).copy()
    longest = lib().orc_refit(n, _p(np.ascontiguousarray(parent, np.uint32)),
                              _p(np.ascontiguousarray(cl, np.uint32)),
                              _p(np.ascontiguousarray(cr, np.uint32)), _p(bmin), _p(bmax))
    return bmin, bmax, longest


def build(scene: Scene, wvp, morton_mode=MORTON_CPUTESTS, delta_mode=DELTA_CLZ64,
          smin=(-700.0, -700.0, -700.0), smax=(700.0, 700.0, 700.0), sort_mode=1) -> np.ndarray:
    n = scene.num_tris
    out = np.zeros(2 * n - 1, dtype=NODE_DTYPE)
    wvp = np.ascontiguousarray(wvp, dtype=np.float32)
    smin = np.ascontiguousarray(smin, dtype=np.float32)
    smax = np.ascontiguousarray(smax, dtype=np.float32)
    rc = lib().orc_build(ctypes.byref(scene.c), _p(wvp), morton_mode, delta_mode, _p(smin), _p(smax),
                         sort_mode, ctypes.c_void_p(out.ctypes.data))
    if rc != 0:
        raise RuntimeError(f"orc_build failed ({rc})")
    return out


def trace(scene: Scene, nodes: np.ndarray, wvp, wv, W, H, bounces, row_begin=0, row_end=None,
          row_step=1, want_intensity=False, want_records=False):
    """Oracle frame (rgba, intensity, stats); with want_records also the reflectRay and
    refractRay RayPresent records as (rows, W, 14) float32 (orc_trace_ex)."""
    n = scene.num_tris
    if row_end is None:
        row_end = H
    rows = len(range(row_begin, min(row_end, H), row_step))
    rgba = np.zeros((rows, W, 4), dtype=np.float32)
    inten = np.zeros((rows, W), dtype=np.float32) if want_intensity else None
    counters = np.zeros(8, dtype=np.uint64)
    wvp = np.ascontiguousarray(wvp, dtype=np.float32)
    wv = np.ascontiguousarray(wv, dtype=np.float32)
    nodes = np.ascontiguousarray(nodes)
    refl = np.zeros((rows, W, 14), dtype=np.float32) if want_records else None
    refr = np.zeros((rows, W, 14), dtype=np.float32) if want_records else None
    rc = lib().orc_trace_ex(ctypes.byref(scene.c), ctypes.c_void_p(nodes.ctypes.data), n, _p(wvp), _p(wv),
                            W, H, bounces, row_begin, row_end, row_step, _p(rgba),
                            _p(inten) if inten is not None else None, _p(counters),
                            _p(refl) if refl is not None else None, _p(refr) if refr is not None else None)
    if rc != 0:
        raise RuntimeError(f"orc_trace failed ({rc})")
    keys = ["primary", "bounce", "internal_visits", "leaf_visits", "hits", "textured_hits",
            "stack_overflows", "max_stack"]
    stats = {k: int(v) for k, v in zip(keys, counters)}
    if want_records:
        return rgba, inten, stats, refl, refr
    return rgba, inten, stats


def sample_texture(tex: np.ndarray, u: float, v: float) -> np.ndarray:
    """orc_sample_texture on an (H, W, 4) uint8 texture."""
    tex = np.ascontiguousarray(tex, dtype=np.uint8)
    t = _Texture(tex.shape[1], tex.shape[0], tex.ctypes.data)
    out = np.zeros(4, np.float32)
    lib().orc_sample_texture(ctypes.byref(t), u, v, _p(out))
    return out


def camera_reference(W, H):
    wvp = np.zeros(16, dtype=np.float32)
    wv = np.zeros(16, dtype=np.float32)
    lib().orc_camera_reference(W, H, _p(wvp), _p(wv))
    return wvp.reshape(4, 4), wv.reshape(4, 4)


def set_threads(n: int) -> None:
    """Threads trace() uses over rows (default 1; the result does not depend on it)."""
    lib().orc_set_threads(int(n))


def fnv1a64(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a)
    return int(lib().orc_fnv1a64(ctypes.c_void_p(a.ctypes.data), a.nbytes))
