"""Host-side mirror of the reference's Manager/Graphics dispatch surface.

The reference drives the path from `class Graphics : public Manager`
(Graphics.h:16-27): onInit -> loadAssets uploads the ObjLoader arrays
(Graphics.cpp:237-665), onUpdate writes the camera cbuffer and calls the private
computeBVH() (Graphics.cpp:40-61, 667-831).  `Graphics` below keeps those names
and meanings over librtbvh.so; `Context` is the thin 1:1 wrapper of the C ABI.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib as _L
from .scene import EYE_REFERENCE, Scene, camera_look, camera_orbit, camera_reference


class Context:
    """One rtbvh_ctx: one HIP device, one stream, the scene/BVH/frame buffers."""

    def __init__(self, device: int = 0, morton_mode: int = _L.MORTON_CPUTESTS, delta_mode: int = _L.DELTA_CLZ64,
                 flags: int = 0, scene_bb_min=(-700.0,) * 3, scene_bb_max=(700.0,) * 3, stream: int | None = None,
                 stack_limit: int = 0):
        L = _L.lib()
        cfg = _L.Config()
        L.rtbvh_config_default(ctypes.byref(cfg))
        cfg.device = device
        cfg.morton_mode = morton_mode
        cfg.delta_mode = delta_mode
        cfg.flags = flags
        cfg.scene_bb_min[:] = list(scene_bb_min)
        cfg.scene_bb_max[:] = list(scene_bb_max)
        cfg.stream = stream
        cfg.stack_limit = stack_limit
        h = ctypes.c_void_p()
        _L.check(L.rtbvh_create(ctypes.byref(cfg), ctypes.byref(h)), None)
        self._h = h
        self.num_tris = 0
        self.width = self.height = 0

    # -- lifecycle --
    def close(self):
        if getattr(self, "_h", None):
            _L.lib().rtbvh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st):
        _L.check(st, self._h)

    # -- inputs --
    def set_scene(self, scene: Scene):
        self._scene = scene   # keep arrays alive for the duration of the call (copied by the library)
        tex = (_L.Texture * max(len(scene.textures), 1))()
        for k, t in enumerate(scene.textures):
            tex[k] = _L.Texture(t.shape[1], t.shape[0], t.ctypes.data)
        self._check(_L.lib().rtbvh_set_scene(self._h, _L.ptr(scene.vertices), len(scene.vertices),
                                             _L.ptr(scene.indices), len(scene.indices), _L.ptr(scene.mat_indices),
                                             _L.ptr(scene.materials), len(scene.materials),
                                             ctypes.byref(tex) if scene.textures else None, len(scene.textures)))
        self.num_tris = scene.num_tris

    def set_camera(self, wvp, wv):
        wvp = np.ascontiguousarray(wvp, dtype=np.float32).reshape(16)
        wv = np.ascontiguousarray(wv, dtype=np.float32).reshape(16)
        self._check(_L.lib().rtbvh_set_camera(self._h, _L.ptr(wvp), _L.ptr(wv)))

    # -- hot path --
    def build(self, sync: bool = True):
        L = _L.lib()
        self._check(L.rtbvh_build(self._h) if sync else L.rtbvh_build_async(self._h))

    def trace(self, width: int, height: int, bounces: int = 1, sync: bool = True):
        L = _L.lib()
        f = L.rtbvh_trace if sync else L.rtbvh_trace_async
        self._check(f(self._h, width, height, bounces))
        self.width, self.height = width, height

    def compute_bvh(self, width: int, height: int, bounces: int = 1):
        self._check(_L.lib().rtbvh_compute_bvh(self._h, width, height, bounces))
        self.width, self.height = width, height

    def verify_walk(self, width: int, height: int, bounces: int = 1) -> int:
        """rtbvh_verify_walk: pixels whose bits differ between the reference-order frame and
        the frame of this context's walks (0: identical); leaves the latter in the framebuffer."""
        n = ctypes.c_uint64()
        self._check(_L.lib().rtbvh_verify_walk(self._h, width, height, bounces, ctypes.byref(n)))
        self.width, self.height = width, height
        return n.value

    def trace_band_async(self, width: int, height: int, bounces: int, rank: int, nranks: int, dev_out_ptr: int,
                         stream_ptr: int | None = None):
        self._check(_L.lib().rtbvh_trace_band_async(self._h, width, height, bounces, rank, nranks,
                                                    ctypes.c_void_p(dev_out_ptr),
                                                    ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def set_band_deal(self, root_share: int):
        """rtbvh_set_band_deal: rank 0's share of the bands in 1/16 of another rank's (16 = b % nranks)."""
        self._check(_L.lib().rtbvh_set_band_deal(self._h, root_share))

    def assemble_bands(self, width: int, height: int, nranks: int, dev_bands_ptr: int, stride_rows: int,
                       dev_frame_ptr: int, stream_ptr: int | None = None):
        """rtbvh_assemble_bands: the frame from the ranks' compact band buffers (one device)."""
        self._check(_L.lib().rtbvh_assemble_bands(self._h, width, height, nranks, ctypes.c_void_p(dev_bands_ptr),
                                                  stride_rows, ctypes.c_void_p(dev_frame_ptr),
                                                  ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def comm_init(self, nranks: int, rank: int, unique_id: bytes) -> int:
        """rtbvh_comm_init: an RCCL communicator (ncclComm_t) for this context's device."""
        assert len(unique_id) == _L.COMM_ID_BYTES
        comm = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * _L.COMM_ID_BYTES).from_buffer_copy(unique_id)
        self._check(_L.lib().rtbvh_comm_init(self._h, nranks, rank, buf, ctypes.byref(comm)))
        return comm.value

    def trace_tiles(self, width: int, height: int, bounces: int, rank: int, nranks: int, comm: int):
        """rtbvh_trace_tiles: this rank's bands + the RCCL gather; rank 0 then holds the frame."""
        self._check(_L.lib().rtbvh_trace_tiles(self._h, width, height, bounces, rank, nranks, ctypes.c_void_p(comm)))
        self.width, self.height = width, height

    def synchronize(self):
        self._check(_L.lib().rtbvh_synchronize(self._h))

    # -- outputs --
    def read_framebuffer(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.float32)
        self._check(_L.lib().rtbvh_read_framebuffer(self._h, _L.ptr(out)))
        return out

    def read_rays(self):
        """(reflectRay, refractRay) RayPresent records of the last full-frame trace made with
        FLAG_REFRACT_RECORDS, each (H, W, 14) float32: intensity, origin, direction,
        invDirection, color (RayTraceGlobal.hlsl:30-35)."""
        refl = np.zeros((self.height, self.width, 14), np.float32)
        refr = np.zeros((self.height, self.width, 14), np.float32)
        self._check(_L.lib().rtbvh_read_rays(self._h, _L.ptr(refl), _L.ptr(refr)))
        return refl, refr

    def present(self) -> np.ndarray:
        """The image the pixel shader shows (RayTraceBVHPS.hlsl:13-16): (H, W, 4) uint8, top row first."""
        out = np.zeros((self.height, self.width, 4), np.uint8)
        self._check(_L.lib().rtbvh_present(self._h, _L.ptr(out)))
        return out

    def read_intensity(self) -> np.ndarray:
        out = np.zeros((self.height, self.width), np.float32)
        self._check(_L.lib().rtbvh_read_intensity(self._h, _L.ptr(out)))
        return out

    def framebuffer_device_ptr(self) -> int:
        return _L.lib().rtbvh_framebuffer_device(self._h) or 0

    def read_bvh(self) -> np.ndarray:
        out = np.zeros(2 * self.num_tris - 1, dtype=_L.NODE_DTYPE)
        self._check(_L.lib().rtbvh_read_bvh(self._h, ctypes.c_void_p(out.ctypes.data), len(out)))
        return out

    def read_wide(self) -> np.ndarray:
        """Node records in slots (both walks' layout): (2(n-1), 16) uint32 records, see rtbvh_read_wide."""
        out = np.zeros((max(2 * (self.num_tris - 1), 0), 16), np.uint32)
        self._check(_L.lib().rtbvh_read_wide(self._h, _L.ptr(out), len(out)))
        return out

    def read_qnodes(self) -> np.ndarray:
        """Quantized 4-wide nodes of the bounce walk in slots: (2n-1, 16) uint32, see rtbvh_read_qnodes."""
        out = np.zeros((max(2 * self.num_tris - 1, 0) if self.num_tris > 1 else 0, 16), np.uint32)
        self._check(_L.lib().rtbvh_read_qnodes(self._h, _L.ptr(out), len(out)))
        return out

    def read_morton(self) -> np.ndarray:
        out = np.zeros(self.num_tris, np.uint32)
        self._check(_L.lib().rtbvh_read_morton(self._h, _L.ptr(out)))
        return out

    def read_sorted(self):
        keys = np.zeros(self.num_tris, np.uint32)
        ids = np.zeros(self.num_tris, np.uint32)
        self._check(_L.lib().rtbvh_read_sorted(self._h, _L.ptr(keys), _L.ptr(ids)))
        return keys, ids

    def stats(self) -> dict:
        """rtbvh_get_stats: counts of the last trace; hipEvent averages since reset_stats()."""
        s = _L.Stats()
        self._check(_L.lib().rtbvh_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        self._check(_L.lib().rtbvh_reset_stats(self._h))

    def set_flags(self, flags: int):
        self._check(_L.lib().rtbvh_set_flags(self._h, flags))

    # -- primitives --
    def sort_pairs(self, keys: np.ndarray, vals: np.ndarray, key_bits: int = 32):
        keys = np.ascontiguousarray(keys, np.uint32)
        vals = np.ascontiguousarray(vals, np.uint32)
        ko = np.zeros_like(keys)
        vo = np.zeros_like(vals)
        self._check(_L.lib().rtbvh_sort_pairs_host(self._h, _L.ptr(keys), _L.ptr(vals), _L.ptr(ko), _L.ptr(vo),
                                                   len(keys), key_bits))
        return ko, vo

    def sort_pairs_device(self, keys_ptr: int, vals_ptr: int, keys_out_ptr: int, vals_out_ptr: int, n: int,
                          key_bits: int = 32):
        self._check(_L.lib().rtbvh_sort_pairs_async(self._h, ctypes.c_void_p(keys_ptr), ctypes.c_void_p(vals_ptr),
                                                    ctypes.c_void_p(keys_out_ptr), ctypes.c_void_p(vals_out_ptr),
                                                    n, key_bits))

    def build_from_codes(self, sorted_codes: np.ndarray, leaf_boxes: np.ndarray) -> np.ndarray:
        codes = np.ascontiguousarray(sorted_codes, np.uint32)
        boxes = np.ascontiguousarray(leaf_boxes, np.float32).reshape(-1, 6)
        out = np.zeros(2 * len(codes) - 1, dtype=_L.NODE_DTYPE)
        self._check(_L.lib().rtbvh_build_from_codes(self._h, _L.ptr(codes), _L.ptr(boxes), len(codes),
                                                    ctypes.c_void_p(out.ctypes.data)))
        return out


class Graphics:
    """Graphics : Manager (Graphics.h:16-27) over librtbvh.so.

    onInit(scene)  ~ Graphics::onInit -> loadAssets (Graphics.cpp:34-38, 237-665)
    onUpdate()     ~ Graphics::onUpdate: camera + computeBVH (Graphics.cpp:40-61)
    computeBVH()   ~ Graphics::computeBVH (Graphics.cpp:667-831)
    """

    def __init__(self, width: int = 800, height: int = 800, bounces: int = 3, **ctx_kwargs):
        # main.cpp:7 opens an 800x800 window; Graphics.cpp:795 runs 3 reflection passes
        self.width, self.height, self.bounces = width, height, bounces
        self.eye = np.array(EYE_REFERENCE, np.float32)   # Graphics.h:200-205
        self.ctx = Context(**ctx_kwargs)

    def onInit(self, scene: Scene):  # noqa: N802
        self.ctx.set_scene(scene)

    def onUpdate(self):  # noqa: N802
        wvp, wv = camera_look(self.eye, self.width, self.height)
        self.ctx.set_camera(wvp, wv)
        self.computeBVH()

    def onKeyDown(self, key: int):  # noqa: N802
        """Graphics::onKeyDown (Graphics.cpp:937-960): KEY_LEFT/RIGHT/UP/DOWN orbit the eye about the origin."""
        self.eye = camera_orbit(self.eye, key)

    def computeBVH(self):  # noqa: N802
        self.ctx.compute_bvh(self.width, self.height, self.bounces)

    def framebuffer(self) -> np.ndarray:
        """reflectRay[].color as (H, W, 4) f32 (the framebuffer of record, RayTraceBVHPS.hlsl:13-16)."""
        return self.ctx.read_framebuffer()

    def onRender(self) -> np.ndarray:  # noqa: N802
        """Graphics::onRender's frame (the presentation pass) as RGBA8."""
        return self.ctx.present()

    def save_bmp(self, path: str):
        """SaveBMP (SaveBMP.cpp:3-62) of the presented frame."""
        save_bmp(path, self.onRender())

    def onDestroy(self):  # noqa: N802
        self.ctx.close()


def comm_unique_id() -> bytes:
    """rtbvh_comm_unique_id: the 128-B RCCL id rank 0 creates and shares with every rank."""
    buf = (ctypes.c_uint8 * _L.COMM_ID_BYTES)()
    _L.check(_L.lib().rtbvh_comm_unique_id(buf))
    return bytes(buf)


def comm_destroy(comm: int):
    """rtbvh_comm_destroy."""
    _L.check(_L.lib().rtbvh_comm_destroy(ctypes.c_void_p(comm)))


def save_bmp(path: str, rgba8: np.ndarray):
    """rtbvh_save_bmp: 24-bit BMP of an (H, W, 4) uint8 image, top row first."""
    img = np.ascontiguousarray(rgba8, dtype=np.uint8)
    _L.check(_L.lib().rtbvh_save_bmp(os.fsencode(path), _L.ptr(img), img.shape[1], img.shape[0]))
