"""Scene inputs of the path (vertices, indices, material indices, materials).

Host-side mirror of ObjLoader's getters (ObjectFileLoader.h:120-240); the
loading itself is native (rtbvh_scene_load_obj in librtbvh.so).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib as _L


@dataclass
class Scene:
    vertices: np.ndarray                 # (V, 8) f32: position xyz, normal xyz, texcoord uv (32-B Vertex)
    indices: np.ndarray                  # (3T,) u32
    mat_indices: np.ndarray              # (T,) u32
    materials: np.ndarray                # (M,) MATERIAL_DTYPE (68-B MaterialUpload)
    texture_paths: list = field(default_factory=list)
    textures: list = field(default_factory=list)   # (H, W, 4) uint8 per texNum, row 0 = v = 0

    def __post_init__(self):
        self.vertices = np.ascontiguousarray(self.vertices, dtype=np.float32).reshape(-1, 8)
        self.indices = np.ascontiguousarray(self.indices, dtype=np.uint32).ravel()
        self.mat_indices = np.ascontiguousarray(self.mat_indices, dtype=np.uint32).ravel()
        m = np.ascontiguousarray(self.materials)
        if m.dtype != _L.MATERIAL_DTYPE:
            m = np.frombuffer(np.ascontiguousarray(m, dtype=np.uint8).tobytes(), dtype=_L.MATERIAL_DTYPE).copy()
        self.materials = m
        self.textures = [np.ascontiguousarray(t, dtype=np.uint8).reshape(t.shape[0], t.shape[1], 4)
                         for t in self.textures]

    @property
    def num_tris(self) -> int:
        return len(self.indices) // 3

    @property
    def material_blob(self) -> np.ndarray:
        return self.materials.view(np.uint8).reshape(-1, 68)

    # ObjLoader getter names (ObjectFileLoader.h:139-212)
    def getNumVertices(self) -> int:  # noqa: N802
        return len(self.vertices)

    def getNumIndices(self) -> int:  # noqa: N802
        return len(self.indices)

    def getNumMaterialIndices(self) -> int:  # noqa: N802
        return len(self.mat_indices)

    def getNumMaterials(self) -> int:  # noqa: N802
        return len(self.materials)


def _from_native(handle) -> Scene:
    L = _L.lib()
    nv = L.rtbvh_scene_num_vertices(handle)
    ni = L.rtbvh_scene_num_indices(handle)
    nm = L.rtbvh_scene_num_materials(handle)
    nt = L.rtbvh_scene_num_textures(handle)
    verts = np.ctypeslib.as_array(ctypes.cast(L.rtbvh_scene_vertices(handle), ctypes.POINTER(ctypes.c_float)),
                                  shape=(nv * 8,)).copy() if nv else np.zeros(0, np.float32)
    idx = np.ctypeslib.as_array(ctypes.cast(L.rtbvh_scene_indices(handle), ctypes.POINTER(ctypes.c_uint32)),
                                shape=(ni,)).copy() if ni else np.zeros(0, np.uint32)
    midx = np.ctypeslib.as_array(ctypes.cast(L.rtbvh_scene_mat_indices(handle), ctypes.POINTER(ctypes.c_uint32)),
                                 shape=(ni // 3,)).copy() if ni else np.zeros(0, np.uint32)
    mats = np.ctypeslib.as_array(ctypes.cast(L.rtbvh_scene_materials(handle), ctypes.POINTER(ctypes.c_uint8)),
                                 shape=(nm * 68,)).copy()
    paths = [L.rtbvh_scene_texture_path(handle, k).decode() for k in range(nt)]
    return Scene(verts.reshape(-1, 8), idx, midx, mats.view(_L.MATERIAL_DTYPE), paths)


def load_texture(path: str) -> np.ndarray:
    """Image::loadImage (Image.cpp:35-61): RGBA8 rows in the order DevIL hands them over
    without IL_ORIGIN_SET -- the file's own order (BMP: bottom row first; JPEG: top row
    first), decoded natively by librtbvh (rtbvh_texture_load: BMP or baseline JPEG).
    Formats the native decoders do not read (PNG, TGA, progressive JPEG, ...), which DevIL
    decodes, fall back to PIL as host-side image I/O, in the same file-order convention."""
    L = _L.lib()
    t = _L.Texture()
    st = L.rtbvh_texture_load(os.fsencode(path), ctypes.byref(t))
    if st == _L.ERR_IO and os.path.isfile(path):
        return _load_texture_pil(path)
    _L.check(st)
    try:
        return np.ctypeslib.as_array(ctypes.cast(t.rgba8, ctypes.POINTER(ctypes.c_uint8)),
                                     shape=(t.height, t.width, 4)).copy()
    finally:
        L.rtbvh_texture_free(ctypes.byref(t))


def _load_texture_pil(path: str) -> np.ndarray:
    """PIL decode of a texture the native decoders reject; rows in file order as DevIL
    hands them over: a TGA stored bottom-up (image descriptor bit 5 clear) bottom row
    first, every other format top row first.  Raises RtbvhError(ERR_IO) if PIL cannot
    read the file either."""
    try:
        from PIL import Image
    except ImportError as e:   # no host image library: the native decoders' error stands
        raise _L.RtbvhError(_L.ERR_IO, f"{path}: not BMP/baseline JPEG and PIL is unavailable") from e
    try:
        with Image.open(path) as im:
            fmt = im.format
            rgba = np.asarray(im.convert("RGBA"), dtype=np.uint8).copy()
    except (OSError, ValueError) as e:
        raise _L.RtbvhError(_L.ERR_IO, f"{path}: {e}") from e
    if fmt == "TGA":
        with open(path, "rb") as f:
            hdr = f.read(18)
        if len(hdr) == 18 and not (hdr[17] & 0x20):   # bottom-left origin: DevIL keeps file order
            rgba = rgba[::-1].copy()
    return rgba


def decode_jpeg(data: bytes) -> np.ndarray:
    """rtbvh_texture_decode_jpeg on an in-memory file: (H, W, 4) uint8, top row first."""
    L = _L.lib()
    t = _L.Texture()
    buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
    _L.check(L.rtbvh_texture_decode_jpeg(buf, len(data), ctypes.byref(t)))
    try:
        return np.ctypeslib.as_array(ctypes.cast(t.rgba8, ctypes.POINTER(ctypes.c_uint8)),
                                     shape=(t.height, t.width, 4)).copy()
    finally:
        L.rtbvh_texture_free(ctypes.byref(t))


def load_obj(path: str, load_textures: bool = True) -> Scene:
    """ObjLoader::Load (ObjectFileLoader.cpp:470-547) via the native loader, plus the map_Kd
    textures (ObjectFileLoader.cpp:459-461 numbers them in material order).  A texture that
    cannot be read is reported and replaced by one white texel (the reference prints the
    error and continues, ObjectFileLoader.cpp:199-208)."""
    L = _L.lib()
    h = ctypes.c_void_p()
    _L.check(L.rtbvh_scene_load_obj(os.fsencode(path), ctypes.byref(h)))
    try:
        sc = _from_native(h)
    finally:
        L.rtbvh_scene_free(h)
    if load_textures:
        base = os.path.dirname(os.path.abspath(path))
        for name in sc.texture_paths:
            try:
                sc.textures.append(load_texture(os.path.join(base, name)))
            except Exception as e:   # noqa: BLE001
                import warnings
                warnings.warn(f"texture {name}: {e}; using white")
                sc.textures.append(np.full((1, 1, 4), 255, np.uint8))
    return sc


def synthetic(ntris: int, seed: int = 0x5EED0004, half_extent=(50.0, 50.0, 50.0)) -> Scene:
    """SURVEY §8(d) synthetic scene (C4: seed 0x5EED0004, +-50; C5: 0x5EED0005, (100,100,50))."""
    L = _L.lib()
    h = ctypes.c_void_p()
    half = np.asarray(half_extent, dtype=np.float32)
    _L.check(L.rtbvh_scene_synthetic(seed, ntris, _L.ptr(half), ctypes.byref(h)))
    try:
        return _from_native(h)
    finally:
        L.rtbvh_scene_free(h)


def load_npz(path: str) -> Scene:
    """Scene fixture written by tests/golden/make_golden.py (parsed reference Obj/ meshes)."""
    z = np.load(path)
    names = [str(x) for x in z["texture_names"]] if "texture_names" in z else []
    return Scene(z["vertices"], z["indices"], z["mat_indices"], z["material_blob"], names)


def srgb_table() -> np.ndarray:
    """The sRGB -> linear table of the texture sampler (rtbvh_srgb_table)."""
    out = np.zeros(256, np.float32)
    _L.lib().rtbvh_srgb_table(_L.ptr(out))
    return out


def camera_reference(width: int, height: int):
    """Graphics::onUpdate camera (Graphics.cpp:44-53): returns (WVP, WV) as (4,4) f32, row-vector convention."""
    wvp = np.zeros(16, np.float32)
    wv = np.zeros(16, np.float32)
    _L.lib().rtbvh_camera_reference(width, height, _L.ptr(wvp), _L.ptr(wv))
    return wvp.reshape(4, 4), wv.reshape(4, 4)


def camera_look(eye, width: int, height: int):
    """Graphics::onUpdate's camera from any eye (at 0, up +y; rtbvh_camera_look): (WVP, WV) as (4,4) f32."""
    e = np.ascontiguousarray(eye, np.float32).reshape(3)
    wvp = np.zeros(16, np.float32)
    wv = np.zeros(16, np.float32)
    _L.lib().rtbvh_camera_look(_L.ptr(e), width, height, _L.ptr(wvp), _L.ptr(wv))
    return wvp.reshape(4, 4), wv.reshape(4, 4)


# Graphics::onKeyDown's keys (Graphics.cpp:937-960)
KEY_LEFT, KEY_RIGHT, KEY_UP, KEY_DOWN = 0, 1, 2, 3
EYE_REFERENCE = (0.0, 5.0, -100.0)   # Graphics.h:200-205


def camera_orbit(eye, key: int) -> np.ndarray:
    """The eye after one Graphics::onKeyDown (rtbvh_camera_orbit): rotated about the origin by CAM_DELTA."""
    e = np.array(eye, np.float32).reshape(3)
    _L.lib().rtbvh_camera_orbit(_L.ptr(e), key)
    return e
