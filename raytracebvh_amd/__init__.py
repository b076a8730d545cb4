"""raytracebvh_amd -- MI355X-native LBVH build + ray traversal (the hot path of
Fierykev/RayTraceBVH) as hand-written HIP kernels for gfx950 behind a C ABI
(include/rtbvh.h, librtbvh.so).  This package is the thin host-side mirror of the
reference's Manager/Graphics + ObjLoader surface; all compute is in the HIP library.
"""
from ._lib import (DELTA_CLZ64, DELTA_CPUTESTS, FLAG_COUNT_VISITS, FLAG_NEAREST_FIRST, FLAG_REFRACT_RECORDS,
                   FLAG_SORT_BOUNCE, FLAG_TIMING, FLAG_AUTO_WALK, FLAG_PACKET_PRIMARY,
                   FLAG_REFILL_BOUNCE, FLAG_WIDE_BVH, FLAG_BINNED_PRIMARY, FLAG_CERTIFIED, FLAG_MULTI_KERNEL_BUILD, FLAG_SPLIT_SHIFT,
                   FLAG_GRAPH, MATERIAL_DTYPE, MORTON_CPUTESTS, MORTON_HLSL, NODE_DTYPE, RtbvhError, lib)
from .graphics import Context, Graphics, comm_destroy, comm_unique_id, save_bmp
from .scene import (EYE_REFERENCE, KEY_DOWN, KEY_LEFT, KEY_RIGHT, KEY_UP, Scene, camera_look, camera_orbit,
                    camera_reference, load_npz, load_obj, synthetic)

__all__ = ["Context", "Graphics", "Scene", "load_obj", "load_npz", "synthetic", "camera_reference", "camera_look",
           "camera_orbit", "EYE_REFERENCE", "KEY_LEFT", "KEY_RIGHT", "KEY_UP", "KEY_DOWN", "lib",
           "RtbvhError", "NODE_DTYPE", "MATERIAL_DTYPE", "MORTON_CPUTESTS", "MORTON_HLSL", "DELTA_CLZ64",
           "DELTA_CPUTESTS", "FLAG_TIMING", "FLAG_COUNT_VISITS", "FLAG_REFRACT_RECORDS", "FLAG_SORT_BOUNCE",
           "FLAG_NEAREST_FIRST", "FLAG_AUTO_WALK", "FLAG_PACKET_PRIMARY", "FLAG_REFILL_BOUNCE", "FLAG_WIDE_BVH", "FLAG_BINNED_PRIMARY", "FLAG_CERTIFIED",
           "FLAG_MULTI_KERNEL_BUILD", "FLAG_SPLIT_SHIFT", "FLAG_GRAPH",
           "save_bmp", "comm_unique_id", "comm_destroy"]
