// rtbvh_device.h -- device-side data layouts and the exact-arithmetic helpers
// shared by the build and trace kernels (gfx950, wave64).
//
// HBM layout (see DESIGN.md "Data layout"):
//   opos   float4[V]     object-space vertex positions (w unused), set_scene
//   tclip  float4[4*T]   per-triangle clip-space vertices (w of the first: the triangle) and
//                        {vertex indices, material index}: 64-B records, TRIANGLE order (Morton kernel)
//   keys/vals u32[T] x2  radix ping-pong (Morton code, triangle id)
//   leaf   float4[4*T]   64-B leaf records in SORTED order: {v0.xyz, e1.x}, {e1.yz, e2.xy},
//                        {e2.z, tri, bmin.xy}, {bmin.z, bmax.xyz}; e1 = v1-v0, e2 = v2-v0
//   rec    Inner[2T-1]   64-B node records in SLOTS (word layout below, not Inner's field
//                        names): the record of internal node k (the boxes and ids of its
//                        two children, and k itself) sits at slot
//                        pint[k] = 2*parent + side, the root's at slot 2T-2; slot pleaf[j]
//                        holds a pseudo-record {box_j, box_j with min.z NaN, LEAF_BIT|j, INVALID}
//                        for leaf j (build.hip store_pseudo_record).
//                        So the records of two siblings share one 128-B line: the binary
//                        walks step to slot 2k+side, the 4-wide walks read slots 2k, 2k+1
//                        (the four grandchild boxes of k) in one line.
//   topo   uint4[T-1]    build scratch indexed by node: Karras child ids + leaf range
//   inner  Inner[T-1]    build scratch: the box hand-off of refit nodes that span
//                        workgroups (only those are touched)
//   pleaf  u32[T], pint u32[T-1]   parent<<1 | side (side 0 = left child)
// Node ids: internal k -> k, leaf j -> LEAF_BIT | j.
// Node record words (so that each corner's (x, y) is an aligned pair for packed fp32):
//   0-1 left.min.xy  2-3 left.max.xy  4-5 right.min.xy  6-7 right.max.xy
//   8 left.min.z  9 left.max.z  10 right.min.z  11 right.max.z  12 id_l  13 id_r  14 own
//   15 bit s: child s's box needs the general slab test for axis-parallel primary rays
//      (not: min < max in x and y, min.z <= max.z, 0 <= max.z < inf; build.hip general_box)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "margin.h"

// A/B probes that render WRONG frames (the cost probes RTBVH_BOUNCE_PROBE / RTBVH_PB_PROBE /
// RTBVH_SMALL_PROBE, the step-by-step walk prints of RTBVH_DEBUG_PIXEL) compile only into A/B
// libraries built with -DRTBVH_AB_BUILD, which the Makefile refuses for librtbvh.so itself
#if (defined(RTBVH_BOUNCE_PROBE) || defined(RTBVH_SMALL_PROBE) || defined(RTBVH_DEBUG_PIXEL) || \
     (defined(RTBVH_PROBE_NOREC) && RTBVH_PROBE_NOREC != 0) || \
     (defined(RTBVH_REFIT_PROBE) && RTBVH_REFIT_PROBE != 0) || defined(RTBVH_TAIL_PROBE) || \
     (defined(RTBVH_PB_PROBE) && RTBVH_PB_PROBE != 0)) && !defined(RTBVH_AB_BUILD)
#error "probe builds render wrong frames: A/B libraries only (-DRTBVH_AB_BUILD, OUT=<another library>)"
#endif

namespace rtbvh {

constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t INVALID = 0xFFFFFFFFu;
constexpr uint32_t ABSENT_MINZ = 0x7FC00000u;   // min.z (a quiet NaN) of a pseudo-record's absent child
constexpr int STACK_SIZE = 66;   // binary walks: >= 64 levels of a clz64 Karras tree + sentinel
constexpr int STACK4 = 100;      // 4-wide primary packets (record pairs: a step descends two levels, pushes
                                 //   <= 3) on a <= 64-level clz64 tree: <= 3 * 32 + sentinel
constexpr int STACK4B = 3 * 64;  // 4-wide bounce walk on QNodes: the greedy collapse (build.hip) may leave
                                 //   entries one and three levels below the node, so a step can descend one
                                 //   level and push 3: <= 3 per level of <= 64 internal levels
// float4 per clip-space triangle in tclip: 64-B aligned records, so the refit's gather in sorted
// order reads one line per triangle (48-B records straddled lines: 1.47 read requests per
// triangle); C4 A/B: Morton +0.03 ms, refit -0.035 ms, build traffic -0.4 GB
#ifndef RTBVH_TCLIP_STRIDE
#define RTBVH_TCLIP_STRIDE 4
#endif
constexpr uint32_t TCS = RTBVH_TCLIP_STRIDE;

// 64-byte child-pair record of internal node k (boxes of both children, then ids)
struct alignas(64) Inner {
    float lmin[3], lmax[3];
    float rmin[3], rmax[3];
    uint32_t child_l, child_r;
    uint32_t aux0, aux1;   // rec: aux0 = own node index, aux1 = word 15 (general-box bits)
};
static_assert(sizeof(Inner) == 64, "Inner must be one 64-B record");

// 64-byte quantized 4-wide node of internal node k, stored at k's slot (qnode[pint[k]], the
// root's at 2T-2, as the records: siblings share a 128-B line): the boxes of
// k's four grandchildren -- the children of k's two children, in the order of the record
// pair at slots 2k, 2k+1 (a leaf child counts once, its second entry has id INVALID) --
// with every corner on an 8-bit per-axis grid whose origin is the min corner of k's box
// and whose step is a power of two:
//   org[3], scl[3]   grid origin and step (scl[0] == 0: not quantized, use the exact pair); the
//                    steps are powers of two, so the low 16 bits of scl[1] / scl[2] carry the
//                    certified walk's margin codes of the node (margin.h mt_node_codes: the largest
//                    edge bound of its leaves, rounded up, and its margin range, rounded down) --
//                    readers mask them off (& 0xFF800000)
//   lo[a], hi[a]     byte c = grandchild c's min / max on axis a in grid steps
//   id[4]            grandchildren: the slot of an internal one, LEAF_BIT | j, or INVALID
// qdecode() is exact in the product (8-bit q times a power of two) and rounds once in
// the add; the build picks q so that the decoded box contains the exact box.  The slab
// test is monotone in the box corners (every operation in it rounds monotonically), so
// a box the exact test hits is hit here too: a walk on these nodes reaches every leaf
// the record-pair walk reaches, pruning only on entry distances that are <= the exact
// ones.  Half the bytes per 4-wide step (64 vs 128).
struct alignas(64) QNode {
    float org[3], scl[3];
    uint32_t lo[3], hi[3];
    uint32_t id[4];
};
static_assert(sizeof(QNode) == 64, "QNode must be one 64-B record");
__device__ __forceinline__ float qdecode(float org, float scl, uint32_t w, int c) {
    return fmaf((float)((w >> (8 * c)) & 255u), scl, org);   // == org + q*scl: the product is exact
}

struct alignas(16) RayQ {   // bounce queue entry (32 B)
    uint32_t idx;           // output pixel index
    float intensity;
    float ox, oy, oz;
    float dx, dy, dz;
};
static_assert(sizeof(RayQ) == 32, "RayQ 32 B");

struct Mat {   // rtbvh_material, 68 B (read with scalar loads)
    float ambient[4], diffuse[4], specular[4];
    float shininess, optical_density, alpha;
    uint32_t specularb;
    int32_t tex_num;
};

// ---- exact helpers: same op order as oracle/rtbvh_oracle.cpp (no FMA: the
// translation unit is compiled with -ffp-contract=off) ----------------------
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 mul(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ f3 vmin(f3 a, f3 b) { return mk(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
__device__ __forceinline__ f3 vmax(f3 a, f3 b) { return mk(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
__device__ __forceinline__ f3 normalize(f3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return mul(v, inv); }
__device__ __forceinline__ f3 reflect(f3 i, f3 n) { float t = 2.0f * dot(i, n); return sub(i, mul(n, t)); }
__device__ __forceinline__ float magnitude(f3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
// 1.f / x, correctly rounded: v_rcp_f32 (within 1 ulp) and one fma Newton step give the IEEE
// quotient for every normal x whose reciprocal is normal (all 4,227,858,432 such fp32 values
// checked on MI355X, scripts/rcp_exhaustive.hip); the rest (0, denormals, |x| >= 2^126, inf,
// NaN) take the division.  4 VALU instead of the division's ~10.
__device__ __forceinline__ float recip(float x) {
    const float r0 = __builtin_amdgcn_rcpf(x);
    float r = fmaf(fmaf(-x, r0, 1.0f), r0, r0);
    if (!(fabsf(x) >= 0x1p-126f && fabsf(x) < 0x1p126f)) {
        asm volatile("");   // a real branch: not speculated and selected
        r = 1.0f / x;
    }
    return r;
}
__device__ __forceinline__ float sat(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }

// A leaf box's footprint on the primary rays' pixel grid (RayTraceLaunch.hlsl:23-24: pixel x is the
// ray at ((x - W/2) / 4, (y - H/2) / 4, 0), d = (0, 0, 1)), as pixel OFFSETS n = x - W/2 (so it does
// not depend on the frame size): the n with lo < n / 4 < hi on each axis -- exactly the rays the 4-wide
// packet walk's axis-parallel test lets through (n / 4 is exact) -- or, for a box that needs the
// general slab test (`general`), the closed superset lo <= n / 4 <= hi (every n when a corner is NaN).
// Written by the build, one 16-B record per sorted leaf: {nx0 | nx1 << 16, ny0 | ny1 << 16, zkey, general},
// offsets as int16 clamped to +-32767 (exact for frames of up to 32768 pixels a side: a clamped bound lies
// outside every such frame).  zkey <= min.z is the leaf's depth key (margin.h mt_primary_zkey): no pixel ray
// whose triangle test accepts the leaf returns t < zkey, so a pixel whose bound is below zkey cannot take
// the leaf -- even when the rounded t falls below min.z (containment failing).  Read by the
// binned primary pass (trace.hip k_pb_bin).
__device__ __forceinline__ void footprint_axis(float lo, float hi, bool general, int& a, int& b) {
    const float r = 4.f * lo, R = 4.f * hi;   // exact (powers of two); +-inf past the float range
    float fa, fb;
    if (!general) {
        fa = floorf(r) + 1.f;   // smallest integer > r (inexact only far outside any frame)
        fb = ceilf(R) - 1.f;    // largest integer < R
    } else if (r == r && R == R) {
        fa = ceilf(fminf(r, R));
        fb = floorf(fmaxf(r, R));
    } else {
        fa = -INFINITY;
        fb = INFINITY;
    }
    a = (int)fminf(fmaxf(fa, -32767.f), 32767.f);
    b = (int)fminf(fmaxf(fb, -32767.f), 32767.f);
}
__device__ __forceinline__ uint4 leaf_footprint(f3 lo, f3 hi, float zkey) {
    // the general bit of build.hip leaf_tri_word
    const bool general = !(lo.x < hi.x && lo.y < hi.y && lo.z <= hi.z && 0.f <= hi.z && hi.z < INFINITY);
    int x0, x1, y0, y1;
    footprint_axis(lo.x, hi.x, general, x0, x1);
    footprint_axis(lo.y, hi.y, general, y0, y1);
    return make_uint4((uint32_t)(x0 & 0xFFFF) | (uint32_t)x1 << 16, (uint32_t)(y0 & 0xFFFF) | (uint32_t)y1 << 16,
                      __float_as_uint(zkey), general ? 1u : 0u);
}
// A leaf's margin data from its record words r[0..2] = {v0, e1.x}, {e1.yz, e2.xy}, {e2.z, ...}: the edge
// bound E (the bounce walk's global margin, margin.h) and the primary rays' depth key, from the
// determinant the kernels compute for d = (0, 0, 1) (trace.hip ray_triangle_flat: dot(e1, cross(d, e2))).
__device__ __forceinline__ void leaf_margin(const float4 (&r)[4], float lo_z, float hi_z, float& E, float& zkey) {
    const f3 e1 = mk(r[0].w, r[1].x, r[1].y), e2 = mk(r[1].z, r[1].w, r[2].x);
    const float dx = dot(e1, cross(mk(0.f, 0.f, 1.f), e2));
    E = mt_edge_bound(e1.x, e1.y, e1.z, e2.x, e2.y, e2.z);
    zkey = mt_primary_zkey(dx, E, lo_z, hi_z);
}
__device__ __forceinline__ float lerpf(float a, float b, float s) { return a + s * (b - a); }

// mul(float4(p,1), M), row-major M (row-vector convention)
__device__ __forceinline__ f3 xform_point(const float* M, f3 p) {
    f3 r;
    r.x = ((p.x * M[0] + p.y * M[4]) + p.z * M[8]) + M[12];
    r.y = ((p.x * M[1] + p.y * M[5]) + p.z * M[9]) + M[13];
    r.z = ((p.x * M[2] + p.y * M[6]) + p.z * M[10]) + M[14];
    return r;
}
// mul(n, (float3x3)M)
__device__ __forceinline__ f3 xform_normal(const float* M, f3 n) {
    f3 r;
    r.x = (n.x * M[0] + n.y * M[4]) + n.z * M[8];
    r.y = (n.x * M[1] + n.y * M[5]) + n.z * M[9];
    r.z = (n.x * M[2] + n.y * M[6]) + n.z * M[10];
    return r;
}

}  // namespace rtbvh
