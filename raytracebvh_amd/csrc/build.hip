// build.hip -- LBVH build kernels for gfx950: scene bounds, Morton codes,
// leaf records + Karras internal nodes, bottom-up refit, reference-layout export.
//
// Reference: MortonCodes.hlsl (2 triangles per thread, writes whole 44-B nodes),
// BVHConstructP1.hlsl (Karras 2012, one thread per internal node), and
// BVHConstructP2.hlsl (atomic 2nd-arriver refit).  Differences by design (see
// DESIGN.md): codes and triangle ids are sorted as 8-B pairs instead of moving
// 44-B nodes; the clip-space triangle is written once in triangle order and
// gathered once into SORTED leaf records; each internal node is one 64-B record
// holding both children's boxes, so traversal reads one line per node.
#include "rtbvh_internal.h"

namespace rtbvh {
namespace {

#ifndef RTBVH_NT_STORES
#define RTBVH_NT_STORES 7
#endif
// Streaming stores of the coalesced build outputs (RTBVH_NT_STORES bit 0: the Morton pass's clip
// triangles, bit 1: the staged leaf records, bit 2: k_refit's staged records / pseudo-records /
// QNodes).  NT = 1 only; scattered 64-B record stores non-temporal ran 3x slower (refit stage
// 1.0 -> 3.3 ms at C4), the same records staged through LDS and stored 16 B per lane 12% faster.
template <int BIT>
__device__ __forceinline__ void st_out(float4* p, float4 v) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    if (RTBVH_NT_STORES & BIT) __builtin_nontemporal_store(v4{v.x, v.y, v.z, v.w}, reinterpret_cast<v4*>(p));
    else *p = v;
}

constexpr uint32_t BLOCK = 256;
#ifndef RTBVH_REFIT_BLOCK
#define RTBVH_REFIT_BLOCK 512
#endif
// leaves (and node indices) per k_refit workgroup: the nodes whose leaf range lies inside
// one join in LDS; the others ("crossing") climb in k_refit_group
constexpr uint32_t RBLOCK = RTBVH_REFIT_BLOCK;
#ifndef RTBVH_REFIT_PROBE
#define RTBVH_REFIT_PROBE 0   // A/B probe builds (-DRTBVH_AB_BUILD): 1 no QNode computed, 3 no phase-4 stores,
                              // 4 no leaf-record stores, 5 no leaf margin / footprint (wrong trees: timing only)
#endif
#ifndef RTBVH_QSKIP
#define RTBVH_QSKIP 1   // k_refit writes only the QNodes the 4-wide walk reads (0: all, A/B)
#endif
#ifndef RTBVH_REFIT_STAGE_SLOTS
#define RTBVH_REFIT_STAGE_SLOTS 512   // slots per phase-4 round (32 KB; C4 A/B: 256 and 512 alike, 1024 slower)
#endif

__device__ __forceinline__ uint32_t expand_bits(uint32_t var) {   // MortonCodes.hlsl:13-31
    var &= 0x000003ffu; var |= var << 16;
    var &= 0x030000ffu; var |= var << 8;
    var &= 0x0300f00fu; var |= var << 4;
    var &= 0x030c30c3u; var |= var << 2;
    return var & 0x09249249u;
}
// Morton Code/main.cpp:84-92 (CPUTests) -- NaN quantises to 0
__device__ __forceinline__ uint32_t quantise_cputests(float p) {
    p *= 1024.f;
    if (p < 0) p = 0;
    else if (p >= 1024) p = 1023;
    if (p != p) return 0u;
    return (uint32_t)p;
}
// MortonCodes.hlsl:42-47: clamp(p, 0, 1023) = min(max(p, 0), 1023)
__device__ __forceinline__ uint32_t quantise_hlsl(float p) {
    p *= 1024.f;
    p = fminf(fmaxf(p, 0.0f), 1023.0f);
    return (uint32_t)p;
}

// Scene AABB of the object-space vertices (ShaderSim/main.cpp:277-285), two launches
// without global atomics: per-block partials (wave shuffles + LDS), then one block
// reduces the partials.  bounds layout: [0..5] = min xyz, max xyz; [8..] partials.
constexpr uint32_t BOUNDS_BLOCKS = 1024;

__device__ __forceinline__ void reduce_box_block(f3& mn, f3& mx, float* s_red /*4*6*/) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mn.x = fminf(mn.x, __shfl_xor(mn.x, off, 64));
        mn.y = fminf(mn.y, __shfl_xor(mn.y, off, 64));
        mn.z = fminf(mn.z, __shfl_xor(mn.z, off, 64));
        mx.x = fmaxf(mx.x, __shfl_xor(mx.x, off, 64));
        mx.y = fmaxf(mx.y, __shfl_xor(mx.y, off, 64));
        mx.z = fmaxf(mx.z, __shfl_xor(mx.z, off, 64));
    }
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_red[6 * w + 0] = mn.x; s_red[6 * w + 1] = mn.y; s_red[6 * w + 2] = mn.z;
        s_red[6 * w + 3] = mx.x; s_red[6 * w + 4] = mx.y; s_red[6 * w + 5] = mx.z;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; k++) {
            mn = vmin(mn, mk(s_red[6 * k + 0], s_red[6 * k + 1], s_red[6 * k + 2]));
            mx = vmax(mx, mk(s_red[6 * k + 3], s_red[6 * k + 4], s_red[6 * k + 5]));
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_bounds(const float4* __restrict__ opos, uint32_t V, float* __restrict__ bounds) {
    __shared__ float s_red[24];
    f3 mn = mk(INFINITY, INFINITY, INFINITY), mx = mk(-INFINITY, -INFINITY, -INFINITY);
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < V; i += (size_t)gridDim.x * BLOCK) {
        const float4 p = opos[i];
        mn = vmin(mn, mk(p.x, p.y, p.z));
        mx = vmax(mx, mk(p.x, p.y, p.z));
    }
    reduce_box_block(mn, mx, s_red);
    if (threadIdx.x == 0) {
        float* o = bounds + 8 + 6 * (size_t)blockIdx.x;
        o[0] = mn.x; o[1] = mn.y; o[2] = mn.z; o[3] = mx.x; o[4] = mx.y; o[5] = mx.z;
    }
}

__global__ __launch_bounds__(BLOCK) void k_bounds_final(float* __restrict__ bounds, uint32_t nparts) {
    __shared__ float s_red[24];
    f3 mn = mk(INFINITY, INFINITY, INFINITY), mx = mk(-INFINITY, -INFINITY, -INFINITY);
    for (uint32_t i = threadIdx.x; i < nparts; i += BLOCK) {
        const float* p = bounds + 8 + 6 * (size_t)i;
        mn = vmin(mn, mk(p[0], p[1], p[2]));
        mx = vmax(mx, mk(p[3], p[4], p[5]));
    }
    reduce_box_block(mn, mx, s_red);
    if (threadIdx.x == 0) {
        bounds[0] = mn.x; bounds[1] = mn.y; bounds[2] = mn.z;
        bounds[3] = mx.x; bounds[4] = mx.y; bounds[5] = mx.z;
    }
}

// MortonCodes.hlsl:54-125 (HLSL mode) / ShaderSim/main.cpp:292-301 (CPUTests mode):
// triangle t's code (also stored in keys/vals) and its clip-space triangle
__device__ __forceinline__ uint32_t morton_code(const BuildArgs& a, uint32_t t, float4 (&clip)[4]) {
    const uint32_t i0 = a.idx[3 * (size_t)t], i1 = a.idx[3 * (size_t)t + 1], i2 = a.idx[3 * (size_t)t + 2];
    const float4 q0 = a.opos[i0], q1 = a.opos[i1], q2 = a.opos[i2];
    const f3 p0 = mk(q0.x, q0.y, q0.z), p1 = mk(q1.x, q1.y, q1.z), p2 = mk(q2.x, q2.y, q2.z);
    const f3 c0 = xform_point(a.cam, p0), c1 = xform_point(a.cam, p1), c2 = xform_point(a.cam, p2);
    uint32_t code;
    if (a.morton_mode == 0) {
        const f3 mn = mk(a.bounds[0], a.bounds[1], a.bounds[2]);
        const f3 mx = mk(a.bounds[3], a.bounds[4], a.bounds[5]);
        const float xv = p0.x + p1.x + p2.x, yv = p0.y + p1.y + p2.y, zv = p0.z + p1.z + p2.z;
        const uint32_t qx = quantise_cputests((xv / 3.f - mn.x) / (mx.x - mn.x));
        const uint32_t qy = quantise_cputests((yv / 3.f - mn.y) / (mx.y - mn.y));
        const uint32_t qz = quantise_cputests((zv / 3.f - mn.z) / (mx.z - mn.z));
        code = expand_bits(qz) | expand_bits(qy) << 1 | expand_bits(qx) << 2;
    } else {
        f3 bmin = vmin(c0, c1);
        bmin = vmin(bmin, c2);   // avg == bbMin after the loop (MortonCodes.hlsl:98 bug)
        const f3 avg = mk(bmin.x / 3.f, bmin.y / 3.f, bmin.z / 3.f);
        const uint32_t qx = quantise_hlsl((avg.x - a.smin[0]) / (a.smax[0] - a.smin[0]));
        const uint32_t qy = quantise_hlsl((avg.y - a.smin[1]) / (a.smax[1] - a.smin[1]));
        const uint32_t qz = quantise_hlsl((avg.z - a.smin[2]) / (a.smax[2] - a.smin[2]));
        code = expand_bits(qx) | expand_bits(qy) << 1 | expand_bits(qz) << 2;
    }
    a.keys[t] = code;
    a.vals[t] = t;
    clip[0] = make_float4(c0.x, c0.y, c0.z, __uint_as_float(t));
    clip[1] = make_float4(c1.x, c1.y, c1.z, 0.f);
    clip[2] = make_float4(c2.x, c2.y, c2.z, 0.f);
    // the shading's gathers in one record: the vertex indices and the material index
    clip[3] = make_float4(__uint_as_float(i0), __uint_as_float(i1), __uint_as_float(i2), __uint_as_float(a.matidx[t]));
    return code;
}
__device__ __forceinline__ uint32_t morton_tri(const BuildArgs& a, uint32_t t) {
    float4 clip[4];
    const uint32_t code = morton_code(a, t, clip);
    float4* o = a.tclip + TCS * (size_t)t;
    o[0] = clip[0]; o[1] = clip[1]; o[2] = clip[2];
    if (TCS == 4) o[3] = clip[3];
    return code;
}
// One thread per triangle; the 48-B clip-space triangles of a wave (3 KB contiguous) are staged
// in LDS and stored 16 B per lane (scripts/write_roofline.hip: 4.1 TB/s against 2.5-2.9 for a
// whole record per lane).
__global__ __launch_bounds__(BLOCK) void k_morton(BuildArgs a) {
    __shared__ float4 s_clip[BLOCK / 64][TCS * 64];
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    if (t < a.T) {
        float4 clip[4];
        morton_code(a, t, clip);
#pragma unroll
        for (int k = 0; k < 3; k++) s_clip[w][TCS * lane + k] = clip[k];
        if (TCS == 4) s_clip[w][TCS * lane + 3] = clip[3];
    }
    __syncthreads();
    const uint32_t t0 = t - lane;   // the wave's first triangle
    const uint32_t n = a.T > t0 ? min(64u, a.T - t0) : 0u;
    float4* dst = a.tclip + TCS * (size_t)t0;
#pragma unroll
    for (uint32_t k = 0; k < TCS; k++)
        if (64 * k + lane < TCS * n) st_out<1>(dst + 64 * k + lane, s_clip[w][64 * k + lane]);
}

// ---- Karras 2012 (BVHConstructP1.hlsl:61-165) --------------------------------
// `c` is the sorted code sequence: a pointer, or an accessor c(j) (the one-workgroup build
// reads the codes from LDS)
// Indices are 32-bit: set_scene takes T < 2^30, so every probe I + k * d of the searches below
// (k <= 2^30: the doubling stops at the first probe outside [0, T)) lies in (-2^31, 2^31), and
// one unsigned compare is the range test (a negative j wraps above n).
template <class C>
__device__ __forceinline__ uint32_t code_at(const C& c, int32_t j) { return c[j]; }

// Branch-free (selects, one code read at a clamped index): the searches' lanes probe different
// j, and a divergent early return or tie branch cost the wave both paths on every probe.
template <class C>
__device__ __forceinline__ int delta_clz64(const C& c, uint32_t n, uint32_t i, uint32_t ci, int32_t j) {
    const bool in = (uint32_t)j < n;   // leadingPrefixBounds :78-84: -1 outside
    const uint32_t jj = in ? (uint32_t)j : i;
    const uint32_t x = ci ^ code_at(c, (int32_t)jj), y = i ^ jj;
    int rx = (int)__clz((int)x), ry = 32 + (int)__clz((int)y);
    asm volatile("" : "+v"(rx), "+v"(ry));   // both computed, then selected (not a divergent branch)
    return in ? (x != 0u ? rx : ry) : -1;
}
__device__ __forceinline__ int debruijn_lz(uint32_t data) {   // RadixBVHCombo/main.cpp:136-151
    const int tbl[32] = {0, 31, 9, 30, 3, 8, 13, 29, 2, 5, 7, 21, 12, 24, 28, 19,
                         1, 10, 4, 14, 6, 22, 25, 20, 11, 15, 23, 26, 16, 27, 17, 18};
    data |= data >> 1; data |= data >> 2; data |= data >> 4; data |= data >> 8; data |= data >> 16;
    data++;
    return data ? tbl[(uint32_t)(data * 0x076be629u) >> 27] : 32;
}
template <class C>
__device__ __forceinline__ int delta_cputests(const C& c, uint32_t n, uint32_t i, uint32_t ci, int32_t j) {
    if ((uint32_t)j >= n) return -1;
    const uint32_t cj = code_at(c, j);
    return debruijn_lz(ci == cj ? (i ^ (uint32_t)j) : (ci ^ cj));
}

template <int MODE, class C>
__device__ __forceinline__ int delta(const C& c, uint32_t n, uint32_t i, uint32_t ci, int32_t j) {
    return MODE == 0 ? delta_clz64(c, n, i, ci, j) : delta_cputests(c, n, i, ci, j);
}

template <int MODE, class C>
__device__ void karras_node(const C& c, uint32_t n, uint32_t i, uint4* __restrict__ topo,
                            uint32_t* __restrict__ pleaf, uint32_t* __restrict__ pint) {
    const uint32_t N = n;
    const int32_t I = (int32_t)i;
    const uint32_t ci = code_at(c, I);
    const int32_t d = delta<MODE>(c, N, i, ci, I + 1) < delta<MODE>(c, N, i, ci, I - 1) ? -1 : 1;
    const int min_lz = delta<MODE>(c, N, i, ci, I - d);
    int32_t bound_len = 2;
    while (min_lz < delta<MODE>(c, N, i, ci, I + bound_len * d)) bound_len <<= 1;
    int32_t dl = bound_len, dsum = 0;
    do {
        dl = (dl + 1) >> 1;
        if (min_lz < delta<MODE>(c, N, i, ci, I + (dsum + dl) * d)) dsum += dl;
    } while (1 < dl);
    const int32_t bound_start = I + dsum * d;
    const int lz = delta<MODE>(c, N, i, ci, bound_start);
    dl = dsum;
    int32_t tmp = 0;
    do {
        dl = (dl + 1) >> 1;
        if (lz < delta<MODE>(c, N, i, ci, I + (tmp + dl) * d)) tmp += dl;
    } while (1 < dl);
    const int32_t loc = I + tmp * d + (d < 0 ? d : 0);
    const bool left_leaf = (I < bound_start ? I : bound_start) == loc;
    const bool right_leaf = (I > bound_start ? I : bound_start) == loc + 1;
    const uint32_t l = (uint32_t)loc, r = (uint32_t)(loc + 1);
    topo[i] = make_uint4(left_leaf ? (LEAF_BIT | l) : l, right_leaf ? (LEAF_BIT | r) : r,
                         (uint32_t)(I < bound_start ? I : bound_start),    // leaf range of node i
                         (uint32_t)(I > bound_start ? I : bound_start));
    if (left_leaf) pleaf[l] = i << 1; else pint[l] = i << 1;
    if (right_leaf) pleaf[r] = (i << 1) | 1u; else pint[r] = (i << 1) | 1u;
}

// the leaf record's word 9: the triangle index, bit 31 set when the leaf box needs the general slab
// test for axis-parallel primary rays (the same rule as general_box below; the primary walk
// re-tests a leaf's box before its triangle, trace.hip traverse_packet4)
__device__ __forceinline__ uint32_t leaf_tri_word(uint32_t t, f3 lo, f3 hi) {
    const bool fast = lo.x < hi.x && lo.y < hi.y && lo.z <= hi.z && 0.f <= hi.z && hi.z < INFINITY;
    return t | (fast ? 0u : LEAF_BIT);
}
// leaf record of sorted position i: gather the clip-space triangle once, store
// (v0, e1, e2) for the triangle test (the reference's edge1/edge2, :43-44) and
// the leaf AABB (MortonCodes.hlsl:87-96: min/max of v0, v1, v2 in that order)
__device__ __forceinline__ void leaf_record_words_of(const BuildArgs& a, uint32_t t, f3& lo, f3& hi, float4 (&r)[4]) {
    const float4* src = a.tclip + TCS * (size_t)t;
    const float4 s0 = src[0], s1 = src[1], s2 = src[2];
    const f3 v0 = mk(s0.x, s0.y, s0.z), v1 = mk(s1.x, s1.y, s1.z), v2 = mk(s2.x, s2.y, s2.z);
    const f3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    lo = vmin(v0, v1);
    hi = vmax(v0, v1);
    lo = vmin(lo, v2);
    hi = vmax(hi, v2);
    r[0] = make_float4(v0.x, v0.y, v0.z, e1.x);
    r[1] = make_float4(e1.y, e1.z, e2.x, e2.y);
    r[2] = make_float4(e2.z, __uint_as_float(leaf_tri_word(t, lo, hi)), lo.x, lo.y);
    r[3] = make_float4(lo.z, hi.x, hi.y, hi.z);
}
__device__ __forceinline__ void leaf_record_words(const BuildArgs& a, uint32_t i, f3& lo, f3& hi, float4 (&r)[4]) {
    leaf_record_words_of(a, a.sorted_vals[i], lo, hi, r);
}
// 64-B records of consecutive indices, one per lane, written with every store instruction of
// the wave covering 1 KB contiguously (16 B per lane): each half-wave's records are staged in
// LDS (`buf`: 128 float4 of this wave's own) and read back transposed.  MI355X (scripts/
// write_roofline.hip): 16-B-per-lane stores stream at 4.1 TB/s, a 64-B record per lane at
// 2.5-2.9 TB/s.  `n` records start at dst (lanes >= n hold none); the whole block calls it.
__device__ __forceinline__ void staged_records(float4* __restrict__ dst, uint32_t n, const float4 (&r)[4],
                                               float4* buf) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
        if ((lane >> 5) == h) {
#pragma unroll
            for (int k = 0; k < 4; k++) buf[4 * (lane & 31u) + k] = r[k];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t m = 0; m < 2; m++) {
            const uint32_t w = lane + 64 * m;                   // float4 w of this half-wave's 32 records
            if (32 * h + (w >> 2) < n) st_out<2>(dst + 128 * h + w, buf[w]);
        }
        __syncthreads();
    }
}
// BVHConstructP1.hlsl:167-188: internal node i for every i < T-1 (topology only: child ids,
// leaf range, parent links); the root's parent is UINT_MAX (:186-187).  The leaf records are
// written by the refit (k_refit), which gathers each leaf's triangle once.
#ifndef RTBVH_KARRAS_WIN
#define RTBVH_KARRAS_WIN 256
#endif
// The sorted codes a workgroup's searches touch most -- the neighbourhood of its 256 nodes:
// the deep nodes' ranges are short -- are staged in LDS (a window of KWIN codes either side);
// codes outside the window come from global memory.
constexpr int64_t KWIN = RTBVH_KARRAS_WIN;
// the window lives in a file-scope LDS array so that its reads compile to ds_read (through a
// generic pointer kept in the accessor they were flat loads, 8 per node)
__shared__ uint32_t s_kwin[BLOCK + 2 * (KWIN > 0 ? KWIN : 0)];
struct WindowCodes {
    const uint32_t* g;
    int32_t lo, hi;   // the window [lo, hi) of the code sequence held in s_kwin
    __device__ uint32_t operator[](int32_t j) const {
        const bool in = (uint32_t)(j - lo) < (uint32_t)(hi - lo);
        uint32_t v = s_kwin[in ? j - lo : 0];   // every lane reads LDS; the few outside also global
        asm volatile("" : "+v"(v));   // keeps the two loads apart (merged: one flat load of a selected pointer)
        if (!in) v = g[j];
        return v;
    }
};
template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_karras(BuildArgs a) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (KWIN > 0) {
        const int64_t base = (int64_t)blockIdx.x * BLOCK;
        const int64_t lo = base - KWIN > 0 ? base - KWIN : 0;
        const int64_t hi = base + BLOCK + KWIN < (int64_t)a.T ? base + BLOCK + KWIN : (int64_t)a.T;
        for (int64_t j = lo + threadIdx.x; j < hi; j += BLOCK) s_kwin[j - lo] = a.sorted_keys[j];
        __syncthreads();
        const WindowCodes codes{a.sorted_keys, (int32_t)lo, (int32_t)hi};
        if (i + 1 < a.T) karras_node<MODE>(codes, a.T, i, a.topo, a.pleaf, a.pint);
    } else {
        if (i + 1 < a.T) karras_node<MODE>(a.sorted_keys, a.T, i, a.topo, a.pleaf, a.pint);
    }
    if (i == 0 && a.T > 1) a.pint[0] = INVALID;
}

// ---- refit (BVHConstructP2.hlsl:8-37) -----------------------------------------
// One thread per leaf climbs; a per-node ticket makes the second arriver union
// both child boxes.  Each box is stored into its parent's 64-B record (side 0/1)
// BEFORE the ticket.  Cross-CU / cross-XCD visibility without a release fence per
// step (an acq_rel RMW writes back the XCD's whole L2 each time: 43 ms at 10M):
// the box bytes are written with agent-scope (sc1, write-through) 8-B stores, the
// storing lane drains them (s_waitcnt vmcnt(0)) before its relaxed agent-scope
// ticket add, and the second arriver -- told by the value its add returned --
// reads the sibling box only with agent-scope (sc1) loads.  This is row 1 of the
// valid hand-off forms of MI355X_MICROARCH.md §"Workgroup dispatch ... visibility".
__device__ __forceinline__ void st_box_sc1(float* dst, f3 lo, f3 hi) {
    uint64_t* d = reinterpret_cast<uint64_t*>(dst);   // 8-B aligned: record offset 0 or 24
    __hip_atomic_store(d + 0, ((uint64_t)__float_as_uint(lo.y) << 32) | __float_as_uint(lo.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d + 1, ((uint64_t)__float_as_uint(hi.x) << 32) | __float_as_uint(lo.z), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d + 2, ((uint64_t)__float_as_uint(hi.z) << 32) | __float_as_uint(hi.y), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ld_box_sc1(const float* src, f3& lo, f3& hi) {
    const uint64_t* s = reinterpret_cast<const uint64_t*>(src);
    const uint64_t a = __hip_atomic_load(s + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load(s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t c = __hip_atomic_load(s + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lo = mk(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)), __uint_as_float((uint32_t)b));
    hi = mk(__uint_as_float((uint32_t)(b >> 32)), __uint_as_float((uint32_t)c), __uint_as_float((uint32_t)(c >> 32)));
}

// the complete record of node p (word layout: rtbvh_device.h "node record"): its
// children's boxes with each corner's (x, y) as an aligned pair, their ids, p itself
// Word 15 bit s: child s's box needs the general slab test in the axis-parallel primary
// walk (trace.hip traverse_packet4 AXIS).  Every box with min < max in x and y,
// min.z <= max.z and 0 <= max.z < inf takes the exact compare-only form of ray_box_xy for
// rays along +z from z = 0 (NaN fails a compare; infinite x/y corners and min.z give the
// slab signs the general test gives; max.z = +inf could let the general test report a hit
// at t = +inf with an empty slab).
__device__ __forceinline__ uint32_t general_box(f3 lo, f3 hi) {
    return lo.x < hi.x && lo.y < hi.y && lo.z <= hi.z && 0.f <= hi.z && hi.z < INFINITY ? 0u : 1u;
}
__device__ __forceinline__ void record_words(f3 lmin, f3 lmax, f3 rmin, f3 rmax, uint32_t cl, uint32_t cr, uint32_t own,
                                             float4 (&d)[4]) {
    const uint32_t gen = general_box(lmin, lmax) | general_box(rmin, rmax) << 1;
    d[0] = make_float4(lmin.x, lmin.y, lmax.x, lmax.y);
    d[1] = make_float4(rmin.x, rmin.y, rmax.x, rmax.y);
    d[2] = make_float4(lmin.z, lmax.z, rmin.z, rmax.z);
    d[3] = make_float4(__uint_as_float(cl), __uint_as_float(cr), __uint_as_float(own), __uint_as_float(gen));
}
__device__ __forceinline__ void store4(void* dst, const float4 (&w)[4]) {
    float4* d = reinterpret_cast<float4*>(dst);
    d[0] = w[0]; d[1] = w[1]; d[2] = w[2]; d[3] = w[3];
}
__device__ __forceinline__ void store_record(Inner* dst, f3 lmin, f3 lmax, f3 rmin, f3 rmax, uint32_t cl,
                                             uint32_t cr, uint32_t own) {
    float4 w[4];
    record_words(lmin, lmax, rmin, rmax, cl, cr, own, w);
    store4(dst, w);
}
// box of child `side` from a node record: min xyz, max xyz
__device__ __forceinline__ void record_box(const Inner* r, uint32_t side, float out[6]) {
    const float* w = reinterpret_cast<const float*>(r);
    const int b = side ? 4 : 0, z = side ? 10 : 8;
    out[0] = w[b]; out[1] = w[b + 1]; out[2] = w[z];
    out[3] = w[b + 2]; out[4] = w[b + 3]; out[5] = w[z + 1];
}
__device__ __forceinline__ uint32_t slot_of(uint32_t parent_code, uint32_t T) {
    return parent_code == INVALID ? 2 * T - 2 : parent_code;
}

// The pseudo-record of leaf j (rtbvh_device.h: the 4-wide walks read a leaf child's slot as a
// record whose two children are the leaf itself and nothing).  The absent second child repeats
// the box with a NaN min.z, which fails the primary walk's fast test (min.z <= bound) for every
// lane, so that walk needs no id check; both bits of word 15 are the leaf box's own.
__device__ __forceinline__ void pseudo_words(uint32_t leaf_id, f3 lo, f3 hi, float4 (&d)[4]) {
    const uint32_t gen = general_box(lo, hi) * 3u;
    d[0] = make_float4(lo.x, lo.y, hi.x, hi.y);
    d[1] = make_float4(lo.x, lo.y, hi.x, hi.y);
    d[2] = make_float4(lo.z, hi.z, __uint_as_float(ABSENT_MINZ), hi.z);
    d[3] = make_float4(__uint_as_float(leaf_id), __uint_as_float(INVALID), __uint_as_float(leaf_id),
                       __uint_as_float(gen));
}
__device__ __forceinline__ void store_pseudo_record(Inner* dst, uint32_t leaf_id, f3 lo, f3 hi) {
    float4 w[4];
    pseudo_words(leaf_id, lo, hi, w);
    store4(dst, w);
}
__device__ __forceinline__ void store_leaf_record(Inner* rec, uint32_t p, uint32_t side, uint32_t leaf_id, f3 lo,
                                                  f3 hi) {
    store_pseudo_record(rec + 2 * (size_t)p + side, leaf_id, lo, hi);
}

// The node boxes of a build without records (BuildArgs::nbox, rtbvh_internal.h): internal node k's box, min xyz
// then max xyz, 24 B at nbox + 6 k (three 8-B stores: consecutive nodes' threads write consecutive bytes)
__device__ __forceinline__ void st_nbox(float* nbox, uint32_t k, f3 lo, f3 hi) {
    float2* d = reinterpret_cast<float2*>(nbox + 6 * (size_t)k);
    d[0] = make_float2(lo.x, lo.y);
    d[1] = make_float2(lo.z, hi.x);
    d[2] = make_float2(hi.y, hi.z);
}
__device__ __forceinline__ void ld_nbox(const float* nbox, uint32_t k, float (&b)[6]) {
    const float2* d = reinterpret_cast<const float2*>(nbox + 6 * (size_t)k);
    const float2 x = d[0], y = d[1], z = d[2];
    b[0] = x.x; b[1] = x.y; b[2] = y.x; b[3] = y.y; b[4] = z.x; b[5] = z.y;
}
// the box of child c (internal node, or LEAF_BIT | j: its leaf record's words 10..15)
__device__ __forceinline__ void child_box(const BuildArgs& a, uint32_t c, float (&b)[6]) {
    if (c & LEAF_BIT) {
        const float4* r = a.leaf + 4 * (size_t)(c & ~LEAF_BIT);
        const float4 w2 = r[2], w3 = r[3];
        b[0] = w2.z; b[1] = w2.w; b[2] = w3.x; b[3] = w3.y; b[4] = w3.z; b[5] = w3.w;
    } else {
        ld_nbox(a.nbox, c, b);
    }
}

// A node of the climb is complete: its record (both children's boxes) at its slot, the
// pseudo-records of its leaf children; returns its box, the union in (childL, childR)
// order as the reference's min(L.bbMin, R.bbMin).
__device__ __forceinline__ void complete_node(const BuildArgs& a, uint32_t p, uint32_t e, f3 l0, f3 l1, f3 r0, f3 r1,
                                              f3& lo, f3& hi) {
    const uint4 ids = a.topo[p];
    if (a.rec_on) {
        store_record(a.rec + slot_of(e, a.T), l0, l1, r0, r1, ids.x, ids.y, p);
        if (a.pseudo && (ids.x & LEAF_BIT)) store_leaf_record(a.rec, p, 0, ids.x, l0, l1);
        if (a.pseudo && (ids.y & LEAF_BIT)) store_leaf_record(a.rec, p, 1, ids.y, r0, r1);
    }
    lo = vmin(l0, r0);
    hi = vmax(l1, r1);
    if (a.nbox) st_nbox(a.nbox, p, lo, hi);
    if (e == INVALID) {
        a.rootbox[0] = lo.x; a.rootbox[1] = lo.y; a.rootbox[2] = lo.z;
        a.rootbox[3] = hi.x; a.rootbox[4] = hi.y; a.rootbox[5] = hi.z;
    }
}

// The largest leaf edge bound below a node (margin.h: its QNode's margin codes).  Where a QNode is
// built from the records (k_qnodes_late, k_qnodes) it is read from inner[k].aux0, written by
// whoever completes node k outside k_refit's in-block climb (refit_climb, refit_top_node,
// k_build_small); inner[p].child_l / child_r carry a child's bound through the climb's hand-off,
// beside its box (the hand-off uses no other word of inner[p]).
__device__ __forceinline__ float* hand_edge(const BuildArgs& a, uint32_t p, uint32_t side) {
    return reinterpret_cast<float*>(&a.inner[p].child_l) + side;
}
__device__ __forceinline__ float* node_edge(const BuildArgs& a, uint32_t k) {
    return reinterpret_cast<float*>(&a.inner[k].aux0);
}
__device__ __forceinline__ void st_edge_sc1(float* dst, float E) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(dst), __float_as_uint(E), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_edge_sc1(const float* src) {
    return __uint_as_float(
        __hip_atomic_load(reinterpret_cast<const uint32_t*>(src), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// The global climb, for the nodes whose leaf range crosses a refit workgroup: from a complete
// node (box lo, hi, edge bound em; e = its parent link) upward, the child box and bound handed
// over through inner[p] (sc1) and a per-node ticket; the second arriver completes p and goes on.
// k_qnodes_late quantizes these nodes afterwards.
__device__ __forceinline__ void refit_climb(f3 lo, f3 hi, float em, uint32_t e, const BuildArgs& a) {
    // a clz64 tree is at most 64 levels deep; the bound only stops a CPUTests-delta
    // tree with a parent cycle from spinning forever
    for (int level = 0; e != INVALID && level < 2 * STACK_SIZE; level++) {
        const uint32_t p = e >> 1, side = e & 1u;
        st_box_sc1(side ? a.inner[p].rmin : a.inner[p].lmin, lo, hi);
        st_edge_sc1(hand_edge(a, p, side), em);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain the box stores before the ticket
        const uint32_t old = __hip_atomic_fetch_add(&a.refit_cnt[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == 0) return;
        asm volatile("" ::: "memory");
        f3 smin, smax;
        ld_box_sc1(side ? a.inner[p].lmin : a.inner[p].rmin, smin, smax);
        em = fmaxf(em, ld_edge_sc1(hand_edge(a, p, side ^ 1u)));
        *node_edge(a, p) = em;   // (read by k_qnodes_late / k_qnodes, later launches)
        e = a.pint[p];
        if (side) complete_node(a, p, e, smin, smax, lo, hi, lo, hi);
        else      complete_node(a, p, e, lo, hi, smin, smax, lo, hi);
    }
}

// crossing: node k's leaf range is not inside the refit workgroup of its index (k_refit's block)
__device__ __forceinline__ bool crossing(uint4 topo_k, uint32_t k) {
    const uint32_t base = k & ~(RBLOCK - 1);
    return !(topo_k.z >= base && topo_k.w < base + RBLOCK);
}

// ---- quantized 4-wide nodes (rtbvh_device.h QNode) ---------------------------------
// One axis of a QNode: the grid origin o = the min of the four boxes, the step s = the
// smallest power of two >= 2^-120 with o + 255 s >= their max in fp32, and for each box
// the largest lo and smallest hi byte whose decoded corners (qdecode, the traversal's own
// arithmetic) still contain it.  false: no finite frame (the node keeps the exact record
// pair).  Division-free: s and 1/s are built from exponent bits (both normal: s is in
// [2^-120, 2^94] for |corners| <= 2^100), so (x - o) * (1/s) is exactly (x - o) / s.
// PMC: the first form (correctly rounded divisions, frexpf/ldexpf) ran ~3,500 VALU per
// node and made the QNode pass VALU-bound (0.90 ms at 10M nodes).
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((uint32_t)(e + 127) << 23); }
__device__ __forceinline__ bool quantize_axis(const float (&lo)[4], const float (&hi)[4], float& org, float& scl,
                                              uint32_t& wlo, uint32_t& whi) {
    float o = lo[0], m = hi[0];
    for (int c = 1; c < 4; c++) {
        o = fminf(o, lo[c]);
        m = fmaxf(m, hi[c]);
    }
    const float ext = m - o;
    // corners within 2^100 (also excludes NaN): the bounce walk's slack test (trace.hip
    // qbox_fast) then stays finite for every ray it takes (|o| <= 2^90, |1/d| <= 2^20)
    if (!(fabsf(o) <= 0x1p100f && fabsf(m) <= 0x1p100f && ext <= 0x1p100f)) return false;
    // ext in [2^E, 2^(E+1)): 255 * 2^(E-8) < ext, so the smallest valid step is >= 2^(E-8)
    int e = -120;
    if (ext > 0.f) {
        const int E = (int)((__float_as_uint(ext) >> 23) & 255u) - 127;   // ext >= 0; denormal: E = -127
        e = max(E - 8, -120);
    }
    while (fmaf(255.f, pow2f(e), o) < m) ++e;   // the rounding of the add (a few steps at most)
    const float s = pow2f(e), rs = pow2f(-e);
    wlo = whi = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t l = (uint32_t)fminf(fmaxf(floorf((lo[c] - o) * rs), 0.f), 255.f);
        uint32_t h = (uint32_t)fminf(fmaxf(ceilf((hi[c] - o) * rs), 0.f), 255.f);
        if (l > 0 && fmaf((float)l, s, o) > lo[c]) --l;     // the rounding of the subtraction: q = 0
        if (h < 255 && fmaf((float)h, s, o) < hi[c]) ++h;   // decodes to o <= lo[c], 255 to >= m
        wlo |= l << (8 * c);
        whi |= h << (8 * c);
    }
    org = o;
    scl = s;
    return true;
}

// the QNode of a node from its four grandchild boxes (x/y/z min and max per grandchild c), ids and
// the largest edge bound of the leaves below it (E, margin.h: its codes in the low 16 bits of the
// power-of-two steps scl[1], scl[2]), written as four 16-B stores
__device__ __forceinline__ void qnode_words(const float (&lx)[4], const float (&ly)[4], const float (&lz)[4],
                                            const float (&hx)[4], const float (&hy)[4], const float (&hz)[4], uint4 ids,
                                            float E, float4 (&d)[4]) {
    QNode q;
    bool ok = quantize_axis(lx, hx, q.org[0], q.scl[0], q.lo[0], q.hi[0]);
    ok = quantize_axis(ly, hy, q.org[1], q.scl[1], q.lo[1], q.hi[1]) && ok;
    ok = quantize_axis(lz, hz, q.org[2], q.scl[2], q.lo[2], q.hi[2]) && ok;
    if (!ok) {
        q.scl[0] = 0.f;   // the traversal reads the exact pair for this node
    } else if (E >= 0.f || E != E) {   // (E < 0: the caller adds the codes, qnode_codes)
        uint32_t ce, ct;
        mt_node_codes(E, ce, ct);
        q.scl[1] = __uint_as_float(__float_as_uint(q.scl[1]) | ce);
        q.scl[2] = __uint_as_float(__float_as_uint(q.scl[2]) | ct);
    }
    q.id[0] = ids.x; q.id[1] = ids.y; q.id[2] = ids.z; q.id[3] = ids.w;
    const float4* qs = reinterpret_cast<const float4*>(&q);
    d[0] = qs[0]; d[1] = qs[1]; d[2] = qs[2]; d[3] = qs[3];
}

// the margin codes into QNode words (qnode_words with E < 0 left them out)
__device__ __forceinline__ void qnode_codes(float4 (&d)[4], float E) {
    if (d[0].w == 0.f) return;
    uint32_t ce, ct;
    mt_node_codes(E, ce, ct);
    d[1].x = __uint_as_float(__float_as_uint(d[1].x) | ce);
    d[1].y = __uint_as_float(__float_as_uint(d[1].y) | ct);
}

// ---- the grouping of a QNode (greedy collapse) ------------------------------------
// A QNode holds up to four subtrees that partition its node's subtree.  Starting from the
// node's two children, the internal entry with the largest box surface is replaced by its two
// children, twice (fewer when the subtree runs out of internal nodes): the grouping a BVH4
// collapse by largest area makes, so every QNode of a node with >= 4 leaves is full and the
// entries are of similar size.  (The first form took the four grandchildren, a leaf child
// counting once: ~half the QNodes near the leaves held 2-3 entries.)  The walk's result does
// not depend on the grouping: every entry's box is the exact union of its subtree's leaves.
struct QEnt {
    uint32_t id;     // internal node index, or LEAF_BIT | j
    uint32_t slot;   // where the entry's record / QNode lives (2 * parent + side)
    float b[6];      // box: min xyz, max xyz
};
__device__ __forceinline__ float half_area(const float (&b)[6]) {
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;   // NaN boxes compare false: never expanded
}
__device__ __forceinline__ void qent_sel(QEnt& d, const QEnt& s, bool take) {
    d.id = take ? s.id : d.id;
    d.slot = take ? s.slot : d.slot;
#pragma unroll
    for (int k = 0; k < 6; k++) d.b[k] = take ? s.b[k] : d.b[k];
}
// Kids(e, c0, c1): the two children of internal entry e
template <class Kids>
__device__ __forceinline__ void greedy_qnode_words(const QEnt& e0, const QEnt& e1, Kids&& kids, float edge,
                                                   float4 (&out)[4], uint32_t (&ent)[4]) {
    QEnt E[4] = {e0, e1, e0, e0};
    uint32_t n = 2;
#pragma unroll
    for (int step = 0; step < 2; step++) {
        int pick = -1;
        float best = -1.f;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            if ((uint32_t)k < n && !(E[k].id & LEAF_BIT)) {
                const float ar = half_area(E[k].b);
                if (ar > best) { best = ar; pick = k; }
            }
        }
        if (pick < 0) break;
        QEnt sel = E[0];
#pragma unroll
        for (int k = 1; k < 3; k++) qent_sel(sel, E[k], k == pick);
        QEnt c0, c1;
        kids(sel, c0, c1);
#pragma unroll
        for (int k = 0; k < 3; k++) qent_sel(E[k], c0, k == pick);
        qent_sel(E[2], c1, n == 2);
        qent_sel(E[3], c1, n == 3);
        ++n;
    }
    // positions: 4 entries in order; 3 -> the fourth absent; 2 -> at 0 and 2 (1 and 3 absent:
    // the walk masks only positions 1 and 3 by their INVALID id).  An absent entry repeats box 0.
    QEnt P[4] = {E[0], E[1], E[2], E[3]};
    if (n == 2) { P[1] = E[0]; P[2] = E[1]; P[3] = E[0]; }
    if (n == 3) P[3] = E[0];
    const bool absent1 = n == 2, absent3 = n < 4;
    float lx[4], ly[4], lz[4], hx[4], hy[4], hz[4];
    uint32_t id[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        lx[k] = P[k].b[0]; ly[k] = P[k].b[1]; lz[k] = P[k].b[2];
        hx[k] = P[k].b[3]; hy[k] = P[k].b[4]; hz[k] = P[k].b[5];
        id[k] = (P[k].id & LEAF_BIT) ? P[k].id : P[k].slot;
    }
    if (absent1) id[1] = INVALID;
    if (absent3) id[3] = INVALID;
#pragma unroll
    for (int k = 0; k < 4; k++) ent[k] = P[k].id;   // the entries as node ids (internal k, LEAF_BIT | j)
    if (absent1) ent[1] = INVALID;
    if (absent3) ent[3] = INVALID;
    qnode_words(lx, ly, lz, hx, hy, hz, make_uint4(id[0], id[1], id[2], id[3]), edge, out);
}
// entries from the node records in global memory (record words: rtbvh_device.h)
__device__ __forceinline__ void record_kids(const Inner* __restrict__ rec, uint32_t slot, QEnt& c0, QEnt& c1) {
    const float4* r = reinterpret_cast<const float4*>(rec + slot);
    const float4 w0 = r[0], w1 = r[1], w2 = r[2], w3 = r[3];
    const uint32_t own = __float_as_uint(w3.z);
    c0.id = __float_as_uint(w3.x);
    c1.id = __float_as_uint(w3.y);
    c0.slot = 2 * own;
    c1.slot = 2 * own + 1;
    c0.b[0] = w0.x; c0.b[1] = w0.y; c0.b[2] = w2.x; c0.b[3] = w0.z; c0.b[4] = w0.w; c0.b[5] = w2.y;
    c1.b[0] = w1.x; c1.b[1] = w1.y; c1.b[2] = w2.z; c1.b[3] = w1.z; c1.b[4] = w1.w; c1.b[5] = w2.w;
}
// the same from the topology and the node boxes (a build without records): the children of internal node k
__device__ __forceinline__ void nbox_kids(const BuildArgs& a, uint32_t k, QEnt& c0, QEnt& c1) {
    const uint4 t = a.topo[k];
    c0.id = t.x;
    c1.id = t.y;
    c0.slot = 2 * k;
    c1.slot = 2 * k + 1;
    child_box(a, t.x, c0.b);
    child_box(a, t.y, c1.b);
}
// the QNode of the node whose record is at `slot`, from the records (crossing nodes, small builds);
// E: the largest edge bound below it (node_edge); PSEUDO_NOGRID: a QNode without a grid gets its
// node's leaf pseudo-records (the bounce walk reads that node's exact record pair, trace.hip
// qchildren), for a build that wrote none
template <bool PSEUDO_NOGRID = false>
__device__ __forceinline__ void qnode_from_records(Inner* __restrict__ rec, uint32_t slot, float E, QNode* dst) {
    QEnt e0, e1;
    record_kids(rec, slot, e0, e1);
    float4 w[4];
    uint32_t ent[4];
    greedy_qnode_words(e0, e1, [&](const QEnt& e, QEnt& c0, QEnt& c1) { record_kids(rec, e.slot, c0, c1); }, E, w,
                       ent);
    store4(dst, w);
    if (PSEUDO_NOGRID && w[0].w == 0.f) {
        if (e0.id & LEAF_BIT)
            store_pseudo_record(rec + e0.slot, e0.id, mk(e0.b[0], e0.b[1], e0.b[2]), mk(e0.b[3], e0.b[4], e0.b[5]));
        if (e1.id & LEAF_BIT)
            store_pseudo_record(rec + e1.slot, e1.id, mk(e1.b[0], e1.b[1], e1.b[2]), mk(e1.b[3], e1.b[4], e1.b[5]));
    }
}

// QNodes of every internal node from the records (the one-workgroup build and
// rtbvh_build_from_codes), one node per thread.
__global__ __launch_bounds__(BLOCK) void k_qnodes(Inner* __restrict__ rec, const uint32_t* __restrict__ pint,
                                                  const Inner* __restrict__ inner, QNode* __restrict__ qn, uint32_t T) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k + 1 >= T) return;
    const uint32_t slot = slot_of(pint[k], T);   // pint[0] = INVALID: the root
    qnode_from_records(rec, slot, __uint_as_float(inner[k].aux0), qn + slot);
}

// the QNode of crossing node k at its slot, from the node boxes or the records (k_qnodes_late, k_pb_count_late)
__device__ __forceinline__ void qnode_cross(const BuildArgs& a, uint32_t k) {
    const uint32_t slot = slot_of(a.pint[k], a.T);
    const float E = *node_edge(a, k);
    if (!a.rec_on) {   // no records: the topology and the node boxes (no pseudo-records either)
        QEnt e0, e1;
        nbox_kids(a, k, e0, e1);
        float4 w[4];
        uint32_t ent[4];
        greedy_qnode_words(e0, e1, [&](const QEnt& e, QEnt& c0, QEnt& c1) { nbox_kids(a, e.id, c0, c1); }, E, w, ent);
        store4(a.qnode + slot, w);
    } else if (a.pseudo) {
        qnode_from_records<false>(a.rec, slot, E, a.qnode + slot);
    } else {
        qnode_from_records<true>(a.rec, slot, E, a.qnode + slot);
    }
}
// the QNodes of the crossing nodes k_refit_group listed: qlate[1, 1 + qlate[0]), one a thread
__global__ __launch_bounds__(BLOCK) void k_qnodes_late(BuildArgs a) {
    const uint32_t n = a.qlate[0];
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < n; j += gridDim.x * BLOCK) qnode_cross(a, a.qlate[1 + j]);
}

// The node records (rtbvh_device.h) of a build that wrote none (a certified-only context's, api.hip), on demand:
// node k's at its slot from the topology and the node boxes, and the leaf pseudo-records of a node whose QNode
// has no grid (the uncertified 4-wide walk reads that node's exact records) -- the words k_refit writes
__global__ __launch_bounds__(BLOCK) void k_records(BuildArgs a) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k + 1 >= a.T) return;
    const uint4 t = a.topo[k];
    float l[6], r[6];
    child_box(a, t.x, l);
    child_box(a, t.y, r);
    const f3 l0 = mk(l[0], l[1], l[2]), l1 = mk(l[3], l[4], l[5]), r0 = mk(r[0], r[1], r[2]), r1 = mk(r[3], r[4], r[5]);
    const uint32_t slot = slot_of(a.pint[k], a.T);
    store_record(a.rec + slot, l0, l1, r0, r1, t.x, t.y, k);
    if (a.qnode && reinterpret_cast<const float4*>(a.qnode + slot)[0].w == 0.f) {
        if (t.x & LEAF_BIT) store_leaf_record(a.rec, k, 0, t.x, l0, l1);
        if (t.y & LEAF_BIT) store_leaf_record(a.rec, k, 1, t.y, r0, r1);
    }
}
// ... and the node boxes of a build that wrote only records (from each node's record: its children's union)
__global__ __launch_bounds__(BLOCK) void k_nbox(BuildArgs a) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k + 1 >= a.T) return;
    const Inner* r = a.rec + slot_of(a.pint[k], a.T);
    float l[6], q[6];
    record_box(r, 0, l);
    record_box(r, 1, q);
    st_nbox(a.nbox, k, vmin(mk(l[0], l[1], l[2]), mk(q[0], q[1], q[2])), vmax(mk(l[3], l[4], l[5]), mk(q[3], q[4], q[5])));
}

// Refit (BVHConstructP2.hlsl:8-37) fused with the leaf records and the node outputs.  One
// workgroup per 256 sorted leaves [base, base + 256):
//  1. each thread gathers its leaf's clip-space triangle once and writes the 64-B leaf record
//     (MortonCodes.hlsl:87-96 box; the reference's edge1/edge2, RayTraceTraversal.hlsl:43-44);
//  2. it climbs from its leaf as BVHConstructP2 does (a per-node ticket; the second arriver
//     unions both children in (childL, childR) order): the nodes whose leaf range lies inside
//     the block join in LDS (both children are climbed by this block exactly then), the few
//     whose range crosses the block through refit_climb's global sc1 hand-off;
//  3. after a barrier every node of the block with an in-block range has both children's
//     boxes in LDS, and so have its internal children: one thread per node writes its record,
//     the pseudo-records of its leaf children and its QNode, all lanes busy.
// Against one pass per stage (round 1: records written during the divergent climb, then a
// QNode pass re-reading every record pair) this writes each output once and reads no record
// back except for the listed crossing nodes.
template <bool PSEUDO>
__global__ __launch_bounds__(RBLOCK) void k_refit(BuildArgs a) {
    __shared__ uint32_t s_cnt[RBLOCK];
    // node base + k: the boxes of its children (side 0, 1); before the climb, the staging
    // buffer of the leaf-record stores (128 float4 per wave)
    // (RBLOCK rows; more when phase 4's staging buffer, which reuses it, needs them)
    __shared__ __align__(16) float s_box[RBLOCK * 12 >= RTBVH_REFIT_STAGE_SLOTS * 16 ? RBLOCK
                                                                                  : RTBVH_REFIT_STAGE_SLOTS * 16 / 12 + 1][2][6];
    static_assert(sizeof(float) * 12 * RBLOCK >= 16 * 128 * (RBLOCK / 64), "leaf staging fits in s_box");
    __shared__ uint4 s_topo[RBLOCK];        // the block's nodes [base, base + BLOCK): ids, leaf range
    __shared__ uint32_t s_pint[RBLOCK];
    __shared__ uint32_t s_xn;
    __shared__ uint32_t s_own[RTBVH_REFIT_STAGE_SLOTS / 32];   // phase 4: staged slots of this round
    __shared__ float s_topo_z[3 * (RBLOCK / 64)];
    const uint32_t T = a.T;
    const uint32_t base = blockIdx.x * RBLOCK, tid = threadIdx.x;
    const uint32_t i = base + tid;
    const uint32_t end = base + RBLOCK;
    s_cnt[tid] = 0;
    if (tid == 0) s_xn = 0;
    if (i == 0 && a.qlate) a.qlate[0] = 0;   // (k_refit_group's list of crossing nodes)
    if (i + 1 < T) {   // coalesced, so the in-block climb makes no dependent global loads
        s_topo[tid] = a.topo[i];
        s_pint[tid] = a.pint[i];
    }
    f3 lo = mk(0.f, 0.f, 0.f), hi = lo;
    uint32_t e = INVALID;
    float emax = 0.f;   // the leaf's edge bound (margin.h): the bounce walk's margin takes the largest
    {
        float4 r[4] = {};
        if (i < T) {
            leaf_record_words(a, i, lo, hi, r);
            float zkey;
#if RTBVH_REFIT_PROBE == 5   // (A/B probe builds only: cost of the leaf's margin and footprint)
            zkey = lo.z;
#else
            leaf_margin(r, lo.z, hi.z, emax, zkey);
            a.lfp[i] = leaf_footprint(lo, hi, zkey);
#endif
        }
        const uint32_t w0 = base + (tid & ~63u);   // this wave's first leaf
        if (RTBVH_REFIT_PROBE != 4) staged_records(a.leaf + 4 * (size_t)w0, T > w0 ? min(64u, T - w0) : 0u, r,
                       reinterpret_cast<float4*>(&s_box[0][0][0]) + 128 * (tid >> 6));
    }
    if (i < T) {
        if (T == 1) {
            a.rootbox[0] = lo.x; a.rootbox[1] = lo.y; a.rootbox[2] = lo.z;
            a.rootbox[3] = hi.x; a.rootbox[4] = hi.y; a.rootbox[5] = hi.z;
        } else {
            e = a.pleaf[i];
        }
    }
    {   // the block's depth range (min lo.z, max hi.z of its leaves) for k_zrange: the binned primary
        // pass buckets by depth as soon as the leaves are written, before the climb above the blocks
        // (and the largest edge bound: an infinite one -- a non-finite triangle -- stays infinite)
        // (rootbox[8], the walk's scene-wide margin for keys stacked before a first hit, takes the finite
        // bounds only: a subtree holding a non-finite triangle is never pruned by distance, its QNodes'
        // tcap being -1)
        float zl = i < T ? lo.z : INFINITY, zh = i < T ? hi.z : -INFINITY, em = emax < INFINITY ? emax : 0.f;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            zl = fminf(zl, __shfl_xor(zl, off, 64));
            zh = fmaxf(zh, __shfl_xor(zh, off, 64));
            em = fmaxf(em, __shfl_xor(em, off, 64));
        }
        if ((tid & 63u) == 0) {
            s_topo_z[3 * (tid >> 6)] = zl;
            s_topo_z[3 * (tid >> 6) + 1] = zh;
            s_topo_z[3 * (tid >> 6) + 2] = em;
        }
    }
    __syncthreads();
    if (tid == 0) {
        float zl = INFINITY, zh = -INFINITY, em = 0.f;
        for (uint32_t w = 0; w < RBLOCK / 64; w++) {
            zl = fminf(zl, s_topo_z[3 * w]);
            zh = fmaxf(zh, s_topo_z[3 * w + 1]);
            em = fmaxf(em, s_topo_z[3 * w + 2]);
        }
        a.zpart[ZPART * blockIdx.x] = zl;
        a.zpart[ZPART * blockIdx.x + 1] = zh;
        a.zpart[ZPART * blockIdx.x + 2] = em;
    }
    for (int level = 0; e != INVALID && level < 2 * STACK_SIZE; level++) {
        const uint32_t p = e >> 1, side = e & 1u;
        bool cross = !(p >= base && p < end);   // p's index is outside the block: so is its range
        uint4 q3;
        if (!cross) {
            q3 = s_topo[p - base];   // ids, leaf range
            cross = !(q3.z >= base && q3.w < end);
        }
        if (cross) {   // k_refit_group takes it from here (kernel boundary: plain stores)
            float* hb = side ? a.inner[p].rmin : a.inner[p].lmin;
            hb[0] = lo.x; hb[1] = lo.y; hb[2] = lo.z; hb[3] = hi.x; hb[4] = hi.y; hb[5] = hi.z;
            *hand_edge(a, p, side) = emax;
            break;
        }
        float* sb = s_box[p - base][side];
        sb[0] = lo.x; sb[1] = lo.y; sb[2] = lo.z; sb[3] = hi.x; sb[4] = hi.y; sb[5] = hi.z;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the LDS box lands before the ticket
        // the ticket carries the edge bound: atomicMax of (bound | bit 31) -- nonzero, ordered as the
        // bounds (non-negative floats order as their bits) -- so the first arriver sees 0, the second
        // the sibling's bound, and the word ends as the node's own (phase 3 reads it)
        const uint32_t tk = atomicMax(&s_cnt[p - base], __float_as_uint(emax) | 0x80000000u);
        if (tk == 0) break;
        emax = fmaxf(emax, __uint_as_float(tk & 0x7FFFFFFFu));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const float* ob = s_box[p - base][side ^ 1u];
        const f3 smin = mk(ob[0], ob[1], ob[2]), smax = mk(ob[3], ob[4], ob[5]);
        // union in (childL, childR) order, as the reference
        if (side) { lo = vmin(smin, lo); hi = vmax(smax, hi); }
        else      { lo = vmin(lo, smin); hi = vmax(hi, smax); }
        e = s_pint[p - base];
        if (e == INVALID) {
            a.rootbox[0] = lo.x; a.rootbox[1] = lo.y; a.rootbox[2] = lo.z;
            a.rootbox[3] = hi.x; a.rootbox[4] = hi.y; a.rootbox[5] = hi.z;
        }
    }
    __syncthreads();
    // the block's crossing nodes (k_refit_group completes them, k_qnodes_late quantizes them):
    // listed at xlist[base, ...) in wave order, their tickets zeroed (no other ticket is used)
    const uint4 q = s_topo[tid];
    const bool xnode = i + 1 < T && !(q.z >= base && q.w < end);
    const uint64_t xb = __ballot(xnode);
    if (xb) {
        const uint32_t lane = tid & 63u;
        uint32_t wbase = 0;
        if (lane == (uint32_t)(__ffsll((unsigned long long)xb) - 1)) wbase = atomicAdd(&s_xn, (uint32_t)__popcll(xb));
        wbase = __shfl(wbase, __ffsll((unsigned long long)xb) - 1, 64);
        if (xnode) {
            a.xlist[base + wbase + (uint32_t)__popcll(xb & ((1ull << lane) - 1))] = i;
            a.refit_cnt[i] = 0;
        }
    }
    __syncthreads();
    if (tid == 0) a.xcnt[blockIdx.x] = s_xn;
    // 3. the block's in-block nodes: record, leaf pseudo-records, QNode
    const bool mine = i + 1 < T && !xnode;
    f3 l0 = mk(0.f, 0.f, 0.f), l1 = l0, r0 = l0, r1 = l0;
    uint32_t slot = INVALID;
    float4 rw[4], qw[4];
    uint32_t ent[4] = {INVALID, INVALID, INVALID, INVALID};
    float E = 0.f;   // the node's edge bound: its QNode's margin codes, added once the QNode is known to be read
    if (mine) {
    const float* L = s_box[tid][0];
    const float* R = s_box[tid][1];
    l0 = mk(L[0], L[1], L[2]); l1 = mk(L[3], L[4], L[5]);
    r0 = mk(R[0], R[1], R[2]); r1 = mk(R[3], R[4], R[5]);
    slot = slot_of(s_pint[tid], T);
    record_words(l0, l1, r0, r1, q.x, q.y, i, rw);
    if (a.nbox) st_nbox(a.nbox, i, vmin(l0, r0), vmax(l1, r1));   // (its own box; node-indexed: coalesced)
    // the QNode: its entries' boxes are in LDS (an in-block node's subtree is in the block)
    const auto lds_kids = [&](uint32_t x, QEnt& c0, QEnt& c1) {   // children of in-block node x
        const uint4 xq = s_topo[x - base];
        c0.id = xq.x;
        c1.id = xq.y;
        c0.slot = 2 * x;
        c1.slot = 2 * x + 1;
#pragma unroll
        for (int k = 0; k < 6; k++) {
            c0.b[k] = s_box[x - base][0][k];
            c1.b[k] = s_box[x - base][1][k];
        }
    };
    QEnt e0, e1;
    lds_kids(i, e0, e1);
    E = __uint_as_float(s_cnt[tid] & 0x7FFFFFFFu);   // the node's edge bound (the climb's ticket)
#if RTBVH_REFIT_PROBE == 1   // (probe: no QNode computed)
    for (int k = 0; k < 4; k++) { qw[k] = make_float4(0.f, 0.f, 0.f, 0.f); ent[k] = INVALID; }
#else
    greedy_qnode_words(e0, e1, [&](const QEnt& e, QEnt& c0, QEnt& c1) { lds_kids(e.id, c0, c1); }, -1.f, qw, ent);
#endif
    }
    // Which of the block's QNodes the 4-wide walk reads: it steps from a QNode to its internal
    // entries only, so a node's QNode is read iff the node is the root or an entry of a read QNode.  A QNode's
    // entries lie 1..3 levels below its node, so every node within 3 levels below a node the block does not own
    // (the root's parent, a crossing node, whose QNode k_qnodes_late builds) is taken as read, and the rest is
    // decided top-down inside the block, one QNode level per round.  Of the others (about two in three: the
    // greedy collapse expands them) no QNode is written.
    uint32_t* s_read = s_cnt;   // (the edge bounds were read above)
    __syncthreads();
    if (!RTBVH_QSKIP) {   // (A/B: every QNode written)
        s_read[tid] = mine ? 1u : 0u;
    } else {
        bool near = false;
        uint32_t x = i;
        for (int up = 0; mine && up < 3 && !near; up++) {
            const uint32_t e = s_pint[x - base];
            const uint32_t p = e >> 1;
            near = e == INVALID || !(p >= base && p < end) || !(s_topo[p - base].z >= base && s_topo[p - base].w < end);
            x = p;
        }
        s_read[tid] = mine && near ? 1u : 0u;
    }
    // A QNode without a grid is walked (uncertified walks, trace.hip qchildren) on its node's exact record
    // pair: the walk steps to the node's binary grandchildren, not to its greedy entries -- so those are the
    // entries whose QNodes it reads (a grandchild the collapse expanded past was left unwritten)
    if (mine && qw[0].w == 0.f) {
#pragma unroll
        for (int side = 0; side < 2; side++) {
            const uint32_t ch = side ? q.y : q.x;
            const uint4 cq = (ch & LEAF_BIT) ? make_uint4(INVALID, INVALID, 0u, 0u) : s_topo[ch - base];
            ent[2 * side] = cq.x;
            ent[2 * side + 1] = cq.y;
        }
    }
    bool pending = mine && RTBVH_QSKIP;   // its entries are not marked yet
    for (;;) {
        __syncthreads();
        bool changed = false;
        if (pending && s_read[tid]) {
            pending = false;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t e = ent[k];   // (an internal entry of an owned node is owned)
                if (e != INVALID && !(e & LEAF_BIT) && s_read[e - base] == 0) {
                    s_read[e - base] = 1;
                    changed = true;
                }
            }
        }
        if (!__syncthreads_or(changed)) break;
    }
    const bool rd = mine && s_read[tid] != 0;
    if (rd) qnode_codes(qw, E);
    // 4. the outputs through LDS.  Every slot this block writes in phase 3 lies in its window
    // [2 base, 2 base + 2 RBLOCK) -- a node's record / QNode at 2 parent + side with the parent in
    // the block, a leaf child's pseudo-record at 2 i + side -- except the record and QNode of a
    // node whose parent crosses the block (a few per block; stored directly).  The window goes
    // out STAGE slots at a time: the writers fill the staging buffer (over s_box, read no more)
    // and mark their slots, then the block stores the marked slots 16 B per lane, consecutive
    // lanes on consecutive bytes (a 64-B record per lane writes at ~0.6x that rate).
    // Unmarked slots (records of crossing nodes, k_refit_group's; other blocks' records) are left
    // alone.
    constexpr uint32_t STAGE = RTBVH_REFIT_STAGE_SLOTS;
    static_assert(sizeof(s_box) >= 64 * STAGE, "staging fits in s_box");
    static_assert((2 * RBLOCK) % STAGE == 0, "whole rounds");
    float4* s_stage = reinterpret_cast<float4*>(&s_box[0][0][0]);
    const uint32_t w0 = 2 * base;
    const bool rin = mine && slot - w0 < 2 * RBLOCK;
    if (mine && !rin) {
        if (a.rec_on) store4(a.rec + slot, rw);
        if (rd) store4(a.qnode + slot, qw);
    }
    const uint32_t nslots = 2 * T - 1;
#pragma unroll
    for (uint32_t kind = 0; kind < 2; kind++) {   // 0: records and pseudo-records (unless none: a.rec_on), 1: QNodes
        if (kind == 0 && !a.rec_on) continue;
        float4* dst = kind ? reinterpret_cast<float4*>(a.qnode) : reinterpret_cast<float4*>(a.rec);
#pragma unroll 1
        for (uint32_t r = 0; r < 2 * RBLOCK; r += STAGE) {
            __syncthreads();   // s_box reads (first round) / the previous round's stores are done
            if (tid < STAGE / 32) s_own[tid] = 0;
            __syncthreads();
            const uint32_t lo_slot = w0 + r;
            const auto put = [&](uint32_t sl, const float4 (&w)[4]) {
                const uint32_t k = sl - lo_slot;
                if (k < STAGE) {
                    s_stage[4 * k] = w[0]; s_stage[4 * k + 1] = w[1];
                    s_stage[4 * k + 2] = w[2]; s_stage[4 * k + 3] = w[3];
                    atomicOr(&s_own[k >> 5], 1u << (k & 31));
                }
            };
            if (rin && (kind == 0 || rd)) put(slot, kind ? qw : rw);
            // the leaf children's pseudo-records: all (PSEUDO), or those of a node whose QNode has no
            // grid and is read (the bounce walk reads that node's exact record pair)
            if (kind == 0 && mine && (PSEUDO || (qw[0].w == 0.f && rd))) {
                float4 pw[4];
                if (q.x & LEAF_BIT) { pseudo_words(q.x, l0, l1, pw); put(2 * i, pw); }
                if (q.y & LEAF_BIT) { pseudo_words(q.y, r0, r1, pw); put(2 * i + 1, pw); }
            }
            __syncthreads();
            for (uint32_t c = tid; c < 4 * STAGE; c += RBLOCK) {
                const uint32_t k = c >> 2;
                if ((s_own[k >> 5] >> (k & 31)) & 1u && lo_slot + k < nslots)
                    if (RTBVH_REFIT_PROBE != 3) st_out<4>(dst + 4 * (size_t)(lo_slot + k) + (c & 3), s_stage[c]);
            }
        }
    }
}

// The global climb of a crossing node k (a few per k_refit workgroup, the top of the tree among them;
// k_refit_group runs it for the nodes that cross their group): k_refit left the box of every
// non-crossing child of a crossing node in inner[node] (leaf or in-block subtree).  Both children
// non-crossing -> k is complete, climb from it; one -> arrive at k's ticket for that child (the other
// arrives by a climb); none -> nothing.  (Round 5 ran it for every crossing node, one wave per refit
// workgroup, as k_refit_top: ~25 levels of device-scope round trips at C5, 0.12 ms.)
__device__ __forceinline__ void refit_top_node(const BuildArgs& a, uint32_t k) {
    const uint4 q = a.topo[k];
    const bool ncl = (q.x & LEAF_BIT) || !crossing(a.topo[q.x], q.x);
    const bool ncr = (q.y & LEAF_BIT) || !crossing(a.topo[q.y], q.y);
    if (!ncl && !ncr) return;
    const float* L = a.inner[k].lmin;
    const float* R = a.inner[k].rmin;
    f3 lo, hi;
    float em;
    uint32_t e = a.pint[k];
    if (ncl && ncr) {
        em = fmaxf(*hand_edge(a, k, 0), *hand_edge(a, k, 1));
        *node_edge(a, k) = em;
        complete_node(a, k, e, mk(L[0], L[1], L[2]), mk(L[3], L[4], L[5]), mk(R[0], R[1], R[2]), mk(R[3], R[4], R[5]),
                      lo, hi);
    } else {   // one child here: its arrival at k's ticket (the other side's box and bound come sc1)
        const uint32_t side = ncl ? 0u : 1u;
        const float* B = side ? R : L;
        const f3 blo = mk(B[0], B[1], B[2]), bhi = mk(B[3], B[4], B[5]);
        em = *hand_edge(a, k, side);
        const uint32_t old = __hip_atomic_fetch_add(&a.refit_cnt[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == 0) return;
        asm volatile("" ::: "memory");
        f3 smin, smax;
        ld_box_sc1(side ? a.inner[k].lmin : a.inner[k].rmin, smin, smax);
        em = fmaxf(em, ld_edge_sc1(hand_edge(a, k, side ^ 1u)));
        *node_edge(a, k) = em;
        if (side) complete_node(a, k, e, smin, smax, blo, bhi, lo, hi);
        else      complete_node(a, k, e, blo, bhi, smin, smax, lo, hi);
    }
    refit_climb(lo, hi, em, e, a);
}

// ---- the crossing nodes, grouped (launch_refit_tail) ---------------------------------------------------
// The global climb makes one device-scope round trip (sc1 box hand-off, ticket atomic) per level of crossing
// nodes, ~25 levels at C5.  A group is RGROUP consecutive refit workgroups (GSPAN node indices), and a crossing
// node whose leaf range lies inside its group's span is "group-internal" (C5: 176K of the 181K).  k_refit_group,
// one workgroup per group, climbs the group-internal ones in LDS (slots by node index through a bitmap rank; the
// same union order and bounds as the global climb), and where a climb leaves the group -- its parent crosses the
// group -- it continues with the global protocol (refit_climb); the group's other crossing nodes start it
// (refit_top_node).  The protocol's tickets take arrivals in any order, so the global climb above the groups is the
// same, a handful of levels.  A group with more than GCAP crossing nodes (a degenerate tree) runs the global
// protocol for all of them.
constexpr uint32_t RGROUP = 64;
constexpr uint32_t GSPAN = RGROUP * RBLOCK;
static_assert((GSPAN & (GSPAN - 1)) == 0, "the group span is a power of two");
constexpr uint32_t GCAP = 1024;
constexpr uint32_t GBLOCK = 1024;
__device__ __forceinline__ bool group_internal(uint4 topo_k, uint32_t k) {
    const uint32_t gb = k & ~(GSPAN - 1);
    return topo_k.z >= gb && topo_k.w < gb + GSPAN;
}
__global__ __launch_bounds__(GBLOCK) void k_refit_group(BuildArgs a) {
    __shared__ uint32_t s_bits[GSPAN / 32];   // the group's crossing nodes, by index
    __shared__ uint32_t s_pre[GSPAN / 32];    // their rank before each word: slot(k) = s_pre[w] + popc(bits below k)
    __shared__ uint32_t s_off[RGROUP + 1];
    __shared__ uint32_t s_sid[GCAP];          // slot -> node
    __shared__ uint32_t s_par[GCAP];          // the node's parent link (pint)
    __shared__ float s_gbox[GCAP][2][6];
    __shared__ float s_ge[GCAP][2];
    __shared__ uint32_t s_tk[GCAP];           // children in (3: not group-internal, the global protocol)
    __shared__ uint32_t s_wsum[GBLOCK / 64];
    const uint32_t g = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t nb = (a.T + RBLOCK - 1) / RBLOCK;
    const uint32_t b0 = g * RGROUP, nbg = min(RGROUP, nb - b0);
    const uint32_t gbase = g * GSPAN;
    if (tid < 64) {   // the lists' offsets (RGROUP <= 64: one wave)
        static_assert(RGROUP <= 64, "one wave scans the group's list counts");
        const uint32_t v = tid < nbg ? a.xcnt[b0 + tid] : 0u;
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if ((int)lane >= d) x += y;
        }
        if (tid < nbg) s_off[tid] = x - v;
        if (tid == nbg - 1) s_off[nbg] = x;
    }
    for (uint32_t w = tid; w < GSPAN / 32; w += GBLOCK) s_bits[w] = 0;
    __syncthreads();
    const uint32_t m = s_off[nbg];
    const auto entry = [&](uint32_t e) {   // the e-th crossing node of the group (list order)
        uint32_t j = 0;
        for (uint32_t st = 32; st; st >>= 1)
            if (j + st <= nbg - 1 && s_off[j + st] <= e) j += st;
        return a.xlist[(size_t)(b0 + j) * RBLOCK + (e - s_off[j])];
    };
    // the group's crossing nodes, listed densely for k_qnodes_late (a wave per refit workgroup ran ~9 of 64
    // lanes)
    __shared__ uint32_t s_lbase;
    if (tid == 0) s_lbase = atomicAdd(&a.qlate[0], m);
    __syncthreads();
    const uint32_t lbase = 1 + s_lbase;
    if (m > GCAP) {   // (uniform) the global protocol for every crossing node of the group
        for (uint32_t e = tid; e < m; e += GBLOCK) {
            const uint32_t k = entry(e);
            a.qlate[lbase + e] = k;
            refit_top_node(a, k);
        }
        return;
    }
    uint32_t k0 = 0;
    if (tid < m) {
        k0 = entry(tid);
        a.qlate[lbase + tid] = k0;
        atomicOr(&s_bits[(k0 - gbase) >> 5], 1u << ((k0 - gbase) & 31));
    }
    __syncthreads();
    {   // the word ranks: an exclusive scan of the words' popcounts (GSPAN / 32 = GBLOCK words, one a thread)
        static_assert(GSPAN / 32 == GBLOCK, "one bitmap word per thread");
        const uint32_t v = (uint32_t)__popc(s_bits[tid]);
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if ((int)lane >= d) x += y;
        }
        if (lane == 63) s_wsum[wv] = x;
        __syncthreads();
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; w++) before += s_wsum[w];
        s_pre[tid] = before + x - v;
    }
    __syncthreads();
    const auto slot_of_k = [&](uint32_t k) {   // k in the group's span and listed
        const uint32_t r = k - gbase;
        return s_pre[r >> 5] + (uint32_t)__popc(s_bits[r >> 5] & ((1u << (r & 31)) - 1u));
    };
    const auto listed = [&](uint32_t k) {
        const uint32_t r = k - gbase;
        return r < GSPAN && ((s_bits[r >> 5] >> (r & 31)) & 1u);
    };
    // each node: its parent link, and the boxes k_refit handed over (leaves and the subtrees it joined)
    static_assert(GCAP == GBLOCK, "one slot per thread");
    bool outside = false;   // this thread's node crosses its group: the global protocol
    if (tid < m) {
        const uint32_t sl = slot_of_k(k0);
        const uint4 t = a.topo[k0];
        s_sid[sl] = k0;
        s_par[sl] = a.pint[k0];
        uint32_t ready = 3;
        if (group_internal(t, k0)) {
            ready = 0;
#pragma unroll
            for (uint32_t side = 0; side < 2; side++) {
                const uint32_t c = side ? t.y : t.x;
                if ((c & LEAF_BIT) || !crossing(a.topo[c], c)) {
                    const float* hb = side ? a.inner[k0].rmin : a.inner[k0].lmin;
#pragma unroll
                    for (int q = 0; q < 6; q++) s_gbox[sl][side][q] = hb[q];
                    s_ge[sl][side] = *hand_edge(a, k0, side);
                    ++ready;
                }
            }
        } else {
            outside = true;
        }
        s_tk[sl] = ready;
    }
    __syncthreads();
    // the starting nodes, read before any climb raises a ticket (a slot per thread)
    const bool start = tid < m && s_tk[tid] == 2;
    __syncthreads();
    if (outside) refit_top_node(a, k0);
    if (start) {
        uint32_t sl = tid;
        for (int level = 0; level < 2 * STACK_SIZE; level++) {   // (bounded: a CPUTests-delta tree may cycle)
            const uint32_t k = s_sid[sl];
            const float* L = s_gbox[sl][0];
            const float* R = s_gbox[sl][1];
            const float em = fmaxf(s_ge[sl][0], s_ge[sl][1]);
            *node_edge(a, k) = em;   // (read by k_qnodes_late, a later launch)
            const uint32_t e = s_par[sl];
            f3 lo, hi;
            complete_node(a, k, e, mk(L[0], L[1], L[2]), mk(L[3], L[4], L[5]), mk(R[0], R[1], R[2]), mk(R[3], R[4], R[5]),
                          lo, hi);
            if (e == INVALID) break;   // the root
            const uint32_t p = e >> 1, side = e & 1u;
            const uint32_t sp = listed(p) ? slot_of_k(p) : GCAP;
            if (sp < GCAP && s_tk[sp] != 3) {   // a group-internal parent: its ticket in LDS
                float* d = s_gbox[sp][side];
                d[0] = lo.x; d[1] = lo.y; d[2] = lo.z; d[3] = hi.x; d[4] = hi.y; d[5] = hi.z;
                s_ge[sp][side] = em;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the box lands before the ticket
                const uint32_t old = atomicAdd(&s_tk[sp], 1u);
                if (old != 1) break;   // the sibling is still to come
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                sl = sp;
            } else {   // the parent crosses the group: the global climb from here
                refit_climb(lo, hi, em, e, a);
                break;
            }
        }
    }
}

// rtbvh_compute_bvh with the binned primary pass: k_refit_group's listed crossing nodes are quantized in the
// launch of the pass's count pass, which reads only what k_refit wrote (leaf footprints, the depth range); the
// gated walk and the bounce walk, which read the whole tree, come after both.
#include "pb_bin.h"
// After k_refit_group (the grouped climb, its own launch): blocks [0, nlate) quantize the crossing nodes it listed
// (k_qnodes_late's work) beside the count.  (8 waves per SIMD, the QNode blocks spilling: 89 us against 98 at
// the QNode code's 84 VGPRs, 5 waves; k_refit_group + this 162 us against round 5's one global climb in the count launch + its QNodes 194, r06_o)
__global__ __launch_bounds__(BLOCK, 8) void k_pb_count_late(BuildArgs b, TraceArgs a, uint32_t nlate,
                                                         uint32_t* __restrict__ off, uint32_t* __restrict__ cur,
                                                         uint4* __restrict__ bins, uint32_t cap, uint32_t ntx) {
    if (blockIdx.x < nlate) {
        const uint32_t n = b.qlate[0];
        for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < n; j += nlate * BLOCK) qnode_cross(b, b.qlate[1 + j]);
        return;
    }
    pb_bin_block<false>(a, blockIdx.x - nlate, off, cur, bins, cap, ntx);
}

__global__ __launch_bounds__(BLOCK) void k_refit_boxes(BuildArgs a, const float* __restrict__ boxes) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= a.T) return;
    const float* b = boxes + 6 * (size_t)i;
    const f3 lo = mk(b[0], b[1], b[2]), hi = mk(b[3], b[4], b[5]);
    if (a.T == 1) {
        for (int k = 0; k < 6; k++) a.rootbox[k] = b[k];
        return;
    }
    refit_climb(lo, hi, INFINITY, a.pleaf[i], a);   // (no triangles: no margin; the walk never prunes by distance)
}

// ---- small scenes: the whole build in one workgroup ------------------------------
// The reference's own meshes (Test.obj: 1,952 triangles) rebuild every frame
// (Graphics.cpp:56), and at that size the multi-kernel build is ~18 dependent launches of
// almost no work.  One 1024-thread workgroup does it all with the same arithmetic (the
// mesh box reduction, morton_tri, leaf_record, karras_node, store_record), everything but
// the outputs resident in LDS (152 KB of the CU's 160):
//  - the sort is a bitonic network over 64-bit (code << 32 | triangle) keys: a total order
//    on distinct keys, hence exactly the stable radix sort's (code, triangle) order;
//  - Karras reads the codes from LDS;
//  - the refit is k_refit's in-block protocol for every node (LDS boxes and tickets).
// Outputs land in the multi-kernel build's buffers (the sorted pairs in the sort's A
// buffers), so every later kernel and export is unchanged.
constexpr uint32_t SMALL_BLOCK = 1024;
constexpr uint32_t SMALL_T = 2048;
static_assert(SMALL_T == 2 * SMALL_BLOCK, "k_build_small: two keys / leaves per thread");

struct LdsCodes {   // sorted code j = the high word of the sorted 64-bit key
    const uint64_t* kv;
    __device__ uint32_t operator[](int32_t j) const { return (uint32_t)(kv[j] >> 32); }
};

// RTBVH_SMALL_PROBE (A/B builds only): thread 0 prints the constant-rate clock at the phase ends
#ifdef RTBVH_SMALL_PROBE
#define SMALL_MARK(k) do { __syncthreads(); if (tid == 0) tmark[k] = wall_clock64(); } while (0)
#else
#define SMALL_MARK(k) do { } while (0)
#endif
template <int MODE>
__global__ __launch_bounds__(SMALL_BLOCK) void k_build_small(BuildArgs a, uint32_t* __restrict__ sk,
                                                             uint32_t* __restrict__ sv) {
    __shared__ uint64_t s_kv[SMALL_T];
    __shared__ uint2 s_ids[SMALL_T];        // node k: child ids
    __shared__ uint32_t s_pint[SMALL_T];    // node k: parent << 1 | side (INVALID: root)
    __shared__ uint32_t s_pleaf[SMALL_T];   // leaf j: parent << 1 | side
    __shared__ float s_box[SMALL_T][2][6];
    __shared__ uint32_t s_cnt[SMALL_T];
    __shared__ float s_red[16 * 6];
    __shared__ uint32_t s_emax;             // the largest leaf edge bound (rootbox[8], margin.h)
    const uint32_t tid = threadIdx.x, T = a.T;
#ifdef RTBVH_SMALL_PROBE
    uint64_t tmark[7];
#endif
    SMALL_MARK(0);
    for (uint32_t k = tid; k < SMALL_T; k += SMALL_BLOCK) s_cnt[k] = 0;
    if (a.morton_mode == 0) {   // k_bounds + k_bounds_final as one reduction
        f3 mn = mk(INFINITY, INFINITY, INFINITY), mx = mk(-INFINITY, -INFINITY, -INFINITY);
        for (uint32_t i = tid; i < a.V; i += SMALL_BLOCK) {
            const float4 p = a.opos[i];
            mn = vmin(mn, mk(p.x, p.y, p.z));
            mx = vmax(mx, mk(p.x, p.y, p.z));
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            mn.x = fminf(mn.x, __shfl_xor(mn.x, off, 64));
            mn.y = fminf(mn.y, __shfl_xor(mn.y, off, 64));
            mn.z = fminf(mn.z, __shfl_xor(mn.z, off, 64));
            mx.x = fmaxf(mx.x, __shfl_xor(mx.x, off, 64));
            mx.y = fmaxf(mx.y, __shfl_xor(mx.y, off, 64));
            mx.z = fmaxf(mx.z, __shfl_xor(mx.z, off, 64));
        }
        const uint32_t w = tid >> 6;
        if ((tid & 63) == 0) {
            s_red[6 * w + 0] = mn.x; s_red[6 * w + 1] = mn.y; s_red[6 * w + 2] = mn.z;
            s_red[6 * w + 3] = mx.x; s_red[6 * w + 4] = mx.y; s_red[6 * w + 5] = mx.z;
        }
        __syncthreads();
        if (tid == 0) {
            for (int k = 1; k < 16; k++) {
                mn = vmin(mn, mk(s_red[6 * k + 0], s_red[6 * k + 1], s_red[6 * k + 2]));
                mx = vmax(mx, mk(s_red[6 * k + 3], s_red[6 * k + 4], s_red[6 * k + 5]));
            }
            a.bounds[0] = mn.x; a.bounds[1] = mn.y; a.bounds[2] = mn.z;
            a.bounds[3] = mx.x; a.bounds[4] = mx.y; a.bounds[5] = mx.z;
        }
        __syncthreads();   // morton_tri reads the box back (same workgroup: visible)
    }
    SMALL_MARK(1);
    // the bitonic network over all SMALL_T keys (padding ~0: above every key), thread tid holding
    // keys 2 tid and 2 tid + 1 in registers: the compare-exchanges at distance j < 128 are within
    // the wave (j = 1 in the thread, 2..64 across lanes tid ^ j/2), only j >= 128 goes through LDS
    // with a barrier per step (10 of the 66 steps; all through LDS: 26 us of the 79)
    uint64_t e[2];
#pragma unroll
    for (uint32_t b = 0; b < 2; b++) {
        const uint32_t t = 2 * tid + b;
        e[b] = t < T ? ((uint64_t)morton_tri(a, t) << 32 | t) : ~0ull;
    }
    SMALL_MARK(2);
    for (uint32_t k = 2; k <= SMALL_T; k <<= 1) {
        uint32_t j = k >> 1;
        if (j >= 128) {
            s_kv[2 * tid] = e[0];
            s_kv[2 * tid + 1] = e[1];
            __syncthreads();
            for (; j >= 128; j >>= 1) {
                // pair tid: index i with bit j clear (tid with a 0 inserted at bit j) and i | j
                const uint32_t i = ((tid & ~(j - 1)) << 1) | (tid & (j - 1)), l = i | j;
                const uint64_t x = s_kv[i], y = s_kv[l];
                const bool up = (i & k) == 0, lt = x < y;
                s_kv[i] = up == lt ? x : y;
                s_kv[l] = up == lt ? y : x;
                __syncthreads();
            }
            e[0] = s_kv[2 * tid];
            e[1] = s_kv[2 * tid + 1];
        }
        for (; j >= 2; j >>= 1) {
            const uint32_t m = j >> 1;   // partner lane distance
#pragma unroll
            for (uint32_t b = 0; b < 2; b++) {
                const uint32_t i = 2 * tid + b;
                const uint64_t x = e[b];
                const uint32_t ylo = (uint32_t)__shfl_xor((int)(uint32_t)x, (int)m, 64);
                const uint32_t yhi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), (int)m, 64);
                const uint64_t y = (uint64_t)yhi << 32 | ylo;
                const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
                e[b] = keep_min == (x < y) ? x : y;
            }
        }
        const bool up = ((2 * tid) & k) == 0;   // j = 1: the thread's own pair
        const bool sw = up != (e[0] < e[1]);
        const uint64_t x0 = e[0];
        e[0] = sw ? e[1] : x0;
        e[1] = sw ? x0 : e[1];
    }
    s_kv[2 * tid] = e[0];
    s_kv[2 * tid + 1] = e[1];
    SMALL_MARK(3);
#pragma unroll
    for (uint32_t b = 0; b < 2; b++) {
        const uint32_t i = 2 * tid + b;
        if (i < T) {
            sk[i] = (uint32_t)(e[b] >> 32);
            sv[i] = (uint32_t)e[b];
        }
    }
    __syncthreads();   // sorted keys in LDS; clip triangles visible to the block
    const LdsCodes codes{s_kv};
    if (tid == 0) s_emax = 0u;
    __syncthreads();
    // leaves i = tid, tid + SMALL_BLOCK: records, margins, Karras nodes; the boxes stay in registers
    // for the refit (the triangle id from the sorted key in LDS)
    f3 llo[2], lhi[2];
    float lem[2];   // the leaves' edge bounds (the climb carries them up: each node's QNode margin)
#pragma unroll
    for (uint32_t b = 0; b < 2; b++) {
        const uint32_t i = tid + b * SMALL_BLOCK;
        llo[b] = lhi[b] = mk(0.f, 0.f, 0.f);
        lem[b] = 0.f;
        if (i < T) {
            f3 lo, hi;
            float4 r[4];
            leaf_record_words_of(a, (uint32_t)s_kv[i], lo, hi, r);
            float4* dst = a.leaf + 4 * (size_t)i;
            dst[0] = r[0]; dst[1] = r[1]; dst[2] = r[2]; dst[3] = r[3];
            float em, zkey;
            leaf_margin(r, lo.z, hi.z, em, zkey);
            a.lfp[i] = leaf_footprint(lo, hi, zkey);
            // (non-negative floats order as their bits; the scene-wide bound takes the finite ones, k_refit)
            if (em < INFINITY) atomicMax(&s_emax, __float_as_uint(em));
            if (i + 1 < T) karras_node<MODE>(codes, T, i, a.topo, a.pleaf, a.pint);
            llo[b] = lo;
            lhi[b] = hi;
            lem[b] = em;
        }
    }
    if (tid == 0 && T > 1) a.pint[0] = INVALID;
    SMALL_MARK(4);
    __syncthreads();   // links written by other threads: copy them into LDS
    if (tid == 0) a.rootbox[8] = __uint_as_float(s_emax);
    for (uint32_t i = tid; i < T; i += SMALL_BLOCK) {
        s_pleaf[i] = a.pleaf[i];
        if (i + 1 < T) {
            const uint4 q = a.topo[i];
            s_ids[i] = make_uint2(q.x, q.y);
            s_pint[i] = a.pint[i];
        }
    }
    __syncthreads();
    SMALL_MARK(5);
    // k_refit's in-block protocol, in LDS only: the second arriver at a node unites the two child
    // boxes (left first, as k_refit) and climbs on; the node records are written afterwards, one
    // thread per node (a store per level kept the climb's chain waiting on the store queue)
#pragma unroll
    for (uint32_t b = 0; b < 2; b++) {
        const uint32_t i = tid + b * SMALL_BLOCK;
        if (i >= T) continue;
        f3 lo = llo[b], hi = lhi[b];
        float em = lem[b];
        if (T == 1) {
            a.rootbox[0] = lo.x; a.rootbox[1] = lo.y; a.rootbox[2] = lo.z;
            a.rootbox[3] = hi.x; a.rootbox[4] = hi.y; a.rootbox[5] = hi.z;
            a.rootbox[6] = lo.z; a.rootbox[7] = hi.z;   // (k_zrange's: the root box's depth range)
            continue;
        }
        uint32_t e = s_pleaf[i];
        store_pseudo_record(a.rec + e, LEAF_BIT | i, lo, hi);
        for (int level = 0; level < 2 * STACK_SIZE; level++) {
            const uint32_t p = e >> 1, side = e & 1u;
            float* sb = s_box[p][side];
            sb[0] = lo.x; sb[1] = lo.y; sb[2] = lo.z; sb[3] = hi.x; sb[4] = hi.y; sb[5] = hi.z;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the LDS box lands before the ticket
            // the ticket carries the edge bound as k_refit's (the word ends as the node's bound)
            const uint32_t tk = atomicMax(&s_cnt[p], __float_as_uint(em) | 0x80000000u);
            if (tk == 0) break;
            em = fmaxf(em, __uint_as_float(tk & 0x7FFFFFFFu));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const float* ob = s_box[p][side ^ 1u];
            const f3 smin = mk(ob[0], ob[1], ob[2]), smax = mk(ob[3], ob[4], ob[5]);
            e = s_pint[p];
            if (side) { lo = vmin(smin, lo); hi = vmax(smax, hi); }
            else      { lo = vmin(lo, smin); hi = vmax(hi, smax); }
            if (e == INVALID) {
                a.rootbox[0] = lo.x; a.rootbox[1] = lo.y; a.rootbox[2] = lo.z;
                a.rootbox[3] = hi.x; a.rootbox[4] = hi.y; a.rootbox[5] = hi.z;
                a.rootbox[6] = lo.z; a.rootbox[7] = hi.z;
                break;
            }
        }
    }
    __syncthreads();   // every node's two child boxes in LDS
    for (uint32_t p = tid; p + 1 < T; p += SMALL_BLOCK) {
        const float* l = s_box[p][0];
        const float* r = s_box[p][1];
        const uint2 ids = s_ids[p];
        store_record(a.rec + slot_of(s_pint[p], T), mk(l[0], l[1], l[2]), mk(l[3], l[4], l[5]), mk(r[0], r[1], r[2]),
                     mk(r[3], r[4], r[5]), ids.x, ids.y, p);
        *node_edge(a, p) = __uint_as_float(s_cnt[p] & 0x7FFFFFFFu);   // (k_qnodes: the QNode's margin)
    }
#ifdef RTBVH_SMALL_PROBE
    SMALL_MARK(6);
    if (tid == 0)
        printf("SMALLPROBE T=%u bounds %llu morton %llu sort %llu leaves+karras %llu links %llu refit %llu (x10ns)\n", T,
               (unsigned long long)(tmark[1] - tmark[0]), (unsigned long long)(tmark[2] - tmark[1]),
               (unsigned long long)(tmark[3] - tmark[2]), (unsigned long long)(tmark[4] - tmark[3]),
               (unsigned long long)(tmark[5] - tmark[4]), (unsigned long long)(tmark[6] - tmark[5]));
#endif
}

// Scenes above k_build_small's 2048 triangles and up to 8192 (C2's Image_Test: 3072): the Morton pass
// and the sort in one workgroup -- the same bitonic network over (code << 32 | triangle) keys as
// k_build_small, KPT keys per thread (steps at distance < KPT in the thread, < 64 KPT across lanes, the
// longer ones through LDS) -- in place of the Morton launch and the radix sort's twelve; the rest of the
// multi-kernel build follows.  (k_build_small's node boxes would not fit in LDS at this size.)
template <uint32_t KPT>
__global__ __launch_bounds__(SMALL_BLOCK) void k_morton_sort_small(BuildArgs a, uint32_t* __restrict__ sk,
                                                                   uint32_t* __restrict__ sv) {
    constexpr uint32_t N = KPT * SMALL_BLOCK;
    __shared__ uint64_t s_kv[N];
    const uint32_t tid = threadIdx.x, T = a.T;
    uint64_t e[KPT];
#pragma unroll
    for (uint32_t b = 0; b < KPT; b++) {
        const uint32_t t = KPT * tid + b;
        e[b] = t < T ? ((uint64_t)morton_tri(a, t) << 32 | t) : ~0ull;
    }
    for (uint32_t k = 2; k <= N; k <<= 1) {
        uint32_t j = k >> 1;
        if (j >= 64 * KPT) {
#pragma unroll
            for (uint32_t b = 0; b < KPT; b++) s_kv[KPT * tid + b] = e[b];
            __syncthreads();
            for (; j >= 64 * KPT; j >>= 1) {
#pragma unroll
                for (uint32_t h = 0; h < KPT / 2; h++) {
                    const uint32_t p = tid + h * SMALL_BLOCK;   // pair p: index i with bit j clear, and i | j
                    const uint32_t i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), l = i | j;
                    const uint64_t x = s_kv[i], y = s_kv[l];
                    const bool up = (i & k) == 0, lt = x < y;
                    s_kv[i] = up == lt ? x : y;
                    s_kv[l] = up == lt ? y : x;
                }
                __syncthreads();
            }
#pragma unroll
            for (uint32_t b = 0; b < KPT; b++) e[b] = s_kv[KPT * tid + b];
        }
        for (; j >= KPT; j >>= 1) {   // partner lane tid ^ (j / KPT)
            const uint32_t m = j / KPT;
#pragma unroll
            for (uint32_t b = 0; b < KPT; b++) {
                const uint32_t i = KPT * tid + b;
                const uint64_t x = e[b];
                const uint32_t ylo = (uint32_t)__shfl_xor((int)(uint32_t)x, (int)m, 64);
                const uint32_t yhi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), (int)m, 64);
                const uint64_t y = (uint64_t)yhi << 32 | ylo;
                const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
                e[b] = keep_min == (x < y) ? x : y;
            }
        }
#pragma unroll
        for (uint32_t jj = KPT / 2; jj >= 1; jj >>= 1) {   // in the thread (jj a constant: e stays in registers)
            if (jj > j) continue;   // (stages k < KPT start below KPT / 2)
#pragma unroll
            for (uint32_t b = 0; b < KPT; b++) {
                if (b & jj) continue;
                const uint32_t i = KPT * tid + b;
                const uint64_t x = e[b], y = e[b | jj];
                const bool sw = ((i & k) == 0) != (x < y);
                e[b] = sw ? y : x;
                e[b | jj] = sw ? x : y;
            }
        }
    }
#pragma unroll
    for (uint32_t b = 0; b < KPT; b++) {
        const uint32_t i = KPT * tid + b;
        if (i < T) {
            sk[i] = (uint32_t)(e[b] >> 32);
            sv[i] = (uint32_t)e[b];
        }
    }
}

// reference layout (RayTraceGlobal.hlsl:39-51): leaves [0,T), internal k at T+k
struct RefNode { uint32_t parent, child_l, child_r, code; float bb_min[3], bb_max[3]; uint32_t index; };
static_assert(sizeof(RefNode) == 44, "44-B Node");

__global__ __launch_bounds__(BLOCK) void k_export(BuildArgs a, RefNode* __restrict__ out) {
    const uint32_t T = a.T;
    const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
    if (r >= 2 * T - 1) return;
    RefNode o;
    float box[6];
    uint32_t e;
    if (r < T) {
        e = T == 1 ? INVALID : a.pleaf[r];
        o.child_l = INVALID;
        o.child_r = INVALID;
        o.code = a.sorted_keys[r];
        o.index = a.leaf ? 3u * (__float_as_uint(a.leaf[4 * (size_t)r + 2].y) & ~LEAF_BIT) : 0u;
    } else {
        const uint32_t k = r - T;
        e = a.pint[k];
        const uint32_t cl = a.topo[k].x, cr = a.topo[k].y;
        o.child_l = (cl & LEAF_BIT) ? (cl & ~LEAF_BIT) : T + cl;
        o.child_r = (cr & LEAF_BIT) ? (cr & ~LEAF_BIT) : T + cr;
        o.code = 0;
        o.index = 0;
    }
    if (e == INVALID) {
        o.parent = INVALID;
        for (int k = 0; k < 6; k++) box[k] = a.rootbox[k];
    } else {
        o.parent = (e >> 1) + T;
        if (a.rec_on) record_box(a.rec + slot_of(a.pint[e >> 1], T), e & 1u, box);   // from the parent's record
        else child_box(a, r < T ? LEAF_BIT | r : r - T, box);                          // (or the node boxes)
    }
    for (int k = 0; k < 3; k++) { o.bb_min[k] = box[k]; o.bb_max[k] = box[3 + k]; }
    out[r] = o;
}

inline uint32_t blocks_for(size_t n) { return (uint32_t)((n + BLOCK - 1) / BLOCK); }

}  // namespace

void launch_bounds(const BuildArgs& a, hipStream_t s) {
    uint32_t blocks = blocks_for(a.V);
    if (blocks > BOUNDS_BLOCKS) blocks = BOUNDS_BLOCKS;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_bounds, dim3(blocks), dim3(BLOCK), 0, s, a.opos, a.V, a.bounds);
    hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(BLOCK), 0, s, a.bounds, blocks);
}
void launch_morton(const BuildArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_morton, dim3(blocks_for(a.T)), dim3(BLOCK), 0, s, a);
}
void launch_karras(const BuildArgs& a, hipStream_t s) {
    if (a.T < 2) return;
    if (a.delta_mode == 0) hipLaunchKernelGGL(k_karras<0>, dim3(blocks_for(a.T)), dim3(BLOCK), 0, s, a);
    else hipLaunchKernelGGL(k_karras<1>, dim3(blocks_for(a.T)), dim3(BLOCK), 0, s, a);
}
uint32_t small_build_max() { return SMALL_T; }
uint32_t small_sort_max() { return 8 * SMALL_BLOCK; }
void launch_morton_sort_small(const BuildArgs& a, hipStream_t s) {
    uint32_t* sk = const_cast<uint32_t*>(a.sorted_keys);
    uint32_t* sv = const_cast<uint32_t*>(a.sorted_vals);
    if (a.T <= 4 * SMALL_BLOCK)
        hipLaunchKernelGGL(k_morton_sort_small<4>, dim3(1), dim3(SMALL_BLOCK), 0, s, a, sk, sv);
    else
        hipLaunchKernelGGL(k_morton_sort_small<8>, dim3(1), dim3(SMALL_BLOCK), 0, s, a, sk, sv);
}
void launch_build_small(const BuildArgs& a, hipStream_t s) {
    uint32_t* sk = const_cast<uint32_t*>(a.sorted_keys);
    uint32_t* sv = const_cast<uint32_t*>(a.sorted_vals);
    if (a.delta_mode == 0) hipLaunchKernelGGL(k_build_small<0>, dim3(1), dim3(SMALL_BLOCK), 0, s, a, sk, sv);
    else hipLaunchKernelGGL(k_build_small<1>, dim3(1), dim3(SMALL_BLOCK), 0, s, a, sk, sv);
}
void launch_qnodes(const BuildArgs& a, hipStream_t s) {
    if (a.T > 1)
        hipLaunchKernelGGL(k_qnodes, dim3((a.T - 1 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, a.rec, a.pint, a.inner,
                           a.qnode, a.T);
}
uint32_t refit_blocks(uint32_t T) { return (T + RBLOCK - 1) / RBLOCK; }
// the leaves' depth range: rootbox[6..7] = min lo.z, max hi.z over k_refit's per-block ranges, and
// rootbox[8] = the largest leaf edge bound (the bounce walk's margin, margin.h)
__global__ __launch_bounds__(1024) void k_zrange(const float* __restrict__ zpart, uint32_t nb, float* __restrict__ rootbox) {
    __shared__ float s_z[3 * 16];
    float zl = INFINITY, zh = -INFINITY, em = 0.f;
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) {
        zl = fminf(zl, zpart[ZPART * b]);
        zh = fmaxf(zh, zpart[ZPART * b + 1]);
        em = fmaxf(em, zpart[ZPART * b + 2]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        zl = fminf(zl, __shfl_xor(zl, off, 64));
        zh = fmaxf(zh, __shfl_xor(zh, off, 64));
        em = fmaxf(em, __shfl_xor(em, off, 64));
    }
    if ((threadIdx.x & 63u) == 0) {
        s_z[3 * (threadIdx.x >> 6)] = zl;
        s_z[3 * (threadIdx.x >> 6) + 1] = zh;
        s_z[3 * (threadIdx.x >> 6) + 2] = em;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < 16; w++) {
            zl = fminf(zl, s_z[3 * w]);
            zh = fmaxf(zh, s_z[3 * w + 1]);
            em = fmaxf(em, s_z[3 * w + 2]);
        }
        rootbox[6] = zl;
        rootbox[7] = zh;
        rootbox[8] = em;
    }
}
void launch_refit_leaves(const BuildArgs& a, hipStream_t s) {
    const uint32_t nb = refit_blocks(a.T);
    if (a.pseudo) hipLaunchKernelGGL(k_refit<true>, dim3(nb), dim3(RBLOCK), 0, s, a);
    else hipLaunchKernelGGL(k_refit<false>, dim3(nb), dim3(RBLOCK), 0, s, a);
    hipLaunchKernelGGL(k_zrange, dim3(1), dim3(1024), 0, s, a.zpart, nb, a.rootbox);
}
void launch_pb_count_top(const BuildArgs& b, const TraceArgs& a, uint32_t* off, uint32_t* cur, uint4* bins, uint32_t cap,
                         uint32_t ntx, uint32_t leaf_blocks, hipStream_t s) {
    const uint32_t nb = refit_blocks(b.T);
    // the grouped climb first, then its list's QNodes beside the count
    const uint32_t nlate = b.T > RBLOCK ? min(1024u, (nb + 15) / 16) : 0u;
    if (nlate) hipLaunchKernelGGL(k_refit_group, dim3((nb + RGROUP - 1) / RGROUP), dim3(GBLOCK), 0, s, b);
    hipLaunchKernelGGL(k_pb_count_late, dim3(nlate + leaf_blocks), dim3(BLOCK), 0, s, b, a, nlate, off, cur, bins, cap, ntx);
}
void launch_refit_tail(const BuildArgs& a, hipStream_t s) {
    const uint32_t nb = refit_blocks(a.T);
    if (a.T > RBLOCK) {   // the crossing nodes: climbed (in LDS within a group, then across), then quantized
        hipLaunchKernelGGL(k_refit_group, dim3((nb + RGROUP - 1) / RGROUP), dim3(GBLOCK), 0, s, a);
        hipLaunchKernelGGL(k_qnodes_late, dim3(min(1024u, (nb + 15) / 16)), dim3(BLOCK), 0, s, a);
    }
}
// leaf j's pseudo-record from its leaf record's box (the bytes k_refit<true> writes)
__global__ __launch_bounds__(BLOCK) void k_pseudo(const float4* __restrict__ leaf, const uint32_t* __restrict__ pleaf,
                                                  Inner* __restrict__ rec, uint32_t T) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= T) return;
    const float4 b0 = leaf[4 * (size_t)j + 2], b1 = leaf[4 * (size_t)j + 3];
    store_pseudo_record(rec + pleaf[j], LEAF_BIT | j, mk(b0.z, b0.w, b1.x), mk(b1.y, b1.z, b1.w));
}
void launch_pseudo(const BuildArgs& a, hipStream_t s) {
    if (a.T > 1) hipLaunchKernelGGL(k_pseudo, dim3((a.T + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, a.leaf, a.pleaf, a.rec, a.T);
}
void launch_refit(const BuildArgs& a, hipStream_t s) {
    launch_refit_leaves(a, s);
    launch_refit_tail(a, s);
}
void launch_records(const BuildArgs& a, hipStream_t s) {
    if (a.T > 1) hipLaunchKernelGGL(k_records, dim3(blocks_for(a.T - 1)), dim3(BLOCK), 0, s, a);
}
void launch_nbox(const BuildArgs& a, hipStream_t s) {
    if (a.T > 1) hipLaunchKernelGGL(k_nbox, dim3(blocks_for(a.T - 1)), dim3(BLOCK), 0, s, a);
}
void launch_export(const BuildArgs& a, void* out, hipStream_t s) {
    hipLaunchKernelGGL(k_export, dim3(blocks_for(2 * (size_t)a.T - 1)), dim3(BLOCK), 0, s, a, (RefNode*)out);
}
void launch_from_codes(const BuildArgs& a, const float* leaf_boxes, hipStream_t s) {
    if (a.delta_mode == 0) hipLaunchKernelGGL(k_karras<0>, dim3(blocks_for(a.T)), dim3(BLOCK), 0, s, a);
    else hipLaunchKernelGGL(k_karras<1>, dim3(blocks_for(a.T)), dim3(BLOCK), 0, s, a);
    if (a.T > 1) (void)hipMemsetAsync(a.refit_cnt, 0, sizeof(uint32_t) * (a.T - 1), s);
    hipLaunchKernelGGL(k_refit_boxes, dim3(blocks_for(a.T)), dim3(BLOCK), 0, s, a, leaf_boxes);
    launch_qnodes(a, s);
}

}  // namespace rtbvh
