// trace.hip -- closest-hit traversal + shading kernels for gfx950.
//
// RayTraceLaunch.hlsl (primary rays, 15x15 thread groups) and
// RayTraceReflection.hlsl (bounce, every pixel re-dispatched, idle lanes for
// rays with intensity 0) on top of findCollision (RayTraceTraversal.hlsl:106-193).
// Here: a wave64 traces one 8x8 pixel tile (a 256-thread workgroup = 4 tiles
// side by side in one 8-row band, which is also the multi-GPU sharding unit);
// every child-pair test reads ONE 64-B node record; leaves read a 64-B record
// holding the clip-space triangle as (v0, e1 = v1-v0, e2 = v2-v0) -- the same
// floats the reference computes per test -- so getUpdateVerts and the edge
// subtractions are hoisted to the build; the bounce pass runs only over a
// wave-compacted queue of live rays (ballot + one atomic per wave).
//
// Traversal orders (DESIGN.md "Traversal"):
//  * reference order (default): the left-first DFS of findCollision exactly,
//    same pruning, strict `<` replacement -> bit-identical to the CPU oracle;
//  * nearest-first (RTBVH_FLAG_NEAREST_FIRST): the nearer child first, with the
//    lexicographic (t, leaf index) minimum kept, which is what the left-first DFS
//    returns whenever box/triangle rounding is consistent.
// The walks that lost their A/B measurements are not compiled here.
//
// Stack limit: the reference keeps a 32-entry stack and never checks it
// (RayTraceTraversal.hlsl:9,115,187).  Every walk here checks its own stack against
// a run-time limit (TraceArgs::stack_limit, <= the compiled capacity); a ray that would
// overflow ends with the best hit found so far, counts into counters[8] (the last
// trace's stats) and into *overflow (never reset: the API turns a change of it into
// RTBVH_ERR_STACK_OVERFLOW).  The walk-length guard (2T + 2 steps, only a cyclic tree
// from the CPUTests delta can trip it) counts the same way.
#include "rtbvh_internal.h"

namespace rtbvh {
namespace {

constexpr uint32_t BLOCK = 256;
constexpr float EPSILON = 0.01f;   // RayTraceTraversal.hlsl:7

struct Counts { uint32_t internal, leaf, overflow, wint, wleaf; };   // w*: packet wave steps (lane 0)

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

// Node records live in SLOTS (rtbvh_device.h): the binary walks keep slots on their
// stacks.  The record of internal node k holds k's own index, so its internal
// children's records are at slots 2k and 2k+1; a leaf child is LEAF_BIT | j.
__device__ __forceinline__ uint32_t child_slot(uint32_t id, uint32_t own, uint32_t side) {
    return (id & LEAF_BIT) ? id : 2 * own + side;
}
__device__ __forceinline__ uint32_t root_slot(uint32_t T) { return T == 1 ? LEAF_BIT : 2 * T - 2; }

// Make loaded values live at this point, so the compiler issues every load of a
// record together (one memory round trip) instead of sinking some of them below
// an early-exit branch that needs only part of the record (ISA showed the leaf's
// v0 fetched in a second dependent round trip after the determinant test).
__device__ __forceinline__ void pin(float4& a) {
    float x = a.x, y = a.y, z = a.z, w = a.w;
    asm volatile("" : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
    a = make_float4(x, y, z, w);
}
__device__ __forceinline__ void pin(float& a) { asm volatile("" : "+v"(a)); }
__device__ __forceinline__ void pin(v4f& a) { asm volatile("" : "+v"(a)); }

// rayTriangleCollision, RayTraceTraversal.hlsl:41-86, with edge1/edge2 precomputed
// by the build (identical floats: the same single subtraction)
__device__ __forceinline__ float ray_triangle(f3 o, f3 d, f3 p0, f3 e1, f3 e2) {
    f3 tmp = cross(d, e2);
    const float dx = dot(e1, tmp);
    if (fabsf(dx) < EPSILON) return -1.f;
    const float idx = 1.f / dx;
    const f3 rt = sub(o, p0);
    const float u = dot(rt, tmp) * idx;
    if (u < .0f || 1.f < u) return -1.f;
    tmp = cross(rt, e1);
    const float v = dot(d, tmp) * idx;
    if (v < .0f || 1.f < u + v) return -1.f;
    const float t = dot(e2, tmp) * idx;
    if (EPSILON < t) return t;
    return -1.f;
}

// rayBoxCollision, RayTraceTraversal.hlsl:92-104 (fminf/fmaxf drop NaN like HLSL
// min/max).  Also returns the entry distance, used by the nearest-first order.
__device__ __forceinline__ bool ray_box(f3 o, f3 inv, float bx0, float by0, float bz0, float bx1, float by1, float bz1,
                                        bool hit, float best, float& tmin) {
    const float tx0 = (bx0 - o.x) * inv.x, ty0 = (by0 - o.y) * inv.y, tz0 = (bz0 - o.z) * inv.z;
    const float tx1 = (bx1 - o.x) * inv.x, ty1 = (by1 - o.y) * inv.y, tz1 = (bz1 - o.z) * inv.z;
    const float mn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
    const float mx = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    tmin = mn;
    return 0 <= mx && mn <= mx && (!hit || mn <= best);
}

// ray_box on a node record's layout (rtbvh_device.h): the (x, y) of a box corner is an
// aligned register pair, so the x and y slabs run as packed fp32 (v_pk_add_f32 /
// v_pk_mul_f32: two IEEE operations per instruction, the roundings of the scalar form,
// no contraction under -ffp-contract=off).
__device__ __forceinline__ bool ray_box_xy(f3 o, f3 inv, f2v lo, f2v hi, float lz, float hz, bool hit, float best,
                                           float& tmin) {
    const f2v oxy = {o.x, o.y}, ixy = {inv.x, inv.y};
    const f2v t0 = (lo - oxy) * ixy, t1 = (hi - oxy) * ixy;
    const float tz0 = (lz - o.z) * inv.z, tz1 = (hz - o.z) * inv.z;
    const float mn = fmaxf(fmaxf(fminf(t0.x, t1.x), fminf(t0.y, t1.y)), fminf(tz0, tz1));
    const float mx = fminf(fminf(fmaxf(t0.x, t1.x), fmaxf(t0.y, t1.y)), fmaxf(tz0, tz1));
    tmin = mn;
    return 0 <= mx && mn <= mx && (!hit || mn <= best);
}

// findCollision, RayTraceTraversal.hlsl:106-193.  The reference keeps stack[0] = -1
// and loops `do { ... } while (stackIndex != -1)`; here the entry at the top of
// the stack is cached in a register (`top`), so a pop hands over the next node at
// once and refills `top` from scratch in the background.  Returns hit;
// best_leaf = sorted leaf index.  `limit` <= STACK_SIZE entries.
// LSB > 0: stack entries [0, LSB) in LDS (`lst`: this lane's column, entry k at lst[k * BLOCK]; a
// wave's lanes on 64 distinct banks), deeper ones in scratch (the one-ray-per-lane kernels).  The pop
// compiles to one flat load of a selected pointer (LDS or scratch); forcing ds_read (a module-scope
// array, every lane reading LDS and the deeper ones scratch as well) was 1-2% slower at C3
#ifndef RTBVH_LANE_LSB
#define RTBVH_LANE_LSB 16
#endif
constexpr int LANE_LSB = RTBVH_LANE_LSB;
template <bool COUNT, bool NEAREST, int LSB = 0>
__device__ __forceinline__ bool traverse(const Inner* __restrict__ inner, const float4* __restrict__ leaf, uint32_t T,
                                         f3 o, f3 d, f3 inv, int limit, float& best, uint32_t& best_leaf, Counts& c,
                                         uint32_t* lst = nullptr) {
    bool hit = false;
    best = 0.f;
    best_leaf = 0;
    uint32_t stack[STACK_SIZE];   // reference entries [0, sp) below the cached top
    int sp = 0;                   // reference stack index; stack[0] is the sentinel = top at start
    uint32_t top = INVALID;
    uint32_t node = root_slot(T);
    uint32_t guard = 2 * T + 2;   // a valid tree is walked in <= 2T-1 steps
    do {
        if (--guard == 0) { c.overflow++; break; }
        if (node & LEAF_BIT) {
            const uint32_t j = node & ~LEAF_BIT;
            const float4* r = leaf + 4 * (size_t)j;
            float4 a = r[0], b = r[1];
            float e2z = r[2].x;
            pin(a); pin(b); pin(e2z);
            if (COUNT) c.leaf++;
            const float t = ray_triangle(o, d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, e2z));
            if (t != -1.f && (!hit || t < best || (NEAREST && t == best && j < best_leaf))) {
                best = t;
                best_leaf = j;
                hit = true;
            }
            node = top;                                 // pop
            if (--sp >= 0) top = LSB > 0 && sp < LSB ? lst[sp * BLOCK] : stack[sp];
            continue;
        }
        if (COUNT) c.internal++;
        const v4f* r = reinterpret_cast<const v4f*>(inner + node);
        const v4f q0 = r[0], q1 = r[1], q2 = r[2];
        const uint4 q3 = reinterpret_cast<const uint4*>(r)[3];
        const uint32_t cl = child_slot(q3.x, q3.z, 0), cr = child_slot(q3.y, q3.z, 1);
        float tl, tr;
        const bool lh = ray_box_xy(o, inv, q0.xy, q0.zw, q2.x, q2.y, hit, best, tl);
        const bool rh = ray_box_xy(o, inv, q1.xy, q1.zw, q2.z, q2.w, hit, best, tr);
        if (!lh && !rh) {
            node = top;                                 // pop
            if (--sp >= 0) top = LSB > 0 && sp < LSB ? lst[sp * BLOCK] : stack[sp];
        } else {
            const bool swap = NEAREST && lh && rh && tr < tl;
            if (lh && rh) {
                if (sp + 1 >= limit) {
                    c.overflow++;
                    node = top;
                    if (--sp >= 0) top = LSB > 0 && sp < LSB ? lst[sp * BLOCK] : stack[sp];
                    continue;
                }
                if (LSB > 0 && sp < LSB) lst[sp * BLOCK] = top;   // push the second child
                else stack[sp] = top;
                sp++;
                top = swap ? cl : cr;
            }
            node = swap ? cr : (lh ? cl : cr);
        }
    } while (sp != -1);
    return hit;
}

// traverse<COUNT, false> (findCollision, the reference order) on the topology and the node boxes, for a build that
// wrote no node records (api.hip: a certified-only context's): at internal node k its children from topo[k], their
// boxes from nbox (internal) or the leaf record (words 10..15), the same slab test in the same operations -- the same
// visits, in the same order, and the same hit.  Two dependent fetches a step instead of one: the certified walks'
// few re-traced rays only.
__device__ __forceinline__ void nb_child_box(const float* __restrict__ nbox, const float4* __restrict__ leaf, uint32_t c,
                                             f2v& mnxy, f2v& mxxy, float& mnz, float& mxz) {
    if (c & LEAF_BIT) {
        const float4* r = leaf + 4 * (size_t)(c & ~LEAF_BIT);
        const float4 w2 = r[2], w3 = r[3];
        mnxy = f2v{w2.z, w2.w}; mnz = w3.x; mxxy = f2v{w3.y, w3.z}; mxz = w3.w;
    } else {
        const float2* d = reinterpret_cast<const float2*>(nbox + 6 * (size_t)c);
        const float2 x = d[0], y = d[1], z = d[2];
        mnxy = f2v{x.x, x.y}; mnz = y.x; mxxy = f2v{y.y, z.x}; mxz = z.y;
    }
}
template <bool COUNT>
__device__ __forceinline__ bool traverse_nb(const uint4* __restrict__ topo, const float* __restrict__ nbox,
                                            const float4* __restrict__ leaf, uint32_t T, f3 o, f3 d, f3 inv,
                                            float& best, uint32_t& best_leaf, Counts& c) {
    bool hit = false;
    best = 0.f;
    best_leaf = 0;
    uint32_t stack[STACK_SIZE];
    int sp = 0;
    uint32_t top = INVALID;
    uint32_t node = T > 1 ? 0u : LEAF_BIT;   // the root: internal node 0 (a one-leaf tree: the leaf)
    uint32_t guard = 2 * T + 2;
    do {
        if (--guard == 0) { c.overflow++; break; }
        if (node & LEAF_BIT) {
            const uint32_t j = node & ~LEAF_BIT;
            const float4* r = leaf + 4 * (size_t)j;
            float4 a = r[0], b = r[1];
            float e2z = r[2].x;
            pin(a); pin(b); pin(e2z);
            if (COUNT) c.leaf++;
            const float t = ray_triangle(o, d, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, e2z));
            if (t != -1.f && (!hit || t < best)) {
                best = t;
                best_leaf = j;
                hit = true;
            }
            node = top;
            if (--sp >= 0) top = stack[sp];
            continue;
        }
        if (COUNT) c.internal++;
        const uint4 q = topo[node];
        const uint32_t cl = q.x, cr = q.y;
        f2v lmn, lmx, rmn, rmx;
        float lz0, lz1, rz0, rz1;
        nb_child_box(nbox, leaf, cl, lmn, lmx, lz0, lz1);
        nb_child_box(nbox, leaf, cr, rmn, rmx, rz0, rz1);
        float tl, tr;
        const bool lh = ray_box_xy(o, inv, lmn, lmx, lz0, lz1, hit, best, tl);
        const bool rh = ray_box_xy(o, inv, rmn, rmx, rz0, rz1, hit, best, tr);
        if (!lh && !rh) {
            node = top;
            if (--sp >= 0) top = stack[sp];
        } else {
            if (lh && rh) {
                if (sp + 1 >= STACK_SIZE) {
                    c.overflow++;
                    node = top;
                    if (--sp >= 0) top = stack[sp];
                    continue;
                }
                stack[sp] = top;
                sp++;
                top = cr;
            }
            node = lh ? cl : cr;
        }
    } while (sp != -1);
    return hit;
}
// the reference-order walk of a re-traced ray: on the records, or (a.nb) the topology and node boxes
template <bool COUNT>
__device__ __forceinline__ bool traverse_ref(const TraceArgs& a, f3 o, f3 d, f3 inv, float& best, uint32_t& bl,
                                             Counts& c) {
    return a.nb ? traverse_nb<COUNT>(a.topo, a.nbox, a.leaf, a.T, o, d, inv, best, bl, c)
                : traverse<COUNT, false>(a.inner, a.leaf, a.T, o, d, inv, STACK_SIZE, best, bl, c);
}

// ---- wave-packet traversal (primary rays) -------------------------------------
// The 64 rays of an 8x8 pixel tile are nearly parallel neighbours, so a wave walks
// ONE node at a time with a per-node lane mask: the node record is fetched by the
// scalar unit (s_load through the constant address space: no vector-memory/TA
// work, which PMC showed saturated), each masked lane tests the child boxes with
// its own (hit, best), and the children are visited with the ballots of the lanes
// that hit them.  In reference order every lane sees exactly its own findCollision
// sequence (the nodes it visits are a subsequence of the wave's walk, in the same
// order, and nothing changes its state in between), so results and per-lane visit
// counts are identical to the per-lane DFS.  In nearest-first mode the wave takes
// the child most of its lanes see first.
typedef float v16f __attribute__((ext_vector_type(16)));
typedef const v16f __attribute__((address_space(4))) cv16f;

// the whole 64-B record in one s_load_dwordx16 (one scalar-memory round trip per step)
__device__ __forceinline__ v16f sload16(const void* p) { return *(cv16f*)p; }

template <bool COUNT, bool NEAREST>
__device__ __forceinline__ bool traverse_packet(const Inner* __restrict__ inner, const float4* __restrict__ leaf,
                                                uint32_t T, f3 o, f3 d, f3 inv, bool valid, int limit, float& best,
                                                uint32_t& best_leaf, Counts& c, uint32_t* s_st /* per wave [3*STACK_SIZE] */) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lanebit = 1ull << lane;
    bool hit = false;
    best = 0.f;
    best_leaf = 0;
    uint64_t mask = __ballot(valid);
    int sp = 0;                      // entries on the wave stack; the top one is cached below
    uint32_t node = root_slot(T), top_node = 0;
    uint64_t top_mask = 0;
    if (mask == 0) return false;
    uint32_t guard = 2 * T + 2;
    while (true) {
        if (--guard == 0) { c.overflow += valid; break; }   // the wave's rays in the frame end early
        bool pop = false;
        if (node & LEAF_BIT) {
            const uint32_t j = node & ~LEAF_BIT;
            const v16f q = sload16(leaf + 4 * (size_t)j);
            if (COUNT && lane == 0) c.wleaf++;
            if (mask & lanebit) {
                if (COUNT) c.leaf++;
                const float t = ray_triangle(o, d, mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]));
                if (t != -1.f && (!hit || t < best || (NEAREST && t == best && j < best_leaf))) {
                    best = t;
                    best_leaf = j;
                    hit = true;
                }
            }
            pop = true;
        } else {
            const v16f q = sload16(inner + node);
            if (COUNT && lane == 0) c.wint++;
            const uint32_t own = __float_as_uint(q[14]);
            const uint32_t cl = child_slot(__float_as_uint(q[12]), own, 0), cr = child_slot(__float_as_uint(q[13]), own, 1);
            bool lh = false, rh = false;
            float tl = 0.f, tr = 0.f;
            if (mask & lanebit) {
                if (COUNT) c.internal++;
                lh = ray_box_xy(o, inv, q.s01, q.s23, q[8], q[9], hit, best, tl);
                rh = ray_box_xy(o, inv, q.s45, q.s67, q[10], q[11], hit, best, tr);
            }
            const uint64_t ml = __ballot(lh), mr = __ballot(rh);
            if ((ml | mr) == 0) {
                pop = true;
            } else if (ml && mr) {
                bool swap = false;
                if (NEAREST) {
                    const uint64_t both = __ballot(lh && rh);
                    const uint64_t rfirst = __ballot(lh && rh && tr < tl);
                    swap = 2 * __popcll(rfirst) > __popcll(both);
                }
                if (sp + 1 >= limit) {   // the lanes of both children lose them
                    c.overflow += ((ml | mr) & lanebit) != 0;
                    pop = true;
                } else {
                    // push the second child and its lanes: the old top goes to LDS, the
                    // new entry stays in SGPRs (top cache, as in the per-lane loop)
                    if (sp > 0 && lane == 0) {
                        s_st[3 * sp] = top_node;
                        s_st[3 * sp + 1] = (uint32_t)top_mask;
                        s_st[3 * sp + 2] = (uint32_t)(top_mask >> 32);
                    }
                    ++sp;
                    top_node = swap ? cl : cr;
                    top_mask = swap ? ml : mr;
                    node = swap ? cr : cl;
                    mask = swap ? mr : ml;
                }
            } else {
                node = ml ? cl : cr;
                mask = ml ? ml : mr;
            }
        }
        if (pop) {
            if (sp == 0) break;
            node = top_node;
            mask = top_mask;
            if (--sp > 0) {   // refill the cached top from LDS (lane 0's earlier write)
                top_node = __builtin_amdgcn_readfirstlane(s_st[3 * sp]);
                const uint32_t lo = __builtin_amdgcn_readfirstlane(s_st[3 * sp + 1]);
                const uint32_t hi = __builtin_amdgcn_readfirstlane(s_st[3 * sp + 2]);
                top_mask = ((uint64_t)hi << 32) | lo;
            }
        }
    }
    return hit;
}

// ray_triangle without early exits, for the packet walk's leaf step: every lane evaluates
// the same operations, and each rejection of the reference's order becomes a select of -1
// (pinned, so the six tests stay VALU selects rather than lane masks combined on the SALU).
// The same floats and the same accept predicate: the same result.  `in` false also gives -1.
__device__ __forceinline__ float ray_triangle_flat(f3 o, f3 d, f3 p0, f3 e1, f3 e2, bool in) {
    const f3 tmp = cross(d, e2);
    const float dx = dot(e1, tmp);
    const float idx = recip(dx);
    const f3 rt = sub(o, p0);
    const float u = dot(rt, tmp) * idx;
    const f3 q = cross(rt, e1);
    const float v = dot(d, q) * idx;
    const float t = dot(e2, q) * idx;
    float r = EPSILON < t ? t : -1.f;
    pin(r);
    r = fabsf(dx) < EPSILON ? -1.f : r;
    pin(r);
    r = u < .0f ? -1.f : r;
    pin(r);
    r = 1.f < u ? -1.f : r;
    pin(r);
    r = v < .0f ? -1.f : r;
    pin(r);
    r = 1.f < u + v ? -1.f : r;
    pin(r);
    return in ? r : -1.f;
}

// (t, leaf) of the best hit as one u64 key, t's bits above: t > EPSILON > 0, so the u64 order is
// the (t, leaf) order; before any hit (+inf, ~0), which every hit beats.  The entry distance of a
// box is then compared with the key's t alone: with no hit it is +inf, and a box whose entry is
// not <= +inf (NaN) fails the slab test's own mn <= mx too, as the reference's !hit || ... does.
constexpr uint64_t NO_HIT = 0x7F800000FFFFFFFFull;
__device__ __forceinline__ float key_t(uint64_t key) { return __uint_as_float((uint32_t)(key >> 32)); }
// a bounce hit record's word (the triangle, INVALID for a miss) with bit 30 flipped: the certified walk
// could not vouch for the ray (k_bounce_trav CERT); the shading hands it to the reference-order re-trace
constexpr uint32_t HIT_FLAG = 0x40000000u;
__device__ __forceinline__ bool hit_flagged(uint32_t w) { return ((w >> 31) ^ (w >> 30)) & 1u; }

// v_writelane_b32: lane K of v := the wave-uniform s (a VALU op, no scalar work)
template <int K> __device__ __forceinline__ void writelane(uint32_t& v, uint32_t s) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "i"(K));
}

// ---- wave-packet traversal on the 4-wide view (primary rays) -------------------
// As traverse_packet, but one step reads the 128-B record pair inner4[2p], inner4[2p+1]
// (two s_load_dwordx16 of one line): the boxes of p's four grandchildren.  Children are
// taken left to right (the left-first DFS's order LL, LR, RL, RR); the per-lane result is
// the (t, leaf) minimum, as for the 4-wide bounce walk.
//
// Axis-parallel box test: the rays run along d = (0, 0, 1) from z = 0 (k_primary), so
// inv = (inf, inf, 1) and each x/y slab of ray_box_xy yields [-inf, inf] (or NaNs that
// fminf/fmaxf drop) exactly when min < o < max, and an empty slab otherwise.  For a box
// whose record bit (word 15, build.hip general_box) is clear -- min < max in x and y,
// min.z <= max.z, 0 <= max.z < inf -- the test is therefore exactly
//     min.x < o.x < max.x  &&  min.y < o.y < max.y  &&  (!hit || min.z <= best)
// (denormals are kept, so min < o has the sign of min - o), evaluated as o - min and
// max - o as packed differences and min(...) > 0.  A node with any bit set takes the
// general test.
//
// Per-step work (one wave step is ~100 instructions, and 32 waves share the CU's one
// scalar unit):
//  * lanes 0..3 of (vid, vlo, vhi) hold child k's id and lane mask (v_writelane), so the hit
//    set is one ballot, the next node a v_readlane and the pushes one vector store per word;
//  * the fast box test needs no AND with the parent's lanes: a box whose bit is clear lies
//    inside its parent's box, so a lane that passes it passed the parent's test (at a bound
//    >= today's) -- lanes outside the frame get a NaN origin, which fails every fast test,
//    and a pseudo-record's absent child has a NaN min.z (build.hip store_pseudo_record);
//  * the leaf test runs on every lane without branches (ray_triangle_flat) and the (t, leaf)
//    minimum is one u64 compare;
//  * stack entry 0 is a sentinel, so a pop has no empty-stack test and the loop one exit.
// A/B at C5 (10M triangles, 3840x2160, frame identical): 2.60 ms for the per-child lane-0
// pushes with the parent-mask AND, 2.23 with the lanes-0..3 form, 2.20 with the sentinel and
// the NaN min.z, 2.18 with the z test as its own lane mask (VALU -> SALU); a branchless tail
// (descend or pop by selects, the stack top read at the step's start) ran 2.45.
// GUARD false (a clz64 tree, k_primary walk 5): no walk-length guard, and without a run-time
// stack limit (CHECK false) no stack check either: a clz64 tree has <= 64 internal levels (each
// child's common-prefix length exceeds its parent's, 0..63), a step descends two levels and
// pushes <= 3 entries, so the stack holds <= 3 * 32 + 1 < STACK4 + 1 entries.
// No lane masks on the stack: a wave needs the lanes that reach a node only at a leaf (which
// lanes test its triangle), and those are the lanes whose ray passes the leaf's own box with the
// current bound -- its record holds the box (words 10..15), so the leaf step tests it again, with
// the fast or the general form as the parent step did.  Every lane the parent step let through
// passes it unless its bound has since fallen below the box's entry, and such a lane cannot improve
// its (t, leaf) minimum there.  Internal steps never needed the masks (a child's box lies inside its
// parent's, and the slab test is monotone in the box), so a stack entry is a node id alone: one
// v_writelane per child for its id and one for its any-lane bit instead of three, one word per push
// and pop.  The visit counters (COUNT) still keep each entry's lanes, beside the same walk.
template <bool COUNT, bool GUARD, bool CHECK>
__device__ __forceinline__ bool traverse_packet4(const Inner* __restrict__ inner4, const float4* __restrict__ leaf,
                                                 uint32_t T, f3 o, f3 d, f3 inv, bool valid, int limit, float& best,
                                                 uint32_t& best_leaf, Counts& c, uint32_t* s_st /* [3*(STACK4+1)] */) {
    constexpr int EW = COUNT ? 3 : 1;   // words per stack entry: the node, and its lanes for the counters
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t mask = __ballot(valid);
    best = 0.f;
    best_leaf = 0;
    if (mask == 0) return false;
    const float qnan = __builtin_nanf("");
    const f2v oxy = valid ? f2v{o.x, o.y} : f2v{qnan, qnan};
    uint64_t key = NO_HIT;
    uint32_t vid = 0, vlo = 0, vhi = 0;
    // entry 0 is a sentinel (node INVALID): popping it ends the walk, so a pop needs no
    // empty-stack test and the loop has one exit
    if (lane == 0) s_st[0] = INVALID;
    int sp = 1;
    uint32_t node = (T == 1) ? LEAF_BIT : 0u;
    uint32_t guard = 2 * T + 2;
    do {
        node = __builtin_amdgcn_readfirstlane(node);
        if (node & LEAF_BIT) {
            const uint32_t j = node & ~LEAF_BIT;
            const v16f q = sload16(leaf + 4 * (size_t)j);
            if (COUNT && lane == 0) c.wleaf++;
            // the lanes that need this leaf: its own box {min q[10..12], max q[13..15]}, tested as the
            // parent step tested it (rtbvh_device.h word 15: the fast form for a box that allows it)
            const float lx = q[10], ly = q[11], lz = q[12], hx = q[13], hy = q[14], hz = q[15];
            const float bound = __uint_as_float((uint32_t)(key >> 32));
            bool in;
            if (!(__float_as_uint(q[9]) & LEAF_BIT)) {   // the box allows the fast form (build.hip leaf_tri_word)
                const f2v d0 = oxy - f2v{lx, ly}, d1 = f2v{hx, hy} - oxy;
                in = fminf(fminf(d0.x, d0.y), fminf(d1.x, d1.y)) > 0.f && lz <= bound;
            } else {
                const bool hit = key != NO_HIT;
                float tt;
                in = valid && ray_box_xy(o, inv, f2v{lx, ly}, f2v{hx, hy}, lz, hz, hit, hit ? bound : 0.f, tt);
            }
            if (COUNT) c.leaf += (mask >> lane) & 1u;
            const float t =
                ray_triangle_flat(o, d, mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), in);
            const uint64_t k = t == -1.f ? ~0ull : (uint64_t)__float_as_uint(t) << 32 | j;
            key = k < key ? k : key;
        } else {
            const v16f A = sload16(inner4 + 2 * (size_t)node);
            const v16f B = sload16(inner4 + 2 * (size_t)node + 1);
            if (COUNT && lane == 0) c.wint++;
            if (COUNT) c.internal += (mask >> lane) & 1u;
            const uint32_t id0 = __float_as_uint(A[12]), id1 = __float_as_uint(A[13]);
            const uint32_t id2 = __float_as_uint(B[12]), id3 = __float_as_uint(B[13]);
            uint64_t m0, m1, m2, m3;
            const float bound = __uint_as_float((uint32_t)(key >> 32));
            if ((__float_as_uint(A[15]) | __float_as_uint(B[15])) == 0) {   // wave-uniform
                // min(o - lo, hi - o) > 0 with lz <= bound folded in as a select (pinned, so the
                // compiler keeps it a VALU select instead of ANDing two lane masks on the SALU)
                const auto lanes = [&](f2v lo, f2v hi, float lz) {
                    const f2v d0 = oxy - lo, d1 = hi - oxy;
                    float m = fminf(fminf(d0.x, d0.y), fminf(d1.x, d1.y));
                    return __builtin_amdgcn_ballot_w64(m > 0.f) & __builtin_amdgcn_ballot_w64(lz <= bound);
                };
                m0 = lanes(A.s01, A.s23, A[8]);
                m1 = lanes(A.s45, A.s67, A[10]);
                m2 = lanes(B.s01, B.s23, B[8]);
                m3 = lanes(B.s45, B.s67, B[10]);
            } else {
                const bool hit = key != NO_HIT;
                const float bst = hit ? bound : 0.f;
                bool h0 = false, h1 = false, h2 = false, h3 = false;
                float t0, t1, t2, t3;
                if (valid) {   // a lane the parent let not through fails these too (monotone)
                    h0 = ray_box_xy(o, inv, A.s01, A.s23, A[8], A[9], hit, bst, t0);
                    h1 = ray_box_xy(o, inv, A.s45, A.s67, A[10], A[11], hit, bst, t1) & (id1 != INVALID);
                    h2 = ray_box_xy(o, inv, B.s01, B.s23, B[8], B[9], hit, bst, t2);
                    h3 = ray_box_xy(o, inv, B.s45, B.s67, B[10], B[11], hit, bst, t3) & (id3 != INVALID);
                }
                m0 = __ballot(h0); m1 = __ballot(h1); m2 = __ballot(h2); m3 = __ballot(h3);
            }
            writelane<0>(vid, id0);
            writelane<1>(vid, id1);
            writelane<2>(vid, id2);
            writelane<3>(vid, id3);
            if (COUNT) {
                writelane<0>(vlo, (uint32_t)m0);
                writelane<1>(vlo, (uint32_t)m1);
                writelane<2>(vlo, (uint32_t)m2);
                writelane<3>(vlo, (uint32_t)m3);
                writelane<0>(vhi, (uint32_t)(m0 >> 32));
                writelane<1>(vhi, (uint32_t)(m1 >> 32));
                writelane<2>(vhi, (uint32_t)(m2 >> 32));
                writelane<3>(vhi, (uint32_t)(m3 >> 32));
            }
            // (an absent second child -- INVALID id, a leaf's pseudo-record -- has a NaN min.z and
            // hits no lane in the fast test; the general test checks its id)
            // which children any lane hits: the OR of each mask's halves in lanes 0..3, one ballot
            // (the same from four 64-bit compares on the SALU: +45% SALU, primary +2%)
            uint32_t vor = 0;
            writelane<0>(vor, (uint32_t)m0 | (uint32_t)(m0 >> 32));
            writelane<1>(vor, (uint32_t)m1 | (uint32_t)(m1 >> 32));
            writelane<2>(vor, (uint32_t)m2 | (uint32_t)(m2 >> 32));
            writelane<3>(vor, (uint32_t)m3 | (uint32_t)(m3 >> 32));
            const uint32_t hs = (uint32_t)__builtin_amdgcn_ballot_w64(vor != 0);   // lanes >= 4 stay 0
            if (hs != 0) {
                const uint32_t rest = hs & (hs - 1);
                const int npush = __builtin_popcount(rest);
                if (!CHECK || sp + npush <= limit + 1) {
                    const uint32_t first = (uint32_t)__builtin_ctz(hs);
                    node = __builtin_amdgcn_readlane(vid, first);
                    if (COUNT)
                        mask = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(vhi, first) << 32 |
                               (uint32_t)__builtin_amdgcn_readlane(vlo, first);
                    if (((uint64_t)rest >> lane) & 1u) {   // the later a child, the deeper its entry
                        const int pos = sp + __builtin_popcount(rest >> (lane + 1));
                        s_st[EW * pos] = vid;
                        if (COUNT) {
                            s_st[EW * pos + 1] = vlo;
                            s_st[EW * pos + 2] = vhi;
                        }
                    }
                    sp += npush;
                    continue;
                }
                // the step's children are skipped: count the rays that hit one of them (once per lane,
                // not 64 per wave event)
                c.overflow += (uint32_t)(((m0 | m1 | m2 | m3) >> lane) & 1u);
            }
        }
        --sp;
        node = __builtin_amdgcn_readfirstlane(s_st[EW * sp]);
        if (COUNT) {
            const uint32_t lo = __builtin_amdgcn_readfirstlane(s_st[EW * sp + 1]);
            const uint32_t hi = __builtin_amdgcn_readfirstlane(s_st[EW * sp + 2]);
            mask = ((uint64_t)hi << 32) | lo;
        }
    } while (node != INVALID && (!GUARD || --guard != 0));
    if (GUARD && guard == 0) c.overflow += valid;
    const bool hit = key != NO_HIT;
    if (hit) { best = __uint_as_float((uint32_t)(key >> 32)); best_leaf = (uint32_t)key; }
    return hit;
}

// Primary walks: 0 per-lane reference order, 1 per-lane nearest-first,
// 2 packet reference order, 3 packet nearest-first, 4 4-wide packet (axis-parallel test),
// 5 the same without the walk-length guard (a clz64 tree has no cycles; ~6 SALU per step)
// 6: the reference order per lane on the topology and the node boxes (a certified trace's overflowed tiles and
// frames past the binned pass's size, on a build without node records: traverse_nb)
template <int K> struct PrimaryWalk {
    static constexpr bool NEAREST = (K == 1 || K == 3);
    static constexpr bool PACKET = (K >= 2 && K <= 5);
    static constexpr bool WIDE = (K == 4 || K == 5);
    static constexpr bool GUARD = (K != 5);   // 5: the 4-wide walk on a clz64 tree (acyclic)
    static constexpr bool NB = (K == 6);
};

struct HitInfo {
    float4 color;   // renderPixel(...) * specular
    f3 hitp, nrm;
    float shininess, alpha, optical_density;
    bool textured;
};

// HLSL refract(i, n, eta) as documented (see oracle refract_hlsl; same operation order)
__device__ __forceinline__ f3 refract_hlsl(f3 i, f3 n, float eta) {
    const float cosi = dot(mk(-i.x, -i.y, -i.z), n);
    const float cost2 = 1.0f - eta * eta * (1.0f - cosi * cosi);
    const float s = eta * cosi - sqrtf(fabsf(cost2));
    const f3 t = add(mul(i, eta), mul(n, s));
    const float keep = cost2 > 0.0f ? 1.0f : 0.0f;
    return mul(t, keep);
}

// RayPresent record (RayTraceGlobal.hlsl:30-35), 14 floats at 56*idx (8-B aligned):
// intensity, origin, direction, invDirection, color.  `ray` false writes a zero ray
// (fields HLSL leaves unset when the intensity is 0, and clearRayPresent on a miss).
__device__ __forceinline__ void put_record(float* rec, size_t idx, float intensity, bool ray, f3 o, f3 d,
                                           float4 color) {
    float2* r = reinterpret_cast<float2*>(rec + 14 * idx);
    if (!ray) { o = mk(0.f, 0.f, 0.f); d = o; }
    const f3 inv = ray ? mk(1.f / d.x, 1.f / d.y, 1.f / d.z) : mk(0.f, 0.f, 0.f);
    r[0] = make_float2(intensity, o.x);
    r[1] = make_float2(o.y, o.z);
    r[2] = make_float2(d.x, d.y);
    r[3] = make_float2(d.z, inv.x);
    r[4] = make_float2(inv.y, inv.z);
    r[5] = make_float2(color.x, color.y);
    r[6] = make_float2(color.z, color.w);
}

// diffuseTex[k].SampleLevel(compSample, uv, 0) as restated in include/rtbvh.h
// (rtbvh_texture): sRGB texels -> linear by table, wrap, fp32 bilinear.
__device__ __forceinline__ float4 texel(const TraceArgs& a, uint32_t first, uint32_t w, uint32_t x, uint32_t y) {
    const uint32_t p = a.texels[first + (size_t)y * w + x];
    return make_float4(a.srgb[p & 255u], a.srgb[(p >> 8) & 255u], a.srgb[(p >> 16) & 255u], (float)(p >> 24) / 255.f);
}
__device__ __forceinline__ uint32_t wrap_index(float f, uint32_t n) {
    if (!(fabsf(f) < 2147483648.f)) f = 0.f;   // NaN / huge coordinates: texel 0 (never out of bounds)
    int64_t i = (int64_t)f % (int64_t)n;
    return (uint32_t)(i < 0 ? i + n : i);
}
__device__ __forceinline__ float4 sample_texture(const TraceArgs& a, uint32_t k, float u, float v) {
    const uint4 ti = a.texinfo[k];
    const float x = u * (float)ti.y - 0.5f, y = v * (float)ti.z - 0.5f;
    const float x0 = floorf(x), y0 = floorf(y);
    const float fx = x - x0, fy = y - y0;
    const uint32_t ix = wrap_index(x0, ti.y), iy = wrap_index(y0, ti.z);
    const uint32_t ix1 = ix + 1 == ti.y ? 0u : ix + 1, iy1 = iy + 1 == ti.z ? 0u : iy + 1;
    const float4 t00 = texel(a, ti.x, ti.y, ix, iy), t10 = texel(a, ti.x, ti.y, ix1, iy);
    const float4 t01 = texel(a, ti.x, ti.y, ix, iy1), t11 = texel(a, ti.x, ti.y, ix1, iy1);
    const float4 top = make_float4(lerpf(t00.x, t10.x, fx), lerpf(t00.y, t10.y, fx), lerpf(t00.z, t10.z, fx),
                                   lerpf(t00.w, t10.w, fx));
    const float4 bot = make_float4(lerpf(t01.x, t11.x, fx), lerpf(t01.y, t11.y, fx), lerpf(t01.z, t11.z, fx),
                                   lerpf(t01.w, t11.w, fx));
    return make_float4(lerpf(top.x, bot.x, fy), lerpf(top.y, bot.y, fy), lerpf(top.z, bot.z, fy),
                       lerpf(top.w, bot.w, fy));
}

// getHitLoc (:15-19) + getNromalTexCoord (RayTraceHelper.hlsl:12-35) + renderPixel*specular
// (RayTraceRender.hlsl:16-29, RayTraceLaunch.hlsl:57-59) for the hit triangle only
// (the reference transforms all three vertices at every leaf it visits).
__device__ __forceinline__ HitInfo shade_hit_tri(const TraceArgs& a, uint32_t tri, f3 o, f3 d, float t) {
    HitInfo h;
    const float4* P = a.tclip + TCS * (size_t)tri;
    const float4 a0 = P[0], a1 = P[1], a2 = P[2];
    // vertex and material indices: the record's fourth float4 (k_morton), else the index arrays
    uint32_t vi[3], mi;
    if (TCS == 4) {
        const float4 a3 = P[3];
        vi[0] = __float_as_uint(a3.x); vi[1] = __float_as_uint(a3.y); vi[2] = __float_as_uint(a3.z);
        mi = __float_as_uint(a3.w);
    } else {
        vi[0] = a.idx[3 * (size_t)tri]; vi[1] = a.idx[3 * (size_t)tri + 1]; vi[2] = a.idx[3 * (size_t)tri + 2];
        mi = a.matidx[tri];
    }
    const f3 P0 = mk(a0.x, a0.y, a0.z), P1 = mk(a1.x, a1.y, a1.z), P2 = mk(a2.x, a2.y, a2.z);
    f3 n[3];
    float uv[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float* v = a.verts + 8 * (size_t)vi[k];
        n[k] = xform_normal(a.cam + 16, mk(v[3], v[4], v[5]));
        uv[k][0] = v[6];
        uv[k][1] = v[7];
    }
    h.hitp = add(o, mul(d, t));
    const f3 v0 = sub(P0, h.hitp), v1 = sub(P1, h.hitp), v2 = sub(P2, h.hitp);
    const float a_0 = magnitude(cross(sub(P0, P1), sub(P0, P2)));
    const float w1 = magnitude(cross(v1, v2)) / a_0;
    const float w2 = magnitude(cross(v2, v0)) / a_0;
    const float w3 = magnitude(cross(v0, v1)) / a_0;
    const float tu = (uv[0][0] * w1 + uv[1][0] * w2) + uv[2][0] * w3;
    const float tv = (uv[0][1] * w1 + uv[1][1] * w2) + uv[2][1] * w3;
    h.nrm = add(add(mul(n[0], w1), mul(n[1], w2)), mul(n[2], w3));
    const Mat& m = a.mats[mi];
    h.textured = m.tex_num != -1;
    float tx = 1.f, ty = 1.f, tz = 1.f, tw = 1.f;   // RayTraceRender.hlsl:19
    if (h.textured && (uint32_t)m.tex_num < a.ntex) {   // :22-26 (no texture bound: white)
        const float4 t = sample_texture(a, (uint32_t)m.tex_num, tu, tv);
        tx = t.x; ty = t.y; tz = t.z; tw = t.w;
    }
    h.color = make_float4(sat(m.ambient[0] + m.diffuse[0] * tx) * m.specular[0],
                          sat(m.ambient[1] + m.diffuse[1] * ty) * m.specular[1],
                          sat(m.ambient[2] + m.diffuse[2] * tz) * m.specular[2],
                          sat(m.ambient[3] + m.diffuse[3] * tw) * m.specular[3]);
    h.shininess = m.shininess;
    h.alpha = m.alpha;
    h.optical_density = m.optical_density;
    return h;
}

// the same for sorted leaf best_leaf (its record holds the triangle index)
__device__ __forceinline__ HitInfo shade_hit(const TraceArgs& a, uint32_t best_leaf, f3 o, f3 d, float t) {
    return shade_hit_tri(a, __float_as_uint(a.leaf[4 * (size_t)best_leaf + 2].y) & ~LEAF_BIT, o, d, t);
}

// A hit record written through to memory (agent scope, 8 B): the certified walk's early shading reads and claims
// records from other XCDs while the walk runs, and a record left dirty in the writer's L2 would be written back over
// the claim (trace.hip RTBVH_EARLY_SHADE)
__device__ __forceinline__ void st_hitrec(float2* p, float2 v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                       (unsigned long long)__float_as_uint(v.x) | (unsigned long long)__float_as_uint(v.y) << 32,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// the set lanes of mask below this lane (v_mbcnt: no 64-bit lane mask held in VGPRs)
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
// wave-aggregated append: one atomic per wave, lanes keep their order
__device__ __forceinline__ uint32_t wave_append(bool active, uint32_t* counter) {
    const uint64_t mask = __ballot(active);
    if (mask == 0) return 0;
    const uint32_t lane = lane_id();
    const int leader = __ffsll((unsigned long long)mask) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    return base + lane_rank(mask);
}

// counters: [base] internal visits, [base+1] leaf visits, [base+2] hits (base 2 primary,
// 5 bounce), [8] stack overflows / guard trips (also added to *overflow), [9] textured hits,
// [14] / [15] internal / leaf wave steps of the primary packet walks (one record fetch each),
// [16] / [17] bin entries of k_primary_binned and those it fetched a leaf record for
template <bool COUNT, bool BINS = false>
__device__ __forceinline__ void flush_counts(const TraceArgs& a, const Counts& c, uint32_t hits, uint32_t tex,
                                             int base) {
    unsigned long long v[7] = {c.internal, c.leaf, hits, c.overflow, tex, c.wint, c.wleaf};
#pragma unroll
    for (int k = 0; k < 7; k++)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
    if (lane_id() == 0) {
        if (COUNT) {
            atomicAdd(&a.counters[base], v[0]);
            atomicAdd(&a.counters[base + 1], v[1]);
            atomicAdd(&a.counters[base + 2], v[2]);
            atomicAdd(&a.counters[9], v[4]);
            if (v[5] | v[6]) {   // wave steps of the primary packet walks, or bin entries (k_primary_binned)
                atomicAdd(&a.counters[base == 2 && BINS ? 16 : 14], v[5]);
                atomicAdd(&a.counters[base == 2 && BINS ? 17 : 15], v[6]);
            }
        }
        if (v[3]) {
            atomicAdd(&a.counters[8], v[3]);
            atomicAdd(a.overflow, v[3]);
        }
    }
}

// RayTraceLaunch.hlsl:40-86 for one pixel of the frame, from its closest hit (phit: sorted leaf bl
// at distance best): colour, intensity, the RayPresent records, and the reflection ray in e
// (returns whether it is live, i.e. traced by RayTraceReflection.hlsl:17-18)
// REC false: a trace without RayPresent records (a.refl_rec, a.refr_rec null; the binned pass's shading then
// holds its registers at 8 waves per SIMD)
// qdst: where a live ray goes, when the caller knows it before the shading (the binned pass: no RayQ held
// across the shading)
template <bool REC = true>
__device__ __forceinline__ bool primary_pixel(const TraceArgs& a, size_t out, f3 o, f3 d, bool phit, float best,
                                              uint32_t bl, uint32_t& hits, uint32_t& tex, RayQ& e,
                                              RayQ* qdst = nullptr) {
    float4 color;
    float intensity = 0.f;
    bool live = false;
    if (phit) {
        hits = 1;
        const HitInfo h = shade_hit(a, bl, o, d, best);
        tex = h.textured;
        intensity = h.shininess / 1000.f * 1;   // :48 (REFLECTION_DECAY 1)
        color = h.color;
        if (0 < intensity) {   // traced by RayTraceReflection.hlsl:17-18 only when > INTENSITY_MIN
            const f3 ro = add(h.hitp, mul(h.nrm, .001f));   // RAY_OFFSET .001
            const f3 rd = normalize(reflect(d, h.nrm));
            e.idx = (uint32_t)out;
            e.intensity = intensity;
            e.ox = ro.x; e.oy = ro.y; e.oz = ro.z;
            e.dx = rd.x; e.dy = rd.y; e.dz = rd.z;
            live = true;
            if (qdst) *qdst = e;
        }
        if (REC && a.refl_rec) {   // :48-67 (the ray is set only when the intensity is not 0)
            const bool rr = intensity != 0;
            put_record(a.refl_rec, out, intensity, rr, rr ? add(h.hitp, mul(h.nrm, .001f)) : o,
                       rr ? normalize(reflect(d, h.nrm)) : d, color);
        }
        if (REC && a.refr_rec) {   // :70-80, REFRACTION_DECAY 1
            const float ri = (1.f - h.alpha) * 1;
            const bool rr = ri != 0;
            put_record(a.refr_rec, out, ri, rr, rr ? sub(h.hitp, mul(h.nrm, .001f)) : o,
                       rr ? normalize(refract_hlsl(d, h.nrm, h.optical_density)) : d,
                       make_float4(1.f, 1.f, 1.f, 1.f));
        }
    } else {
        color = make_float4(.5f, .5f, .5f, 1.f);   // getBackground, :85-86
        if (REC && a.refl_rec) put_record(a.refl_rec, out, 0.f, false, o, d, color);   // clearRayPresent
        if (REC && a.refr_rec) put_record(a.refr_rec, out, 0.f, false, o, d, color);
    }
    a.color[out] = color;
    if (a.intensity) a.intensity[out] = intensity;
    return live;
}

// RayTraceLaunch.hlsl:6-93.  LIM: a run-time stack limit (rtbvh_config.stack_limit); without
// it the limit is the compiled capacity, a constant (a run-time limit kept in the walk loop
// costs the SGPR-bound packet walks a kernel-argument reload per step)
template <bool COUNT, int K, bool LIM>
__global__ __launch_bounds__(BLOCK, 8) void k_primary(TraceArgs a, RayQ* __restrict__ q, uint32_t* __restrict__ qcount,
                                                      int emit) {
    using PW = PrimaryWalk<K>;
    const int lim = LIM ? a.stack_limit : STACK_SIZE, lim4 = LIM ? a.stack_limit4 : STACK4;
    constexpr int PST = PW::WIDE ? 3 * (STACK4 + 1) : 3 * STACK_SIZE;   // per-wave packet stack words (+ sentinel)
    __shared__ uint32_t s_pst[PW::PACKET ? 4 * PST : 1];
    __shared__ uint32_t s_lst[PW::PACKET || PW::NB || LANE_LSB == 0 ? 1 : LANE_LSB * BLOCK];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t x = blockIdx.x * 32 + w * 8 + (lane & 7);
    const uint32_t k = a.band0 + blockIdx.y * a.bstep;   // the rank's k-th band
    // behind k_primary_binned: trace only the blocks whose 32 x 32 screen tile overflowed its bins
    if (a.pb_gate && a.pb_gate[(((k * 8) >> 5) * a.pb_ntx + blockIdx.x + 1) * PB_NZ] <= a.pb_cap) return;
    const uint32_t band = a.band_list ? a.band_list[k] : k * a.nranks + a.rank;
    const uint32_t y = band * 8 + (lane >> 3);
    const bool valid = x < a.W && y < a.H;
    const size_t out = ((size_t)k * 8 + (lane >> 3)) * a.W + x;
    Counts c = {0, 0, 0, 0, 0};
    uint32_t hits = 0, tex = 0;
    bool live = false;
    RayQ e;
    const float hw = (float)(a.W >> 1), hh = (float)(a.H >> 1);
    const f3 o = mk(((float)x - hw) / 4.f, ((float)y - hh) / 4.f, 0.f);   // :23-24
    const f3 d = mk(0.f, 0.f, 1.f);
    const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    float best = 0.f;
    uint32_t bl = 0;
    bool phit = false;
    if (PW::WIDE)     // whole wave, before any divergence
        phit = traverse_packet4<COUNT, PW::GUARD, PW::GUARD || LIM>(a.inner, a.leaf, a.T, o, d, inv, valid, lim4, best, bl, c,
                                            s_pst + w * PST);
    else if (PW::PACKET)
        phit = traverse_packet<COUNT, PW::NEAREST>(a.inner, a.leaf, a.T, o, d, inv, valid, lim, best, bl, c,
                                                   s_pst + w * PST);
    if (valid) {
        const bool h = PW::PACKET ? phit
                       : PW::NB   ? traverse_nb<COUNT>(a.topo, a.nbox, a.leaf, a.T, o, d, inv, best, bl, c)
                                  : traverse<COUNT, PW::NEAREST, PW::PACKET ? 0 : LANE_LSB>(a.inner, a.leaf, a.T, o, d, inv, lim,
                                                                                           best, bl, c, s_lst + threadIdx.x);
        live = primary_pixel(a, out, o, d, h, best, bl, hits, tex, e);
    }
    const uint32_t slot = wave_append(emit && live, qcount);
    if (emit && live) q[slot] = e;
    flush_counts<COUNT>(a, c, hits, tex, 2);
}

// the trace's counters and bin counts zeroed by one launch instead of a memset each (blockIdx.y: the array)
__global__ __launch_bounds__(BLOCK) void k_zero(ZeroList z) {
    uint32_t* p = z.ptr[blockIdx.y];
    const size_t n = z.words[blockIdx.y];
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) p[i] = 0;
}

// ---- binned primary rays (RTBVH_FLAG_BINNED_PRIMARY) ----------------------------------------
// The primary rays are orthographic: pixel (x, y) is the ray o = ((x - W/2) / 4, (y - H/2) / 4, 0),
// d = (0, 0, 1) (RayTraceLaunch.hlsl:16-30).  The 4-wide packet walk (traverse_packet4) returns, per
// pixel, the lexicographic (t, leaf) minimum over the leaves whose box passes the axis-parallel test
// -- min.x < o.x < max.x, min.y < o.y < max.y (the general slab test for a box whose bit is set) --
// and whose triangle it hits; its box tests on the way down and its z pruning (min.z <= bound) only
// skip leaves that cannot beat the bound (containment).  On a regular pixel grid the
// pixels a box passes form a rectangle, which the build records exactly per leaf (rtbvh_device.h
// leaf_footprint).  So the same minimum is found level-synchronously at the leaves: every leaf is
// listed in the (32 x 32 screen tile, depth bucket) bins its rectangle covers (k_pb_bin, two passes
// streaming the leaves in slot order), then per tile (k_primary_binned) each listed leaf is tested
// against the pixels of its rectangle whose current bound its min.z does not exceed, nearest depth
// bucket first, the per-pixel (t, leaf) keys in LDS -- the bound carried from bucket to bucket.  Order
// only changes which tests the bound skips, never the minimum.  At C5: 13.7M (leaf, tile) entries,
// a third of them past the 8 x 8-block bound test, 35M triangle tests, all independent, in place of
// 17.9M dependent record fetches of 8x8-pixel packets.  k_pb_shade then writes k_primary's outputs
// (shading, RayPresent records, the bounce queue).  A tile whose bins overflowed the buffer is
// traced by k_primary (the per-lane nearest-first walk) behind these kernels (pb_gate).

#include "pb_bin.h"
// image row of the rank's compact row
__device__ __forceinline__ uint32_t pb_image_row(const TraceArgs& a, uint32_t crow) {
    const uint32_t k = crow >> 3;
    return (a.band_list ? a.band_list[k] : k * a.nranks + a.rank) * 8 + (crow & 7u);
}

template <bool FILL>
__global__ __launch_bounds__(BLOCK) void k_pb_bin(TraceArgs a, uint32_t* __restrict__ off,
                                                  uint32_t* __restrict__ cur, uint4* __restrict__ bins, uint32_t cap,
                                                  uint32_t ntx) {
    pb_bin_block<FILL>(a, blockIdx.x, off, cur, bins, cap, ntx);
}

// exclusive scan of the n bin counts in place, off[n] = the total, the fill cursors zeroed: blocks of
// PB_SCAN counts, first each block's total (k_pb_sums), then each block adds the totals of the blocks
// before it to its own scan (k_pb_scan; C5: 130,560 counts, 128 blocks)
constexpr uint32_t PB_SCAN = 1024;
__device__ __forceinline__ uint32_t block_sum_1024(uint32_t v, uint32_t* s_w) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0) s_w[w] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) t += s_w[k];
    return t;
}
__global__ __launch_bounds__(1024) void k_pb_sums(const uint32_t* __restrict__ off, uint32_t* __restrict__ sums,
                                                  uint32_t n) {
    __shared__ uint32_t s_w[16];
    const uint32_t i = blockIdx.x * PB_SCAN + threadIdx.x;
    const uint32_t t = block_sum_1024(i < n ? off[i] : 0u, s_w);
    if (threadIdx.x == 0) sums[blockIdx.x] = t;
}
__global__ __launch_bounds__(1024) void k_pb_scan(uint32_t* __restrict__ off, uint32_t* __restrict__ cur,
                                                  const uint32_t* __restrict__ sums, uint32_t n) {
    __shared__ uint32_t s_w[16], s_v[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    // the totals of the blocks before this one
    uint32_t p = 0;
    for (uint32_t k = tid; k < blockIdx.x; k += 1024) p += sums[k];
    const uint32_t before = block_sum_1024(p, s_v);
    const uint32_t i = blockIdx.x * PB_SCAN + tid;
    const uint32_t v = i < n ? off[i] : 0u;
    uint32_t x = v;   // inclusive scan over the wave, then over the waves
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if ((int)lane >= d) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t run = before + x - v;
    for (uint32_t k = 0; k < w; k++) run += s_w[k];
    if (i < n) { off[i] = run; cur[i] = 0; }
    if (i == n - 1) off[n] = run + v;
}

// one 32 x 32 tile of the rank's frame per workgroup: the (t, leaf) keys of its pixels in LDS and
// the largest bound of each 8 x 8 block.  The waves claim the tile's bins in batches of 64 entries
// (one per lane; nearest depth bucket first; the next batch's entries load while this one runs):
//  1. coarse: an entry whose min.z exceeds the largest bound of every block its rectangle touches
//     cannot win any of its pixels (C5: two thirds of the entries end here, before any leaf fetch);
//  2. the survivors' triangles (v0, e1, e2), one vector load per lane;
//  3. fine: per survivor, its rectangle's pixels as lanes; those whose bound min.z does not exceed go
//     to the wave's queue of (entry, pixel) tests;
//  4. the queue, 64 tests at a time (every lane a test: the triangle from its entry's lane by
//     ds_bpermute, the bound re-read), folded into the keys with an LDS atomic min;
//  then the block maxima are refreshed.  The keys go to `keys` (the frame's (t, leaf) per pixel);
//  k_pb_shade turns them into k_primary's outputs.
// A stale bound (another wave's newer key, a maximum refreshed later) only tests more, never less.
constexpr uint32_t PB_QCAP = 256;   // queued tests per wave
// a pixel's key slot: rows 40 keys (80 words, 16 banks) apart, so that the t words read by the lanes
// of an 8 x 8, 16 x 4 or 32 x 2 pixel block spread over the 32 odd banks two to a bank, the fewest
// (a 32-key row is 64 words: every row on the same banks, 8-way conflicts)
constexpr uint32_t PB_KS = 40;
__device__ __forceinline__ uint32_t pb_slot(uint32_t pi) { return (pi / PB_TILE) * PB_KS + (pi % PB_TILE); }
static_assert(PB_TILE == 32, "k_primary_binned: 10-bit pixel indices, 4 x 4 blocks of 8 x 8, a row per half-wave");
// RTBVH_PB_PROF builds: shader-clock cycles per phase of k_primary_binned, summed over the waves into
// counters[32..39] (read back as rtbvh_stats.trav_steps_log2[0..7]; scripts/pb_phases.py)
#ifdef RTBVH_PB_PROF
#define PB_T(i) do { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); const uint64_t _t = clock64(); pt[i] += _t - pt_last; pt_last = _t; } while (0)
#else
#define PB_T(i) do { } while (0)
#endif
#ifndef RTBVH_PB_RASTER_BLOCK
#define RTBVH_PB_RASTER_BLOCK 256
#endif
constexpr uint32_t PB_RASTER_BLOCK = RTBVH_PB_RASTER_BLOCK;   // threads per tile of k_primary_binned
constexpr uint32_t PB_RASTER_BLOCK_SMALL = 512;   // ... for a small pass one frame at a time (launch_pb_pass)
// cost probes (A/B builds only, wrong frames): 1 = no fine phase, 2 = the fine phase's tests skipped
#ifndef RTBVH_PB_PROBE
#define RTBVH_PB_PROBE 0
#endif
template <bool COUNT, bool CERT, uint32_t NT, bool REC, class KeyAt>
__device__ void pb_shade_tile(const TraceArgs& a, uint32_t rows, KeyAt&& key_at, RayQ* __restrict__ q,
                              uint32_t* __restrict__ qcount, int emit, uint32_t* __restrict__ redo,
                              uint32_t* __restrict__ redo_count, uint32_t* s_cnt, uint64_t* s_mask, uint32_t& s_base);
// FUSE (the default; RTBVH_PB_FUSE=0 builds the separate k_pb_shade launch, A/B): the tile's shading (k_pb_shade's work, pb_shade_tile) at the end of the
// same workgroup, from the keys in LDS -- no keys round trip through HBM, one launch fewer, and a tile's
// dependent shading gathers run beside other tiles' rasterisation on the CU
#ifndef RTBVH_PB_FUSE
#define RTBVH_PB_FUSE 1
#endif
#ifndef RTBVH_PB_WAVES
#define RTBVH_PB_WAVES 8   // k_primary_binned's launch bounds: 8 waves per SIMD with 37 VGPRs spilled beat
                                   // 6 (16 spilled) and 5 (none) -- primary pass 0.87-0.89 / 0.91-0.93 / 0.98 ms
#endif
// RB: threads per tile -- PB_RASTER_BLOCK, or PB_RASTER_BLOCK_SMALL for a small pass traced one frame at a time
// (api.hip: a rank's ~1,000 tiles then all run at once, and more waves per tile shorten the longest tile)
template <bool COUNT, bool CERT = false, bool FUSE = false, bool REC = true, uint32_t RB = PB_RASTER_BLOCK>
__global__ __launch_bounds__(RB, RTBVH_PB_WAVES) void k_primary_binned(TraceArgs a, const uint32_t* __restrict__ off,
                                                             const uint4* __restrict__ bins, uint32_t cap,
                                                             uint32_t ntx, uint32_t rows,
                                                             unsigned long long* __restrict__ keys, RayQ* __restrict__ q,
                                                             uint32_t* __restrict__ qcount, int emit,
                                                             uint32_t* __restrict__ redo,
                                                             uint32_t* __restrict__ redo_count) {
    __shared__ unsigned long long s_key[PB_TILE * PB_KS];
    __shared__ float s_bmax[(PB_TILE / 8) * (PB_TILE / 8)];
    __shared__ uint32_t s_q[RB / 64][PB_QCAP];
    __shared__ uint32_t s_next;
    const uint32_t* s_t = reinterpret_cast<const uint32_t*>(s_key);   // [2 slot + 1]: a pixel's bound (t bits)
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.y * ntx + blockIdx.x;
    const uint32_t X0 = blockIdx.x * PB_TILE, C0 = blockIdx.y * PB_TILE;
    const uint32_t beg = off[tile * PB_NZ], end = off[(tile + 1) * PB_NZ];
    if (end > cap) return;   // bins overflowed: k_primary traces this tile (pb_gate)
#ifdef RTBVH_PB_PROF
    uint64_t pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt_last = clock64();
#endif
    // keys of the pixels outside the frame (or the rank's rows) start at t = 0: no entry covers them,
    // and they never raise a block's largest bound
    for (uint32_t i = threadIdx.x; i < PB_TILE * PB_KS; i += RB)
        s_key[i] = X0 + i % PB_KS < a.W && C0 + i / PB_KS < rows ? NO_HIT : 0ull;
    if (threadIdx.x < (PB_TILE / 8) * (PB_TILE / 8)) s_bmax[threadIdx.x] = INFINITY;
    if (threadIdx.x == 0) s_next = 0;
    __syncthreads();
    const float hw = (float)(a.W >> 1), hh = (float)(a.H >> 1);
    const f3 d = mk(0.f, 0.f, 1.f);
    const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    uint32_t* sq = s_q[w];
    Counts c = {0, 0, 0, 0, 0};
    const uint32_t nbatch = (end - beg + 63) / 64;
    const auto claim = [&]() {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(&s_next, 1u);
        return (uint32_t)__builtin_amdgcn_readfirstlane(b);
    };
    const auto fetch = [&](uint32_t b) {
        const uint32_t e = beg + b * 64 + lane;
        return b < nbatch && e < end ? bins[e] : make_uint4(0, 0, 0, INVALID);
    };
    uint32_t bn = claim();
    uint4 fn = fetch(bn);
    PB_T(7);
    while (bn < nbatch) {
        const uint4 f = fn;
        bn = claim();
        fn = fetch(bn);   // the next batch's entries, in flight during this one
        const bool ve = f.w != INVALID;
        const uint32_t j = f.w & ~LEAF_BIT;
        const bool gen = ve && (f.w & LEAF_BIT) != 0;
        // the entry's rectangle in tile coordinates (it overlaps the tile by construction)
        const int rx0 = max((int)(f.x & 0xFFFFu), (int)X0) - (int)X0, rx1 = min((int)(f.x >> 16), (int)X0 + 31) - (int)X0;
        const int ry0 = max((int)(f.y & 0xFFFFu), (int)C0) - (int)C0, ry1 = min((int)(f.y >> 16), (int)C0 + 31) - (int)C0;
        const float zmin = __uint_as_float(f.z);
        PB_T(0);
        // 1: coarse
        bool surv = false;
        if (ve) {
            float m = -INFINITY;
            for (int by = ry0 >> 3; by <= ry1 >> 3; by++)
                for (int bx = rx0 >> 3; bx <= rx1 >> 3; bx++) m = fmaxf(m, s_bmax[by * (PB_TILE / 8) + bx]);
            surv = gen || zmin <= m;
        }
        if (COUNT) {
            const uint32_t nv = (uint32_t)__popcll(__ballot(ve)), ns = (uint32_t)__popcll(__ballot(surv));
            if (lane == 0) { c.wint += nv; c.wleaf += ns; }
        }
        // 2: the survivors' triangles
        float4 r0 = make_float4(0, 0, 0, 0), r1 = r0, r2 = r0;
        if (surv) {
            const float4* r = a.leaf + 4 * (size_t)j;
            r0 = r[0]; r1 = r[1]; r2 = r[2];
        }
        PB_T(1);
        // 4: the queued tests, every lane one (entry lane k, pixel pi)
        uint32_t qn = 0;
        const auto flush = [&]() {
            PB_T(3);
            for (uint32_t q0 = 0; q0 < (RTBVH_PB_PROBE == 2 ? 0u : qn); q0 += 64) {
                const bool act = q0 + lane < qn;
                const uint32_t v = act ? sq[q0 + lane] : 0u;
                const int k = (int)(v >> 10);
                const uint32_t pi = v & 1023u;
#define BP(x) __uint_as_float((uint32_t)__shfl((int)__float_as_uint(x), k, 64))
                const f3 p0 = mk(BP(r0.x), BP(r0.y), BP(r0.z)), e1 = mk(BP(r0.w), BP(r1.x), BP(r1.y));
                const f3 e2 = mk(BP(r1.z), BP(r1.w), BP(r2.x));
                const float kz = BP(zmin);
#undef BP
                const uint32_t kw = (uint32_t)__shfl((int)f.w, k, 64);
                const uint32_t kj = kw & ~LEAF_BIT;
                const bool kg = (kw & LEAF_BIT) != 0;
                const uint32_t px = pi % PB_TILE, py = pi / PB_TILE;
                const f3 o = mk(((float)(X0 + px) - hw) / 4.f, ((float)pb_image_row(a, C0 + (act ? py : 0u)) - hh) / 4.f,
                                0.f);
                bool in = false;
                if (act) {
                    if (kg) {   // the general slab test on the leaf's box, no pruning (traverse_packet4's leaf step)
                        const float4 b2 = a.leaf[4 * (size_t)kj + 2], b3 = a.leaf[4 * (size_t)kj + 3];
                        float tt;
                        in = ray_box_xy(o, inv, f2v{b2.z, b2.w}, f2v{b3.y, b3.z}, b3.x, b3.w, false, 0.f, tt);
                    } else {
                        in = kz <= __uint_as_float(s_t[2 * pb_slot(pi) + 1]);
                    }
                }
                if (COUNT) c.leaf += in;
                const float t = ray_triangle_flat(o, d, p0, e1, e2, in);
                if (t != -1.f) atomicMin(&s_key[pb_slot(pi)], (unsigned long long)__float_as_uint(t) << 32 | kj);
            }
            qn = 0;
            PB_T(4);
        };
        // 3: fine, survivor by survivor
        for (uint64_t todo = RTBVH_PB_PROBE == 1 ? 0ull : __ballot(surv); todo; todo &= todo - 1) {
            const int k = __ffsll((unsigned long long)todo) - 1;
            const bool sg = __builtin_amdgcn_readlane((int)gen, k) != 0;
            const int sx0 = __builtin_amdgcn_readlane(rx0, k), sx1 = __builtin_amdgcn_readlane(rx1, k);
            const int sy0 = __builtin_amdgcn_readlane(ry0, k), sy1 = __builtin_amdgcn_readlane(ry1, k);
            const float sz = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(zmin), k));
            const int lw = sx1 - sx0 + 1;
            const int cs = lw <= 8 ? 3 : lw <= 16 ? 4 : 5;   // lanes as 8x8, 16x4 or 32x2 pixels
            const int col = (int)(lane & ((1u << cs) - 1)), px = sx0 + col;
            for (int y0 = sy0; y0 <= sy1; y0 += 64 >> cs) {
                const int y = y0 + (int)(lane >> cs);
                const bool ok = col < lw && y <= sy1;
                const uint32_t pi = (uint32_t)(y * (int)PB_TILE + px);
                const bool need = ok && (sg || sz <= __uint_as_float(s_t[2 * pb_slot(pi) + 1]));
                const uint64_t nm = __ballot(need);
                if (qn + (uint32_t)__popcll(nm) > PB_QCAP) flush();
                if (need) sq[qn + lane_rank(nm)] = (uint32_t)k << 10 | pi;
                qn += (uint32_t)__popcll(nm);
            }
        }
        flush();
        PB_T(3);
        // the block maxima from the keys (pixels outside the frame hold t = 0): lane l reads column
        // l % 32 of rows l / 32, + 2, + 4, ... (two whole rows per read: 2-way bank conflicts at most),
        // one running maximum per block row, then the maxima of the 8 lanes of a block column and of
        // the two half-waves
        float m[PB_TILE / 8] = {0.f, 0.f, 0.f, 0.f};
        const uint32_t* bt = s_t + 2 * ((lane / 32) * PB_KS + lane % 32) + 1;
#pragma unroll
        for (uint32_t r = 0; r < PB_TILE / 2; r++) m[r / 4] = fmaxf(m[r / 4], __uint_as_float(bt[2 * (2 * r * PB_KS)]));
#pragma unroll
        for (uint32_t by = 0; by < PB_TILE / 8; by++) {
            m[by] = fmaxf(m[by], __shfl_xor(m[by], 1, 64));
            m[by] = fmaxf(m[by], __shfl_xor(m[by], 2, 64));
            m[by] = fmaxf(m[by], __shfl_xor(m[by], 4, 64));
            m[by] = fmaxf(m[by], __shfl_xor(m[by], 32, 64));
        }
        if (lane < PB_TILE && (lane & 7u) == 0) {
#pragma unroll
            for (uint32_t by = 0; by < PB_TILE / 8; by++) s_bmax[by * (PB_TILE / 8) + lane / 8] = m[by];
        }
        PB_T(5);
    }
    __syncthreads();
    if (FUSE) {
        __shared__ uint32_t s_cnt[(PB_TILE / 8) * (PB_TILE / 8)];
        __shared__ uint64_t s_mask[2 * (PB_TILE / 8) * (PB_TILE / 8)];
        __shared__ uint32_t s_base;
        pb_shade_tile<COUNT, CERT, RB, REC>(
            a, rows, [&](uint32_t crow, uint32_t x) { return s_key[(crow - C0) * PB_KS + (x - X0)]; }, q, qcount, emit,
            redo, redo_count, s_cnt, s_mask, s_base);
    } else {
        // the tile's keys, row segments of 32 pixels
        for (uint32_t i = threadIdx.x; i < PB_TILE * PB_TILE; i += RB) {
            const uint32_t px = i % PB_TILE, py = i / PB_TILE;
            if (X0 + px < a.W && C0 + py < rows) keys[(size_t)(C0 + py) * a.W + X0 + px] = s_key[py * PB_KS + px];
        }
    }
#ifdef RTBVH_PB_PROF
    PB_T(6);
    if (lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&a.counters[32 + i], (unsigned long long)pt[i]);
#endif
    flush_counts<COUNT, true>(a, c, 0, 0, 2);
}

// k_primary's outputs from the binned pass's keys, one 32 x 32 tile per block (a wave takes its
// 8 x 8 sub-tiles w, w + 4, ...).  The reflection rays go to the bounce queue with ONE atomic per
// block: its live rays are counted first (hit and shininess > 0, RayTraceLaunch.hlsl:48 and
// RayTraceReflection.hlsl:17-18), the block's base claimed, then every pixel shaded and its ray
// written at base + its rank.  (One atomic per wave -- k_primary's wave_append -- is 130K claims on
// one counter per C5 frame, ~1.2 ms at the ~100 claims per us one address takes.)  Tiles whose bins
// overflowed return (k_primary traced them).
// (a 1024-thread block, one pixel per thread: 256 threads with four pixels each held 86 VGPRs,
// 5 waves per SIMD, for the shading's dependent gathers)
#ifndef RTBVH_PB_SHADE_BLOCK
#define RTBVH_PB_SHADE_BLOCK 1024
#endif
constexpr uint32_t PB_SHADE_BLOCK = RTBVH_PB_SHADE_BLOCK;
// CERT (the certified pass): the binned pass tested every leaf whose triangle could be
// accepted below a pixel's bound (its depth key, margin.h); a pixel's (t, leaf) is the reference's when
// the leaf's own box passes the reference slab test with the bound t (k_bounce_shade's leaf_certified,
// here from the leaf record's box).  Pixels that fail it go to the re-trace list (redo: compact pixel
// index) and are left to k_primary_redo, outside the block's bounce-queue claim.
// One tile of k_pb_shade's work over NT threads, the pixels' keys from key_at(compact row, x).  s_cnt: 16
// words of LDS, s_mask: 2 x 16 words, s_base: one.  The 16 sub-tiles of 8 x 8 pixels go to the waves in
// turn; a first pass counts each one's live rays (and certificates) into LDS, the tile claims its queue
// range, then a second pass shades them (no per-sub-tile registers held across the claim).
// (Inlined: out of line, A/B round 5, the fused binned pass took 1.07 ms against 0.86.)
// The kernel's TraceArgs (its first argument) read again from the kernel-argument segment where they are used:
// scalar loads the compiler cannot hoist out of a loop (held in SGPRs across the shading loop's iterations they
// spilled into VGPR lanes, and the shading's VGPRs to scratch)
__device__ __forceinline__ const TraceArgs& kernel_trace_args() {
    auto p = (const __attribute__((address_space(4))) TraceArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const TraceArgs*)p;
}
template <bool COUNT, bool CERT, uint32_t NT, bool REC, class KeyAt>
__device__ __forceinline__ void pb_shade_tile(const TraceArgs& a, uint32_t rows, KeyAt&& key_at, RayQ* __restrict__ q,
                                              uint32_t* __restrict__ qcount, int emit, uint32_t* __restrict__ redo,
                                              uint32_t* __restrict__ redo_count, uint32_t* s_cnt, uint64_t* s_mask,
                                              uint32_t& s_base) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t X0 = blockIdx.x * PB_TILE, C0 = blockIdx.y * PB_TILE;
    constexpr uint32_t NST = (PB_TILE / 8) * (PB_TILE / 8) / (NT / 64);   // sub-tiles per wave
    constexpr uint32_t NSUB = (PB_TILE / 8) * (PB_TILE / 8);
    const float hw = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint((float)(a.W >> 1))));
    const float hh = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint((float)(a.H >> 1))));
    const auto pixel = [&](uint32_t i, uint32_t& x, uint32_t& crow) {
        const uint32_t st = w + i * (NT / 64);
        x = X0 + (st % (PB_TILE / 8)) * 8 + (lane & 7u);
        crow = C0 + (st / (PB_TILE / 8)) * 8 + (lane >> 3);
        return x < a.W && crow < rows;
    };
    // the live reflection rays: hit, and the hit material's shininess > 0
#pragma unroll 1
    for (uint32_t i = 0; i < NST; i++) {
        uint32_t x, crow;
        const bool valid = pixel(i, x, crow);
        const uint64_t key = valid ? key_at(crow, x) : NO_HIT;
        bool live = false, flag = false;
        if (CERT && key != NO_HIT) {   // the certificate: the leaf's box, the reference slab test at t
            const float4 b2 = a.leaf[4 * (size_t)(uint32_t)key + 2], b3 = a.leaf[4 * (size_t)(uint32_t)key + 3];
            const f3 o = mk(((float)x - hw) / 4.f, ((float)pb_image_row(a, crow) - hh) / 4.f, 0.f);
            const f3 d = mk(0.f, 0.f, 1.f);
            float tm;
            flag = !ray_box(o, mk(1.f / d.x, 1.f / d.y, 1.f / d.z), b2.z, b2.w, b3.x, b3.y, b3.z, b3.w, true,
                            key_t(key), tm);
        }
        if (emit && key != NO_HIT && !flag) {
            const uint32_t tri = __float_as_uint(a.leaf[4 * (size_t)(uint32_t)key + 2].y) & ~LEAF_BIT;
            const uint32_t mi = TCS == 4 ? __float_as_uint(a.tclip[TCS * (size_t)tri + 3].w) : a.matidx[tri];
            live = 0 < a.mats[mi].shininess / 1000.f * 1;
        }
        const uint64_t livem = __ballot(live), flagm = CERT ? __ballot(flag) : 0ull;
        const uint32_t st = w + i * (NT / 64);
        if (lane == 0) {
            s_cnt[st] = (uint32_t)__popcll(livem);
            s_mask[st] = livem;
            s_mask[NSUB + st] = flagm;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t k = 0; k < NSUB; k++) {
            const uint32_t v = s_cnt[k];
            s_cnt[k] = run;
            run += v;
        }
        s_base = run && emit ? atomicAdd(qcount, run) : 0u;
    }
    __syncthreads();
    const uint32_t sbase = (uint32_t)__builtin_amdgcn_readfirstlane(s_base);
    uint32_t hits = 0, tex = 0;
#pragma unroll 1
    for (uint32_t i = 0; i < NST; i++) {
        uint32_t x, crow;
        const bool valid = pixel(i, x, crow);
        const uint32_t st = w + i * (NT / 64);
        // (wave-uniform: into SGPRs, so the shading below keeps its VGPRs)
        const auto uni64 = [](uint64_t v) {
            return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32;
        };
        const uint64_t livem = uni64(s_mask[st]), flagm = CERT ? uni64(s_mask[NSUB + st]) : 0ull;
        const uint32_t qb = sbase + (uint32_t)__builtin_amdgcn_readfirstlane(s_cnt[st]);
        const bool flag = CERT && ((flagm >> lane) & 1u);
        if (CERT && flagm) {   // (rare) the re-trace list, one atomic per wave
            const uint32_t slot = wave_append(flag, redo_count);
            if (flag) redo[slot] = crow * a.W + x;
        }
        if (valid && !flag) {
            const TraceArgs& a = kernel_trace_args();   // (a is the kernel's first argument: k_primary_binned, k_pb_shade)
            const uint64_t key = key_at(crow, x);
            const f3 o = mk(((float)x - hw) / 4.f, ((float)pb_image_row(a, crow) - hh) / 4.f, 0.f);
            const bool phit = key != NO_HIT;
            uint32_t h1 = 0, t1 = 0;
            RayQ e;
            // (the live rays were counted above: this lane's queue entry is known before the shading)
            RayQ* dst = emit && ((livem >> lane) & 1u) ? q + qb + lane_rank(livem)
                                                        : nullptr;
            (void)primary_pixel<REC>(a, (size_t)crow * a.W + x, o, mk(0.f, 0.f, 1.f), phit, phit ? key_t(key) : 0.f,
                                     phit ? (uint32_t)key : 0u, h1, t1, e, dst);
            hits += h1;
            tex += t1;
        }
    }
    if (COUNT) {
        Counts c = {0, 0, 0, 0, 0};
        flush_counts<COUNT>(a, c, hits, tex, 2);
    }
}
template <bool COUNT, bool CERT>
__global__ __launch_bounds__(PB_SHADE_BLOCK, 8) void k_pb_shade(TraceArgs a, const uint32_t* __restrict__ off, uint32_t cap,
                                                    uint32_t ntx, uint32_t rows,
                                                    const unsigned long long* __restrict__ keys, RayQ* __restrict__ q,
                                                    uint32_t* __restrict__ qcount, int emit,
                                                    uint32_t* __restrict__ redo, uint32_t* __restrict__ redo_count) {
    __shared__ uint32_t s_cnt[(PB_TILE / 8) * (PB_TILE / 8)];
    __shared__ uint64_t s_mask[2 * (PB_TILE / 8) * (PB_TILE / 8)];
    __shared__ uint32_t s_base;
    const uint32_t tile = blockIdx.y * ntx + blockIdx.x;
    if (off[(tile + 1) * PB_NZ] > cap) return;
    pb_shade_tile<COUNT, CERT, PB_SHADE_BLOCK, true>(
        a, rows, [&](uint32_t crow, uint32_t x) { return keys[(size_t)crow * a.W + x]; }, q, qcount, emit, redo,
        redo_count, s_cnt, s_mask, s_base);
}

// The reference-order re-trace of the pixels a certified primary pass flagged (redo: compact pixel
// indices crow * W + x): the exact findCollision DFS per pixel (traverse), then k_primary's outputs
// (primary_pixel) and the bounce queue.  A fixed grid over the count on the device.
template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void k_primary_redo(TraceArgs a, const uint32_t* __restrict__ redo,
                                                        const uint32_t* __restrict__ redo_count, RayQ* __restrict__ q,
                                                        uint32_t* __restrict__ qcount, int emit) {
    const uint32_t n = *redo_count;
    Counts c = {0, 0, 0, 0, 0};
    uint32_t hits = 0, tex = 0;
    const float hw = (float)(a.W >> 1), hh = (float)(a.H >> 1);
    const f3 d = mk(0.f, 0.f, 1.f);
    const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    for (uint32_t base = blockIdx.x * BLOCK; base < n; base += gridDim.x * BLOCK) {
        const uint32_t i = base + threadIdx.x;
        bool live = false;
        RayQ e;
        if (i < n) {
            const uint32_t p = redo[i], crow = p / a.W, x = p % a.W;
            const f3 o = mk(((float)x - hw) / 4.f, ((float)pb_image_row(a, crow) - hh) / 4.f, 0.f);
            float best;
            uint32_t bl, h1 = 0, t1 = 0;
            const bool h = traverse_ref<COUNT>(a, o, d, inv, best, bl, c);
            live = primary_pixel(a, p, o, d, h, best, bl, h1, t1, e);
            hits += h1;
            tex += t1;
        }
        const uint32_t slot = wave_append(emit && live, qcount);
        if (emit && live) q[slot] = e;
    }
    flush_counts<COUNT>(a, c, hits, tex, 2);
}

// RayTraceReflection.hlsl:6-62 over the compacted queue of live rays (in `perm`
// order when the queue was sorted for coherence), one ray per lane
template <bool COUNT, bool NEAREST, bool LIM>
__global__ __launch_bounds__(BLOCK, 8) void k_bounce(TraceArgs a, const RayQ* __restrict__ qin,
                                                     const uint32_t* __restrict__ qin_count,
                                                     const uint32_t* __restrict__ perm, RayQ* __restrict__ qout,
                                                     uint32_t* __restrict__ qout_count, int emit) {
    __shared__ uint32_t s_lst[LANE_LSB == 0 ? 1 : LANE_LSB * BLOCK];
    const uint32_t n = *qin_count;
    Counts c = {0, 0, 0, 0, 0};
    uint32_t hits = 0, tex = 0;
    for (uint32_t base = blockIdx.x * BLOCK; base < n; base += gridDim.x * BLOCK) {
        const uint32_t i = base + threadIdx.x;
        bool live = false;
        RayQ e;
        if (i < n) {
            e = qin[perm ? perm[i] : i];
            const f3 o = mk(e.ox, e.oy, e.oz), d = mk(e.dx, e.dy, e.dz);
            const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
            float best;
            uint32_t bl;
            float4 col = a.color[e.idx];
            float intensity = e.intensity;
#ifdef RTBVH_BOUNCE_PROBE   // cost probes (A/B builds, wrong frames): 1 no walk (every ray misses), 2 no shading
            const bool th = RTBVH_BOUNCE_PROBE == 1 ? false
                                                    : traverse<COUNT, NEAREST, LANE_LSB>(a.inner, a.leaf, a.T, o, d, inv,
                                                          LIM ? a.stack_limit : STACK_SIZE, best, bl, c, s_lst + threadIdx.x);
            if (RTBVH_BOUNCE_PROBE == 2 && th) {
                hits++;
                col = make_float4(best, (float)bl, 0.f, 1.f);
            } else if (th) {
#else
            if (traverse<COUNT, NEAREST, LANE_LSB>(a.inner, a.leaf, a.T, o, d, inv, LIM ? a.stack_limit : STACK_SIZE,
                                                   best, bl, c, s_lst + threadIdx.x)) {
#endif
                hits++;
                const HitInfo h = shade_hit(a, bl, o, d, best);
                tex += h.textured;
                col = make_float4(lerpf(col.x, h.color.x, intensity), lerpf(col.y, h.color.y, intensity),
                                  lerpf(col.z, h.color.z, intensity), lerpf(col.w, h.color.w, intensity));
                intensity *= h.shininess / 1000.f * 1;
                const f3 ro = add(h.hitp, mul(h.nrm, .0001f));   // RAY_OFFSET .0001
                const f3 rd = normalize(reflect(d, h.nrm));
                e.intensity = intensity;
                e.ox = ro.x; e.oy = ro.y; e.oz = ro.z;
                e.dx = rd.x; e.dy = rd.y; e.dz = rd.z;
                live = 0 < intensity;
            } else {
                col = make_float4(lerpf(col.x, .5f, intensity), lerpf(col.y, .5f, intensity),
                                  lerpf(col.z, .5f, intensity), lerpf(col.w, 1.f, intensity));
                intensity = 0.f;
            }
            a.color[e.idx] = col;
            if (a.intensity) a.intensity[e.idx] = intensity;
        }
        const uint32_t slot = wave_append(emit && live, qout_count);
        if (emit && live) qout[slot] = e;
    }
    flush_counts<COUNT>(a, c, hits, tex, 5);
}

// ---- bounce pass split in two: persistent traversal with lane refill + shading ----
// The one-ray-per-lane bounce kernel keeps a wave until its slowest ray is done:
// PMC on C5 showed ~12 of 64 lanes active per traversal step (1.6e8 wave loads for
// 4.7e8 lane visits).  Here each lane that finishes its ray takes the next one from
// the queue (one atomic per wave per refill, Aila & Laine's dynamic fetch), so the
// wave stays full; the finished ray's (t, leaf) goes to a hit record, and the
// shading runs afterwards as a plain one-thread-per-ray kernel (k_bounce_shade).
// Per-lane traversal state and visit order are exactly those of traverse().
// A wave refills when at least REFILL_MIN lanes are idle.  A/B on C5 (bounce pass):
// 4 -> 15.6 ms, 8 -> 9.2, 16 -> 5.5, 24 -> 4.13, 32 -> 3.87, 40 -> 3.84, 48 -> 3.90,
// 64 -> 5.36 (the single work counter's atomic contention below 32).  Round 2's walk, bounce stage
// with shading: 8 -> 2.67 ms, 16 -> 2.57, 24 -> 2.59, 32 -> 2.62.
// Work counters: the queue is cut into NEXT_SEGS contiguous segments, each with its own
// counter on its own 128-B line.  Workgroup b runs on XCD b % 8 (round-robin dispatch); its
// waves claim from the segments of their XCD first (starting at one picked by b / 8), then from
// the other XCDs' in turn.  A single counter serialised the claims of all 8192 waves (~88 per
// us), which is what kept REFILL_MIN from going lower; and an XCD's waves now walk rays of
// neighbouring queue positions (neighbouring pixels), whose upper-tree nodes its L2 shares.
#ifndef RTBVH_REFILL_MIN
#define RTBVH_REFILL_MIN 16
#endif
constexpr uint32_t REFILL_MIN = RTBVH_REFILL_MIN;
constexpr uint32_t XCDS = 8;
constexpr uint32_t SEGS_PER_XCD = NEXT_SEGS >= XCDS ? NEXT_SEGS / XCDS : 1;
__device__ __forceinline__ uint32_t claim_segment(uint32_t k) {   // the wave's k-th segment
    if (NEXT_SEGS < XCDS) return k;
    const uint32_t xcd = blockIdx.x % XCDS, sub = (blockIdx.x / XCDS) % SEGS_PER_XCD;
    const uint32_t g = (xcd + k / SEGS_PER_XCD) % XCDS;
    return g * SEGS_PER_XCD + (sub + k) % SEGS_PER_XCD;
}

__device__ __forceinline__ void sort2(float& ta, uint32_t& ia, float& tb, uint32_t& ib) {
    const bool sw = tb < ta;
    const float t = sw ? tb : ta;
    const uint32_t i = sw ? ib : ia;
    tb = sw ? ta : tb;
    ib = sw ? ia : ib;
    ta = t;
    ia = i;
}

// A 16-bit key for an entry distance t that never exceeds it: the upper half of max(t, 0)
// (fmaxf drops NaN).  Positive t is truncated (rounded down); t <= 0 becomes 0, which is below
// every best distance (a hit's t > EPSILON), as t is: an entry is dropped on pop only when the
// exact test would drop it too.  One v_max_f32; the store takes the high half (the first
// form rounded negative t away from zero: six VALU and two SALU per push).
__device__ __forceinline__ uint16_t bf16_down(float t) { return (uint16_t)(__float_as_uint(fmaxf(t, 0.f)) >> 16); }
__device__ __forceinline__ float bf16_up(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// Walk modes of k_bounce_trav: 0 reference order, 1 nearest-first (binary records), 2 the
// 4-wide nearest-first walk on the quantized nodes (qn, rtbvh_device.h QNode: one 64-B node
// per 4-wide step; a node without a finite grid falls back to its exact record pair).
// Binary modes keep the stack entries [0, SB) in LDS, [entry][lane] (a wave's lanes hit
// 64 distinct banks whatever their depths), and only deeper entries in scratch: the
// all-scratch stack of 8192 resident waves (17 KB each) does not fit in L2 and PMC
// showed ~3.6 GB of stack write-back per C5 bounce pass.  The 4-wide walk keeps
// (node, entry distance) entries [0, SW) in LDS as a node id and the distance as a bf16
// rounded toward -inf (6 B each; the pop's prune test on the rounded-down distance keeps
// every entry the exact test keeps), deeper entries as full pairs in scratch.
constexpr int SB = 16;   // 16 x 4 B x 256 lanes = 16 KB per block
// 13 x 6 B x 256 lanes = 19.5 KB per block: 8 blocks per CU in 160 KB.  A/B (C5 bounce stage):
// 8 entries 2.75-2.77 ms (deeper entries go to scratch), 12 2.50-2.55, 13 2.47-2.52, 14 2.51-2.53
// (7 blocks per CU)
#ifndef RTBVH_SW
#define RTBVH_SW 13
#endif
constexpr int SW = RTBVH_SW;
static_assert(SW * 6 * 256 * 8 <= 160 * 1024, "the 4-wide bounce walk's LDS stack: 8 blocks per CU");

// ---- the slack test of a quantized node --------------------------------------------------
// The exact form (RTBVH_QBOX below) decodes each corner, org + q * scl, and runs the reference
// slab test on it: 6 decodes + 12 slab operations per box.  Here the slab is evaluated in the
// node's grid, t(q) = q * b + a with b = scl * inv (exact: a power of two times inv) and
// a = (org - o) * inv, shared by the node's four boxes; and the ray's sign picks each axis's
// near and far corner word once per node, so a box costs 6 cvt + 6 fma + max3 + min3.
// Conservative against the reference test on the EXACT box: for every corner x the box
// contains and its decoded corner D (D <= x on the near side), the reference's
// RN(RN(x - o) * inv) and t(q) both lie within 8u * M * |inv| of (org + q scl - o) * inv
// (u = 2^-24, M = |org| + |o| + 256 scl: the roundings of the decode, the subtraction, the
// products and the fma), so the near distances are taken E = 2^-20 * M * |inv| (16u) low and
// the far ones E high.  Every box the exact test hits is hit, at an entry distance <= the
// exact one: the walk reaches every leaf the exact walk reaches and prunes only what it would.
// Finite for |o| <= 2^90, |inv| <= 2^20 (qnode_fast_ray) and corners within 2^100 (a QNode
// with larger ones keeps the exact record pair, build.hip quantize_axis); other rays take the
// exact decode.
__device__ __forceinline__ bool qnode_fast_ray(f3 o, f3 inv) {
    const float mi = fmaxf(fmaxf(fabsf(inv.x), fabsf(inv.y)), fabsf(inv.z));
    const float mo = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    return mi <= 0x1p20f && mo <= 0x1p90f;   // NaN: false
}
struct QAxis { uint32_t nw, fw; float b, an, af; };
// CERT (the certified walk): the near side is widened by the margin rr as well, in
// position (rr * |inv| in distance): the entry of the box grown by rr on every side (margin.h).
template <bool CERT = false>
__device__ __forceinline__ QAxis qaxis(float org, float scl, uint32_t lw, uint32_t hw, float o, float inv,
                                       float rr = 0.f) {
    QAxis r;
    const bool neg = inv < 0.f;
    r.nw = neg ? hw : lw;
    r.fw = neg ? lw : hw;
    const float m = fmaf(scl, 256.f, fabsf(org) + fabsf(o));
    const float e = m * fabsf(inv);
    const float a = (org - o) * inv;
    if (CERT) r.an = fmaf(-fmaf(m, 0x1p-20f, rr), fabsf(inv), a);
    else r.an = fmaf(e, -0x1p-20f, a);
    r.af = fmaf(e, 0x1p-20f, a);
    r.b = scl * inv;
    return r;
}
__device__ __forceinline__ float qt(uint32_t w, int c, float b, float a) {
    return fmaf((float)((w >> (8 * c)) & 255u), b, a);
}
__device__ __forceinline__ bool qbox_fast(const QAxis& x, const QAxis& y, const QAxis& z, int c, bool hit, float best,
                                          float& tmin) {
    const float mn = fmaxf(fmaxf(qt(x.nw, c, x.b, x.an), qt(y.nw, c, y.b, y.an)), qt(z.nw, c, z.b, z.an));
    const float mx = fminf(fminf(qt(x.fw, c, x.b, x.af), qt(y.fw, c, y.b, y.af)), qt(z.fw, c, z.b, z.af));
    tmin = mn;
    return 0 <= mx && mn <= mx && (!hit || mn <= best);
}

// The certified walk's box test: qbox_fast, and the box's stack key, capped at its node's margin range tcn
// (margin.h: past it the node's margin says nothing, so the box is never pruned by distance -- kept while
// min(key, tcn) <= best, the pop's test too).  After the first bound the key is the entry of the box grown
// by the node's margin rho_n(best) (rr, qaxis<true>).  Before it (best +inf: nothing pruned, rr = 0) it is
// the entry of the box grown by rho_n(t_e), t_e its margin-free entry: pops compare a key with later,
// finite bounds kb, and for kb <= t_e, rho_n(kb) <= rho_n(t_e), so the key is at most the entry of the box
// grown by rho_n(kb) -- a box the certified walk must visit (that entry <= kb) keeps key <= kb; for
// kb > t_e the key (<= t_e) is kept anyway, the margin-free entry being below the bound.  The grown entry
// is the max over axes of near - rho |1/d| (branch-free: rho = 0 after the first bound).
__device__ __forceinline__ bool qbox_fast_cert(const QAxis& x, const QAxis& y, const QAxis& z, int c, float best,
                                               const MtNodeK& nk, const MtNodeRho& nr, f3 ainv, float tcn,
                                               float& key) {
    const float nx = qt(x.nw, c, x.b, x.an), ny = qt(y.nw, c, y.b, y.an), nz = qt(z.nw, c, z.b, z.an);
    const float mn = fmaxf(fmaxf(nx, ny), nz);
    const float mx = fminf(fminf(qt(x.fw, c, x.b, x.af), qt(y.fw, c, y.b, y.af)), qt(z.fw, c, z.b, z.af));
    const float rb = best == __builtin_inff() ? mt_node_eval(nr, fmaxf(mn, 0.f)) : 0.f;
    // (the looser bound mn - rho max|1/d|, 2 VALU instead of 5, A/B round 5: 5.9 ms against 2.5 -- the walk
    // keeps far more entries before its first bound)
    key = fminf(fmaxf(fmaxf(fmaf(-rb, ainv.x, nx), fmaf(-rb, ainv.y, ny)), fmaf(-rb, ainv.z, nz)), tcn);
    return 0 <= mx && mn <= mx && key <= best;
}
// GUARD false: no walk-length guard (a clz64 tree has no cycles; the census of COUNT keeps it).
// CERT (MODE 2 only): the certified walk.  Every box test's entry distance is taken on the
// box grown by its node's margin rho_n(best) (margin.h: no hit the triangle test accepts at t <= best lies
// outside that box; rho_n from the largest edge bound of the leaves below the node, carried by its QNode),
// and a box is not pruned by distance at all while best is past its node's margin range: so the walk sees
// EVERY leaf whose triangle could be accepted at t <= best, and its (t, leaf) minimum is the minimum over
// all triangles the reference could test.  A ray the bound does not cover -- a slack-test-free ray
// (qnode_fast_ray), |d| off unit, a node without a grid, a stack overflow -- is flagged in its hit record
// (HIT_FLAG) for the reference-order re-trace (k_bounce_redo).
// The deferred rays of a certified bounce pass (the rays its margin does not cover: |1/d| > 2^20, |o| > 2^90,
// |d| off unit).  The walk lists them at claim time in the pass's defer list -- entry k at defer[k] with
// DEFER_VALID set, k from the counter next[DEFER_COUNT] -- and writes a "deferred" hit record (t = -inf, flagged:
// k_bounce_shade skips it).  Drained waves claim entries through next[DEFER_CLAIM] and walk them in the
// reference order; k_bounce_redo takes the rest.  Readers clear the entries they take.
#ifndef RTBVH_DEFER_INWALK
#define RTBVH_DEFER_INWALK 1   // (0, A/B: every deferred ray to k_bounce_redo)
#endif
// a deferred ray's reference-order walk: its hit record, "exact" (t negated; a miss -inf with id INVALID)
template <bool COUNT>
__device__ __forceinline__ float2 defer_walk(const Inner* __restrict__ inner, const uint4* __restrict__ topo,
                                             const float* __restrict__ nbox, const float4* __restrict__ leaf,
                                             uint32_t T, const RayQ* e, Counts& c) {
    const float4 q0 = reinterpret_cast<const float4*>(e)[0], q1 = reinterpret_cast<const float4*>(e)[1];
    const f3 o = mk(q0.z, q0.w, q1.x), d = mk(q1.y, q1.z, q1.w);
    const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    float best;
    uint32_t bl;
    const bool h = nbox ? traverse_nb<COUNT>(topo, nbox, leaf, T, o, d, inv, best, bl, c)
                        : traverse<COUNT, false>(inner, leaf, T, o, d, inv, STACK_SIZE, best, bl, c);
    const uint32_t tri = h ? __float_as_uint(leaf[4 * (size_t)bl + 2].y) & ~LEAF_BIT : INVALID;
    return make_float2(h ? -best : -__builtin_inff(), __uint_as_float(tri));
}

// One wave takes deferred rays -- up to 64 at a time, lane k the k-th -- and walks each in the reference order,
// until the list holds none it has not taken
template <bool COUNT>
__device__ __forceinline__ void defer_walk_all(uint32_t* __restrict__ next, uint32_t* __restrict__ defer,
                                               const Inner* __restrict__ inner, const uint4* __restrict__ topo,
                                               const float* __restrict__ nbox, const float4* __restrict__ leaf,
                                               uint32_t T, const RayQ* __restrict__ qin, float2* __restrict__ hitrec,
                                               Counts& c, bool wt) {
    const uint32_t lane = threadIdx.x & 63u;
    for (;;) {
        uint32_t base = 0, m = 0;
        if (lane == 0) {
            uint32_t v = __hip_atomic_load(next + DEFER_CLAIM, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (;;) {
                const uint32_t nd = __hip_atomic_load(next + DEFER_COUNT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v >= nd) break;
                const uint32_t want = min(nd - v, 64u);
                if (__hip_atomic_compare_exchange_strong(next + DEFER_CLAIM, &v, v + want, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    base = v;
                    m = want;
                    break;
                }
            }
        }
        base = __builtin_amdgcn_readfirstlane(base);
        m = __builtin_amdgcn_readfirstlane(m);
        if (m == 0) return;
        if (lane < m) {
            // (the appending lane stores its entry right after its count add: wait for it)
            uint32_t e;
            do {
                e = __hip_atomic_load(defer + base + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            } while (!(e & DEFER_VALID));
            defer[base + lane] = 0u;   // (the list is clean for the next pass)
            const float2 hv = defer_walk<COUNT>(inner, topo, nbox, leaf, T, qin + (e & ~DEFER_VALID), c);
            if (wt) st_hitrec(hitrec + (e & ~DEFER_VALID), hv);
            else hitrec[e & ~DEFER_VALID] = hv;
        }
    }
}
// the deferral workers: wave 0 of the first DEFER_WORKERS workgroups (one per XCD) walks the deferred rays as they
// come, from the start of the pass -- beside the walk, not after it -- and leaves once every queue segment is
// claimed and the list is empty (a ray deferred after that goes to the drained waves or k_bounce_redo)
#ifndef RTBVH_DEFER_WORKERS
#define RTBVH_DEFER_WORKERS 8
#endif
constexpr uint32_t DEFER_WORKERS = RTBVH_DEFER_WORKERS;

// Early shading (RTBVH_EARLY_SHADE, certified passes): the walk's launch carries shading workgroups after its
// persistent ones.  They are dispatched as the walk's workgroups retire -- in the walk's tail -- and each takes 1024
// queue positions in order: a ray whose hit record is final (the pass's records start "not written yet", k_hit_init)
// is claimed by a compare-and-swap to "shaded" and shaded there (bounce_shade_ray, k_bounce_shade's work); the
// pass's k_bounce_shade shades the rest.  So the shading of most rays runs beside the walk's last rays.
#ifndef RTBVH_EARLY_SHADE
#define RTBVH_EARLY_SHADE 1
#endif
#ifndef RTBVH_ESHADE_RAYS
#define RTBVH_ESHADE_RAYS 1024
#endif
constexpr uint32_t ESHADE_RAYS = RTBVH_ESHADE_RAYS;   // queue positions per shading workgroup
// hit-record words of a certified pass with early shading (RTBVH_EARLY_SHADE): not written yet, and shaded already
constexpr uint32_t HIT_NOT_READY = 0xFFFFFFFFu, HIT_SHADED = 0xFFFFFFFEu;   // (x words: NaN patterns no walk writes)
template <bool CERT>
__device__ __forceinline__ void bounce_shade_ray(const TraceArgs& a, const RayQ* __restrict__ qin, uint32_t i, float2 h2,
                                                 bool valid, RayQ& e, bool& live, bool& flagged, uint32_t& hits,
                                                 uint32_t& tex);
// ES: the instance with early shading (a frame traced one at a time); the walk without it (frames in flight) is its
// own instance without the shading role's code.  The role's shading spills 13 VGPRs in its own blocks (the walk's
// loop has none: its scratch accesses are the deep stack's, as in the plain instance); as an out-of-line call it
// made the one-frame walk 2.70 -> 3.16 ms (r06_hab3)
template <bool COUNT, int MODE, bool LIM, bool GUARD, bool CERT = false, bool ES = false>
__global__ __launch_bounds__(BLOCK, BOUNCE_WAVES) void k_bounce_trav(const Inner* __restrict__ inner,
                                                          const QNode* __restrict__ qn,
                                                          const float4* __restrict__ leaf, uint32_t T,
                                                          const RayQ* __restrict__ qin,
                                                          const uint32_t* __restrict__ qin_count,
                                                          const uint32_t* __restrict__ perm,
                                                          float2* __restrict__ hitrec, uint32_t* __restrict__ next,
                                                          unsigned long long* __restrict__ counters,
                                                          unsigned long long* __restrict__ overflow, int stack_limit,
                                                          uint32_t* __restrict__ defer, const uint4* __restrict__ topo,
                                                          const float* __restrict__ nbox, uint32_t nwalk, TraceArgs ta,
                                                          RayQ* __restrict__ qout, uint32_t* __restrict__ qout_count,
                                                          int emit, uint32_t* __restrict__ redo,
                                                          uint32_t* __restrict__ redo_count) {
    constexpr bool NEAREST = MODE >= 1, WIDE = MODE == 2;
    static_assert(!CERT || (WIDE && !LIM), "the certified walk is the 4-wide one, without a stack limit");
    const int limit = LIM ? stack_limit : WIDE ? STACK4B : STACK_SIZE;
    const uint32_t n = *qin_count;
    if (n == 0) return;
    const uint32_t lane = lane_id();
    Counts c = {0, 0, 0, 0, 0};
    // (early shading on: the hit records are written through to memory, st_hitrec)
    constexpr bool wt = CERT && ES && RTBVH_EARLY_SHADE;   // (the ES instance is launched with shading workgroups)
    if (CERT && ES && RTBVH_EARLY_SHADE && blockIdx.x >= nwalk) {   // a shading workgroup (early shading, above)
        const uint32_t b0 = (blockIdx.x - nwalk) * ESHADE_RAYS;
        uint32_t hits = 0, tex = 0;
        for (uint32_t base = b0; base < b0 + ESHADE_RAYS && base < n; base += BLOCK) {   // (uniform)
            const uint32_t i = base + threadIdx.x;
            bool valid = false;
            float2 h2 = make_float2(0.f, 0.f);
            if (i < n) {
                unsigned long long* hp = reinterpret_cast<unsigned long long*>(hitrec + i);
                const unsigned long long v = __hip_atomic_load(hp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t xb = (uint32_t)v, yb = (uint32_t)(v >> 32);
                // final: written, not taken, and not a deferred ray's "deferred" record (its walk writes it again)
                const bool ready = xb != HIT_NOT_READY && xb != HIT_SHADED &&
                                   !(xb == 0xFF800000u && yb == (INVALID ^ HIT_FLAG));
                if (ready) {
                    unsigned long long exp = v;
                    valid = __hip_atomic_compare_exchange_strong(
                        hp, &exp, (unsigned long long)HIT_SHADED | (unsigned long long)yb << 32, __ATOMIC_RELAXED,
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                h2 = make_float2(__uint_as_float(xb), __uint_as_float(yb));
            }
            RayQ e;
            bool live, flagged;
            uint32_t h1 = 0, t1 = 0;   // (bounce_apply sets them: one ray's)
            bounce_shade_ray<true>(ta, qin, i, h2, valid, e, live, flagged, h1, t1);
            hits += h1;
            tex += t1;
            const uint32_t rs = wave_append(flagged, redo_count);
            if (flagged) redo[rs] = i;
            const uint32_t qs = wave_append(emit && live, qout_count);
            if (emit && live) qout[qs] = e;
        }
        if (COUNT) flush_counts<COUNT>(ta, c, hits, tex, 5);
        return;
    }
#ifdef RTBVH_TAIL_PROBE   // (A/B probe builds: each wave's end of walk, 100-us buckets from its start, into counters[32..63])
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    if (CERT && DEFER_WORKERS && blockIdx.x < DEFER_WORKERS && gridDim.x > 2 * DEFER_WORKERS && threadIdx.x < 64) {
        for (;;) {
            defer_walk_all<COUNT>(next, defer, inner, topo, nbox, leaf, T, qin, hitrec, c, wt);
            // every segment claimed (lane k: segment k's counter past its length): no ray left to defer but
            // those being claimed right now
            bool used = true;
            for (uint32_t seg = lane; seg < NEXT_SEGS; seg += 64) {
                const uint32_t s0 = (uint32_t)((uint64_t)n * seg / NEXT_SEGS);
                const uint32_t len = (uint32_t)((uint64_t)n * (seg + 1) / NEXT_SEGS) - s0;
                used = used && __hip_atomic_load(next + NEXT_STRIDE * seg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= len;
            }
            if (__ballot(!used) == 0) break;
            __builtin_amdgcn_s_sleep(64);
        }
        defer_walk_all<COUNT>(next, defer, inner, topo, nbox, leaf, T, qin, hitrec, c, wt);
        if (COUNT) {
            unsigned long long v[2] = {c.internal, c.leaf};
#pragma unroll
            for (int k = 0; k < 2; k++)
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
            if (lane == 0) {
                atomicAdd(&counters[5], v[0]);
                atomicAdd(&counters[6], v[1]);
            }
        }
        return;
    }
    bool has = false, hit = false, qfast = false;
    uint32_t r = 0, node = 0, top = INVALID, bl = 0, guard = 0;
    uint32_t btri = 0;       // triangle of the best hit (leaf record word 9): the hit record's id
    uint64_t key = NO_HIT;   // WIDE: the lexicographic (t, leaf) minimum (hit / best / bl of the binary walks)
    int sp = 0;
    float best = 0.f;
    f3 o = mk(0.f, 0.f, 0.f), d = o, inv = o;
    // CERT: the per-node margin's coefficients (margin.h rho_n; each QNode carries its node's edge bound
    // and margin range) and the ray's flag
    const MtNodeK nk = mt_node_consts();
    bool flg = false;
    __shared__ uint32_t s_stk[WIDE ? 1 : SB][WIDE ? 1 : BLOCK];   // (none for WIDE: its LDS is the 6-B stack)
    uint32_t stack[WIDE ? 1 : STACK_SIZE - SB];   // entries [SB, STACK_SIZE)
    __shared__ uint32_t s_wid[WIDE ? SW : 1][BLOCK];
    __shared__ uint16_t s_wt[WIDE ? SW : 1][BLOCK];
    uint2 wstack[WIDE ? STACK4B - SW : 1];       // entries [SW, STACK4B)
    const uint32_t tid = threadIdx.x;
    auto spush = [&](uint32_t v) {
        if (sp < SB) s_stk[sp][tid] = v;
        else stack[sp - SB] = v;
        ++sp;
    };
    auto spop_top = [&]() {   // --sp; refill the cached top from entry sp
        if (--sp >= 0) top = sp < SB ? s_stk[sp][tid] : stack[sp - SB];
    };
    auto wpush = [&](uint32_t id, float t) {
        if (sp < SW) {
            s_wid[sp][tid] = id;
            s_wt[sp][tid] = bf16_down(t);
        } else {
            wstack[sp - SW] = make_uint2(id, __float_as_uint(t));
        }
        ++sp;
    };
    // WIDE: the QNode at `node` (words q0..q3): its four entries, hit ones first by entry distance
    // (k: entry distance, i: id; a missing child has INVALID and +inf)
    auto qchildren = [&](v4f q0, v4f q1, v4f q2, v4f q3, float& k0, float& k1, float& k2, float& k3, uint32_t& i0,
                         uint32_t& i1, uint32_t& i2, uint32_t& i3) {
        // the four grandchildren: ids (a3.x, a3.y, b3.x, b3.y), entry distances t0..t3
        uint4 a3, b3;
        float t0, t1, t2, t3;
        bool h0, h1, h2, h3;
        const float kbb = key_t(key);
        if (CERT || q0.w != 0.f) {   // quantized node: q0..q3 = QNode words 0..15 (CERT: the step checked)
            // scl[1], scl[2] carry the node's margin codes in their (otherwise zero) mantissas (margin.h)
            const uint32_t wy = __float_as_uint(q1.x), wz = __float_as_uint(q1.y);
            const float ox = q0.x, oy = q0.y, oz = q0.z, sx = q0.w;
            const float sy = __uint_as_float(wy & 0xFF800000u), sz = __uint_as_float(wz & 0xFF800000u);
            const uint32_t lx = __float_as_uint(q1.z), ly = __float_as_uint(q1.w), lz = __float_as_uint(q2.x);
            const uint32_t hx = __float_as_uint(q2.y), hy = __float_as_uint(q2.z), hz = __float_as_uint(q2.w);
            a3 = make_uint4(__float_as_uint(q3.x), __float_as_uint(q3.y), 0u, 0u);
            b3 = make_uint4(__float_as_uint(q3.z), __float_as_uint(q3.w), 0u, 0u);
            // (CERT: a ray the slack test cannot take never steps -- it is flagged at its first step -- so
            // every stepping ray takes this branch)
            if (qfast || CERT) {
                // CERT: the node's margin rho_n(best) (0 before the first bound) and its range
                float rr = 0.f, tcn = 0.f;
                MtNodeRho nr{0.f, 0.f};
                if (CERT) {
                    nr = mt_node_prep(nk, mt_code_val(wy));
                    tcn = mt_code_val(wz);
                    rr = kbb < __builtin_inff() ? mt_node_eval(nr, kbb) : 0.f;
                }
                const QAxis X = qaxis<CERT>(ox, sx, lx, hx, o.x, inv.x, rr),
                            Y = qaxis<CERT>(oy, sy, ly, hy, o.y, inv.y, rr),
                            Z = qaxis<CERT>(oz, sz, lz, hz, o.z, inv.z, rr);
                if (CERT) {
                    const f3 ai = mk(fabsf(inv.x), fabsf(inv.y), fabsf(inv.z));
                    h0 = qbox_fast_cert(X, Y, Z, 0, kbb, nk, nr, ai, tcn, t0);
                    h1 = qbox_fast_cert(X, Y, Z, 1, kbb, nk, nr, ai, tcn, t1);
                    h2 = qbox_fast_cert(X, Y, Z, 2, kbb, nk, nr, ai, tcn, t2);
                    h3 = qbox_fast_cert(X, Y, Z, 3, kbb, nk, nr, ai, tcn, t3);
                } else {
                    h0 = qbox_fast(X, Y, Z, 0, true, kbb, t0);
                    h1 = qbox_fast(X, Y, Z, 1, true, kbb, t1);
                    h2 = qbox_fast(X, Y, Z, 2, true, kbb, t2);
                    h3 = qbox_fast(X, Y, Z, 3, true, kbb, t3);
                }
            } else {
    #define RTBVH_QBOX(c, t)                                                                                      \
ray_box(o, inv, qdecode(ox, sx, lx, c), qdecode(oy, sy, ly, c), qdecode(oz, sz, lz, c), qdecode(ox, sx, hx, c), \
        qdecode(oy, sy, hy, c), qdecode(oz, sz, hz, c), true, kbb, t)
                h0 = RTBVH_QBOX(0, t0);
                h1 = RTBVH_QBOX(1, t1);
                h2 = RTBVH_QBOX(2, t2);
                h3 = RTBVH_QBOX(3, t3);
    #undef RTBVH_QBOX
            }
            h1 = h1 & (a3.y != INVALID);
            h3 = h3 & (b3.y != INVALID);
        } else {
            // a node without a finite grid: its exact record pair (node = its slot; the
            // pair of its children's records is at 2 * own, own = word 14 of its record; the
            // build writes the pseudo-records of such a node's leaf children whatever the flags).
            // (Not widened by the margin: a certified walk ends the ray there, flagged -- below)
            const uint32_t own = __float_as_uint(reinterpret_cast<const v4f*>(inner + node)[3].z);
            const v4f* pr = reinterpret_cast<const v4f*>(inner + 2 * (size_t)own);
            q0 = pr[0]; q1 = pr[1]; q2 = pr[2]; q3 = pr[3];
            const v4f q4 = pr[4], q5 = pr[5], q6 = pr[6], q7 = pr[7];
            a3 = make_uint4(__float_as_uint(q3.x), __float_as_uint(q3.y), 0u, 0u);
            b3 = make_uint4(__float_as_uint(q7.x), __float_as_uint(q7.y), 0u, 0u);
            // grandchild ids -> slots (2 * parent + side; parent = word 14)
            const uint32_t ol = __float_as_uint(q3.z), orr = __float_as_uint(q7.z);
            if (!(a3.x & LEAF_BIT)) a3.x = 2 * ol;
            if (a3.y != INVALID && !(a3.y & LEAF_BIT)) a3.y = 2 * ol + 1;
            if (!(b3.x & LEAF_BIT)) b3.x = 2 * orr;
            if (b3.y != INVALID && !(b3.y & LEAF_BIT)) b3.y = 2 * orr + 1;
            h0 = ray_box_xy(o, inv, q0.xy, q0.zw, q2.x, q2.y, true, kbb, t0);
            h1 = ray_box_xy(o, inv, q1.xy, q1.zw, q2.z, q2.w, true, kbb, t1) & (a3.y != INVALID);
            h2 = ray_box_xy(o, inv, q4.xy, q4.zw, q6.x, q6.y, true, kbb, t2);
            h3 = ray_box_xy(o, inv, q5.xy, q5.zw, q6.z, q6.w, true, kbb, t3) & (b3.y != INVALID);
        }
        const float INF = __builtin_inff();
        k0 = h0 ? t0 : INF; k1 = h1 ? t1 : INF; k2 = h2 ? t2 : INF; k3 = h3 ? t3 : INF;
        i0 = h0 ? a3.x : INVALID; i1 = h1 ? a3.y : INVALID; i2 = h2 ? b3.x : INVALID; i3 = h3 ? b3.y : INVALID;
        // 4-element sorting network on the entry distance (missing children last)
        sort2(k0, i0, k1, i1);
        sort2(k2, i2, k3, i3);
        sort2(k0, i0, k2, i2);
        sort2(k1, i1, k3, i3);
        sort2(k1, i1, k2, i2);
    };
    bool drained = false;
    uint32_t kseg = 0;   // segments claimed from so far (wave-uniform)
    unsigned long long wsteps = 0, mixed = 0, active_lanes = 0;
    while (true) {
        const uint64_t idle = __ballot(!has);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (!drained && (nidle >= REFILL_MIN || nidle == 64)) {
            const uint32_t seg = claim_segment(kseg);
            const uint32_t s0 = (uint32_t)((uint64_t)n * seg / NEXT_SEGS);
            const uint32_t len = (uint32_t)((uint64_t)n * (seg + 1) / NEXT_SEGS) - s0;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(next + NEXT_STRIDE * seg, nidle);
            base = __builtin_amdgcn_readfirstlane(base);
            if (base + nidle >= len && ++kseg == NEXT_SEGS) drained = true;   // segment (and the last) used up
            if (!has) {
                const uint32_t p = base + lane_rank(idle);
                if (p < len) {
                    r = perm ? perm[s0 + p] : s0 + p;
                    const float4 q0 = reinterpret_cast<const float4*>(qin + r)[0];
                    const float4 q1 = reinterpret_cast<const float4*>(qin + r)[1];
                    o = mk(q0.z, q0.w, q1.x);
                    d = mk(q1.y, q1.z, q1.w);
                    inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
                    qfast = WIDE && qnode_fast_ray(o, inv);
                    has = true;
                    hit = false;
                    best = 0.f;
                    bl = 0;
                    key = NO_HIT;
                    sp = 0;
                    top = INVALID;
                    node = root_slot(T);
                    guard = 2 * T + 2;
                    if (CERT) {   // a ray the margin does not cover is deferred (DEFER_* below)
                        flg = !(qfast && dot(d, d) <= MT_DD);
                        if (flg) {
                            // the "deferred" record first, then the entry with release order: a wave that takes
                            // the entry (acquire) writes the walk's record after this one, never under it
                            const float2 mk_def = make_float2(-__builtin_inff(), __uint_as_float(INVALID ^ HIT_FLAG));
                            if (wt) st_hitrec(hitrec + r, mk_def);
                            else hitrec[r] = mk_def;
                            const uint32_t k = atomicAdd(next + DEFER_COUNT, 1u);
                            __hip_atomic_store(defer + k, r | DEFER_VALID, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                            has = false;
                            flg = false;
                        }
                    }
                }
            }
        }
        // every refill either hands out rays or moves on to the next segment (the last one
        // sets `drained`), so a wave with no ray left loops back to refill until the queue is drained
        if (__ballot(has) == 0 && drained) break;
        if (COUNT) {   // wave-level divergence census (stats trav_*; all lanes converged here)
            const uint64_t act = __ballot(has);
            const uint64_t lf = __ballot(has && (node & LEAF_BIT) != 0);
            wsteps++;
            active_lanes += (uint32_t)__popcll(act);
            mixed += (lf != 0 && lf != act);
        }
        if (!has) continue;
        bool done = false;
        if (WIDE) {
            // A step: the QNode of an internal `node`, then one leaf test -- the nearest child when it
            // is a leaf (the next child is visited), or the leaf the step began at -- so a leaf found
            // by the node test costs no step of its own, and the leaf test is one block of code.
            uint32_t L = INVALID;
            if (GUARD && --guard == 0) {
                c.overflow++;
                done = true;
                if (CERT) flg = true;
            } else {
                if (node & LEAF_BIT) {
                    L = node;
                    node = INVALID;
                } else {
                    const v4f* rr = reinterpret_cast<const v4f*>(qn + node);
                    v4f q0 = rr[0], q1 = rr[1], q2 = rr[2], q3 = rr[3];
                    pin(q0); pin(q1); pin(q2); pin(q3);
                    if (COUNT) c.internal++;
                    float k0 = 0.f, k1 = 0.f, k2 = 0.f, k3 = 0.f;
                    uint32_t i0 = INVALID, i1 = INVALID, i2 = INVALID, i3 = INVALID;
                    // CERT: a node without a finite grid (its corners past 2^100: the margin does not cover
                    // its exact boxes) ends the walk, the ray flagged for the reference-order re-trace
                    if (CERT && q0.w == 0.f) {
                        flg = true;
                        done = true;
                    } else {
                        qchildren(q0, q1, q2, q3, k0, k1, k2, k3, i0, i1, i2, i3);
                    }
#ifdef RTBVH_DEBUG_PIXEL   // (scripts/debug_walk.py: one ray's walk, step by step, from the COUNT kernel)
                    if (COUNT && qin[r].idx == (uint32_t)RTBVH_DEBUG_PIXEL)
                        printf("DBG %d q %u sp %d kb %.6g key %.6g | %.6g %x %.6g %x %.6g %x %.6g %x\n", (int)CERT, node,
                               sp, key_t(key), key_t(key), k0, i0, k1, i1, k2, i2, k3, i3);
#endif
                    const bool lf0 = i0 != INVALID && (i0 & LEAF_BIT);
                    L = lf0 ? i0 : INVALID;
                    node = lf0 ? i1 : i0;   // INVALID when no child is left -> pop below
                    if (sp + 3 > limit) {
                        c.overflow++;
                        done = true;
                        if (CERT) flg = true;
                    } else {   // push the others farthest first
                        if (i3 != INVALID) wpush(i3, k3);
                        if (i2 != INVALID) wpush(i2, k2);
                        if (!lf0 && i1 != INVALID) wpush(i1, k1);
                    }
                }
#ifdef RTBVH_DEBUG_PIXEL
                if (COUNT && L != INVALID && qin[r].idx == (uint32_t)RTBVH_DEBUG_PIXEL)
                    printf("DBG %d leaf %x sp %d kb %.6g key %.6g\n", (int)CERT, L, sp, key_t(key), key_t(key));
#endif
                if (L != INVALID) {   // branch-free test (the same accept predicate), u64 key minimum
                    const uint32_t j = L & ~LEAF_BIT;
                    const v4f* lr = reinterpret_cast<const v4f*>(leaf + 4 * (size_t)j);
                    v4f la = lr[0], lb = lr[1], lc = lr[2];
                    pin(la); pin(lb); pin(lc);
                    if (COUNT) c.leaf++;
                    const float tw = ray_triangle_flat(o, d, mk(la.x, la.y, la.z), mk(la.w, lb.x, lb.y),
                                                       mk(lb.z, lb.w, lc.x), true);
                    const uint64_t k = tw == -1.f ? ~0ull : (uint64_t)__float_as_uint(tw) << 32 | j;
                    btri = k < key ? __float_as_uint(lc.y) & ~LEAF_BIT : btri;
                    key = k < key ? k : key;
                }
                if (!done && node == INVALID) {   // pop, dropping entries that cannot improve
                    while (sp > 0) {
                        --sp;
                        uint2 e;
                        if (sp < SW) e = make_uint2(s_wid[sp][tid], __float_as_uint(bf16_up(s_wt[sp][tid])));
                        else e = wstack[sp - SW];
                        if (__uint_as_float(e.y) <= key_t(key)) {
                            node = e.x;
                            break;
                        }
                    }
                    done = node == INVALID;
                }
            }
        } else {
            // binary walks: one fetch for every active lane, leaf or internal, before the branch: a
            // wave holding both kinds would otherwise wait for two dependent round trips (leaf records
            // and child-pair records are both 64-B aligned records)
            const bool isleaf = (node & LEAF_BIT) != 0;
            const v4f* rr = isleaf ? reinterpret_cast<const v4f*>(leaf + 4 * (size_t)(node & ~LEAF_BIT))
                                   : reinterpret_cast<const v4f*>(inner + node);
            v4f q0 = rr[0], q1 = rr[1], q2 = rr[2], q3 = rr[3];
            pin(q0); pin(q1); pin(q2); pin(q3);
            if (GUARD && --guard == 0) {
                c.overflow++;
                done = true;
            } else if (isleaf) {
                const uint32_t j = node & ~LEAF_BIT;
                if (COUNT) c.leaf++;
                const float t = ray_triangle(o, d, mk(q0.x, q0.y, q0.z), mk(q0.w, q1.x, q1.y), mk(q1.z, q1.w, q2.x));
                if (t != -1.f && (!hit || t < best || (NEAREST && t == best && j < bl))) {
                    best = t;
                    bl = j;
                    btri = __float_as_uint(q2.y) & ~LEAF_BIT;
                    hit = true;
                }
                node = top;                             // pop
                spop_top();
                done = sp == -1;
            } else {
                if (COUNT) c.internal++;
                const uint32_t own = __float_as_uint(q3.z);
                const uint32_t cl = child_slot(__float_as_uint(q3.x), own, 0), cr = child_slot(__float_as_uint(q3.y), own, 1);
                float tl, tr;
                const bool lh = ray_box_xy(o, inv, q0.xy, q0.zw, q2.x, q2.y, hit, best, tl);
                const bool rh = ray_box_xy(o, inv, q1.xy, q1.zw, q2.z, q2.w, hit, best, tr);
                if (!lh && !rh) {
                    node = top;                             // pop
                    spop_top();
                    done = sp == -1;
                } else {
                    const bool swap = NEAREST && lh && rh && tr < tl;
                    if (lh && rh) {
                        if (sp + 1 >= limit) {
                            c.overflow++;
                            node = top;
                            spop_top();
                            done = sp == -1;
                        } else {
                            spush(top);                     // push the second child
                            top = swap ? cl : cr;
                            node = swap ? cr : cl;
                        }
                    } else {
                        node = lh ? cl : cr;
                    }
                }
            }
        }
        if (done) {
            // (t, triangle) of the hit, INVALID for a miss: the shading reads no leaf record
            if (WIDE) {
                uint32_t w = key != NO_HIT ? btri : INVALID;
                if (CERT && flg) w ^= HIT_FLAG;   // (a hit: bit 30 set; a miss: bit 30 cleared)
                if (CERT && wt) st_hitrec(hitrec + r, make_float2(key_t(key), __uint_as_float(w)));
                else hitrec[r] = make_float2(key_t(key), __uint_as_float(w));
            }
            else hitrec[r] = make_float2(best, __uint_as_float(hit ? btri : INVALID));
            has = false;
            if (COUNT && GUARD) {   // walk length census (stats trav_max_steps / trav_steps_log2)
                const uint32_t steps = 2 * T + 2 - guard;
                atomicAdd(&counters[32 + (31 - __clz(steps | 1u))], 1ull);
                atomicMax(&counters[13], (unsigned long long)steps);
                atomicMax(&counters[20], (unsigned long long)steps << 32 | qin[r].idx);   // (the longest: its pixel)
            }
        }
    }
#ifdef RTBVH_TAIL_PROBE
    if (lane == 0 && !COUNT) {
        const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t_start;   // 100 MHz: 10000 ticks = 100 us
        atomicAdd(&counters[32 + min(31u, (uint32_t)(dt / 10000u))], 1ull);
    }
#endif
    if (CERT && RTBVH_DEFER_INWALK) {
        // The deferred rays (the slack test cannot take them) the workers above have not taken yet: once its part
        // of the queue is drained, the wave walks them in the reference order; the hit record says "exact" (t
        // negated), so k_bounce_shade shades it without a certificate.  A deferred ray no wave takes here
        // (appended after the waves looked) is re-traced by k_bounce_redo.
        defer_walk_all<COUNT>(next, defer, inner, topo, nbox, leaf, T, qin, hitrec, c, wt);
    }
    if (COUNT || __ballot(c.overflow != 0)) {
        unsigned long long v[3] = {c.internal, c.leaf, c.overflow};
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
        if (lane == 0) {
            if (COUNT) {
                atomicAdd(&counters[5], v[0]);
                atomicAdd(&counters[6], v[1]);
                atomicAdd(&counters[10], wsteps);
                atomicAdd(&counters[11], mixed);
                atomicAdd(&counters[12], active_lanes);
            }
            if (v[2]) {
                atomicAdd(&counters[8], v[2]);
                atomicAdd(overflow, v[2]);
            }
        }
    }
}

// RayTraceReflection.hlsl:19-60 for one queued ray e from its closest hit (tri at t; tri INVALID: a
// miss): colour, intensity, the reflectRay record, and the next ray in e (returns whether it is live)
__device__ __forceinline__ bool bounce_apply(const TraceArgs& a, RayQ& e, uint32_t tri, float t, uint32_t& hits,
                                             uint32_t& tex) {
    const f3 o = mk(e.ox, e.oy, e.oz), d = mk(e.dx, e.dy, e.dz);
    float4 col = a.color[e.idx];
    float intensity = e.intensity;
    bool live = false;
    if (tri != INVALID) {
        hits = 1;
        const HitInfo h = shade_hit_tri(a, tri, o, d, t);
        tex = h.textured;
        col = make_float4(lerpf(col.x, h.color.x, intensity), lerpf(col.y, h.color.y, intensity),
                          lerpf(col.z, h.color.z, intensity), lerpf(col.w, h.color.w, intensity));
        intensity *= h.shininess / 1000.f * 1;
        const f3 ro = add(h.hitp, mul(h.nrm, .0001f));   // RAY_OFFSET .0001
        const f3 rd = normalize(reflect(d, h.nrm));
        e.intensity = intensity;
        e.ox = ro.x; e.oy = ro.y; e.oz = ro.z;
        e.dx = rd.x; e.dy = rd.y; e.dz = rd.z;
        live = 0 < intensity;
        if (a.refl_rec) put_record(a.refl_rec, e.idx, intensity, true, ro, rd, col);   // :42-46
    } else {
        col = make_float4(lerpf(col.x, .5f, intensity), lerpf(col.y, .5f, intensity),
                          lerpf(col.z, .5f, intensity), lerpf(col.w, 1.f, intensity));
        intensity = 0.f;
        if (a.refl_rec) {   // :50-55: the ray stays, intensity 0, colour blended
            float* r = a.refl_rec + 14 * (size_t)e.idx;
            r[0] = 0.f;
            r[10] = col.x; r[11] = col.y; r[12] = col.z; r[13] = col.w;
        }
    }
    a.color[e.idx] = col;
    if (a.intensity) a.intensity[e.idx] = intensity;
    return live;
}

// The certificate of a certified walk's hit: the reference's findCollision
// (RayTraceTraversal.hlsl:106-193) reaches leaf x -- and, the walk having seen every triangle that could
// be accepted at t <= its best, returns x -- when x's own box passes the reference slab test with the
// bound t (every box above contains it: the slab test is monotone in the box, so they pass too, at every
// bound the reference holds, all >= t).  The box is the leaf's: min / max of its clip-space vertices
// (build.hip leaf_record_words, MortonCodes.hlsl:87-96), from the triangle's record.
__device__ __forceinline__ bool leaf_certified(const TraceArgs& a, uint32_t tri, f3 o, f3 inv, float t) {
    const float4* P = a.tclip + TCS * (size_t)tri;
    const float4 a0 = P[0], a1 = P[1], a2 = P[2];
    const f3 v0 = mk(a0.x, a0.y, a0.z), v1 = mk(a1.x, a1.y, a1.z), v2 = mk(a2.x, a2.y, a2.z);
    const f3 lo = vmin(vmin(v0, v1), v2), hi = vmax(vmax(v0, v1), v2);
    float tm;
    return ray_box(o, inv, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, true, t, tm);
}

// RayTraceReflection.hlsl:19-60 for queued ray i from its hit record h2 (valid: i is a ray to shade now).  CERT: a ray
// whose walk flagged it or whose hit fails the certificate is flagged (the caller lists it for the re-trace) instead
template <bool CERT>
__device__ __forceinline__ void bounce_shade_ray(const TraceArgs& a, const RayQ* __restrict__ qin, uint32_t i, float2 h2,
                                                 bool valid, RayQ& e, bool& live, bool& flagged, uint32_t& hits,
                                                 uint32_t& tex) {
    live = false;
    flagged = false;
    if (!valid) return;
    e = qin[i];
    uint32_t tri = __float_as_uint(h2.y);
    bool skip = false;
    if (CERT) {
        flagged = hit_flagged(tri);
        tri = (tri & LEAF_BIT) ? INVALID : tri & ~HIT_FLAG;
        if (signbit(h2.x)) {   // the walk's deferred rays (trace.hip DEFER_*): walked in the reference order
            skip = flagged;    //   by the walk's drained waves (exact: shaded as is), or by k_bounce_redo
            flagged = false;
            h2.x = -h2.x;
        } else if (!flagged && tri != INVALID) {
            const f3 d = mk(e.dx, e.dy, e.dz);
            flagged = !leaf_certified(a, tri, mk(e.ox, e.oy, e.oz), mk(1.f / d.x, 1.f / d.y, 1.f / d.z), h2.x);
        }
    }
    if (!flagged && !skip) live = bounce_apply(a, e, tri, h2.x, hits, tex);
}
template <bool COUNT, bool CERT>
__global__ __launch_bounds__(BLOCK) void k_bounce_shade(TraceArgs a, const RayQ* __restrict__ qin,
                                                        const uint32_t* __restrict__ qin_count,
                                                        const float2* __restrict__ hitrec, RayQ* __restrict__ qout,
                                                        uint32_t* __restrict__ qout_count, int emit,
                                                        uint32_t* __restrict__ redo, uint32_t* __restrict__ redo_count) {
    const uint32_t n = *qin_count;
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (blockIdx.x * BLOCK >= n) return;   // whole block past the queue (wave_append below needs all lanes)
    bool live = false, flagged = false;
    uint32_t hits = 0, tex = 0;
    RayQ e;
    float2 h2 = make_float2(0.f, 0.f);
    if (i < n) h2 = hitrec[i];
    // (a ray the walk's early shading took is done: RTBVH_EARLY_SHADE)
    bounce_shade_ray<CERT>(a, qin, i, h2, i < n && !(CERT && __float_as_uint(h2.x) == HIT_SHADED), e, live, flagged, hits,
                           tex);
    if (CERT) {
        const uint32_t slot = wave_append(flagged, redo_count);
        if (flagged) redo[slot] = i;
    }
    const uint32_t slot = wave_append(emit && live, qout_count);
    if (emit && live) qout[slot] = e;
    if (COUNT) {
        Counts c = {0, 0, 0, 0, 0};
        flush_counts<COUNT>(a, c, hits, tex, 5);
    }
}
// (early shading: every hit record of the pass "not written yet" before the walk)
__global__ __launch_bounds__(BLOCK) void k_hit_init(float2* __restrict__ hitrec, const uint32_t* __restrict__ qin_count) {
    const uint32_t n = *qin_count;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK)
        hitrec[i] = make_float2(__uint_as_float(HIT_NOT_READY), __uint_as_float(HIT_NOT_READY));
}

// The reference-order re-trace of the rays a certified bounce pass flagged (redo: queue indices): the
// exact findCollision DFS (traverse, reference order), then the shading as k_bounce_shade.  A fixed grid
// over the count on the device (a captured frame replays it as it is).
// Then the walk's deferred rays no drained wave claimed (trace.hip DEFER_*: entries [next[DEFER_CLAIM],
// next[DEFER_COUNT]) of the defer list, cleared as they are read) come first in the index space.
template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void k_bounce_redo(TraceArgs a, const RayQ* __restrict__ qin,
                                                       const uint32_t* __restrict__ redo,
                                                       const uint32_t* __restrict__ redo_count,
                                                       RayQ* __restrict__ qout, uint32_t* __restrict__ qout_count,
                                                       int emit, uint32_t* __restrict__ defer,
                                                       const uint32_t* __restrict__ dnext) {
    const uint32_t d0 = defer ? min(dnext[DEFER_CLAIM], dnext[DEFER_COUNT]) : 0u;
    const uint32_t nd = defer ? dnext[DEFER_COUNT] - d0 : 0u;
    const uint32_t n = nd + *redo_count;
    Counts c = {0, 0, 0, 0, 0};
    uint32_t hits = 0, tex = 0;
    for (uint32_t base = blockIdx.x * BLOCK; base < n; base += gridDim.x * BLOCK) {
        const uint32_t i = base + threadIdx.x;
        bool live = false;
        RayQ e;
        if (i < n) {
            uint32_t r;
            if (i < nd) {
                r = defer[d0 + i] & ~DEFER_VALID;
                defer[d0 + i] = 0u;
            } else {
                r = redo[i - nd];
            }
            e = qin[r];
            const f3 o = mk(e.ox, e.oy, e.oz), d = mk(e.dx, e.dy, e.dz);
            const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
            float best;
            uint32_t bl;
            const bool h = traverse_ref<COUNT>(a, o, d, inv, best, bl, c);
            const uint32_t tri = h ? __float_as_uint(a.leaf[4 * (size_t)bl + 2].y) & ~LEAF_BIT : INVALID;
            uint32_t h1 = 0, t1 = 0;
            live = bounce_apply(a, e, tri, best, h1, t1);
            hits += h1;
            tex += t1;
        }
        const uint32_t slot = wave_append(emit && live, qout_count);
        if (emit && live) qout[slot] = e;
    }
    flush_counts<COUNT>(a, c, hits, tex, 5);
}

// bounce-ray coherence sort key (results do not depend on the order): direction
// octant in bits 27..29, 9-bit-per-axis Morton code of the origin inside the scene
// box in bits 0..26.  Entries past the live count get the largest key and sort last.
__device__ __forceinline__ uint32_t spread9(uint32_t v) {
    v &= 0x1FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
__device__ __forceinline__ uint32_t q9(float x, float lo, float hi) {
    float t = (x - lo) / (hi - lo) * 512.f;
    t = fminf(fmaxf(t, 0.f), 511.f);
    return (uint32_t)t;
}
__global__ __launch_bounds__(BLOCK) void k_bounce_keys(const RayQ* __restrict__ q, const uint32_t* __restrict__ count,
                                                       const float* __restrict__ box, uint32_t P,
                                                       uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= P) return;
    uint32_t key = 0xFFFFFFFFu;
    if (i < *count) {
        const RayQ e = q[i];
        const uint32_t oct = (e.dx < 0.f) | ((e.dy < 0.f) << 1) | ((e.dz < 0.f) << 2);
        const uint32_t m = spread9(q9(e.ox, box[0], box[3])) << 2 | spread9(q9(e.oy, box[1], box[4])) << 1 |
                           spread9(q9(e.oz, box[2], box[5]));
        key = oct << 27 | m;
    }
    keys[i] = key;
    vals[i] = i;
}

// RayTraceBVHPS.hlsl:13-16 + the R8G8B8A8_UNORM target: screen row y <- framebuffer row H-1-y
__device__ __forceinline__ uint32_t unorm8(float c) { return (uint32_t)floorf(sat(c) * 255.f + .5f); }
__global__ __launch_bounds__(BLOCK) void k_present(const float4* __restrict__ color, uint32_t W, uint32_t H,
                                                   uint32_t* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= (size_t)W * H) return;
    const uint32_t y = (uint32_t)(i / W), x = (uint32_t)(i % W);
    const float4 c = color[(size_t)(H - 1 - y) * W + x];
    out[i] = unorm8(c.x) | unorm8(c.y) << 8 | unorm8(c.z) << 16 | unorm8(c.w) << 24;
}

// frame row y of a W x H frame traced as 8-row bands dealt over nranks: band b = y / 8 is
// rank r's p-th band, so it sits at row p * 8 + y % 8 of that rank's compact buffer, buffers
// stacked stride_rows apart (tiles.py layout).  Round-robin (slots null): r = b % nranks,
// p = b / nranks; a weighted deal (rtbvh_deal_bands): slots[b] = r << 24 | p.
__global__ __launch_bounds__(BLOCK) void k_assemble(const float4* __restrict__ bands,
                                                    const uint32_t* __restrict__ slots, uint32_t stride_rows,
                                                    uint32_t W, uint32_t H, uint32_t nranks,
                                                    float4* __restrict__ frame) {
    const size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= (size_t)W * H) return;
    const uint32_t y = (uint32_t)(i / W), x = (uint32_t)(i % W);
    const uint32_t b = y >> 3, sl = slots ? slots[b] : (b % nranks) << 24 | (b / nranks);
    const uint32_t r = sl >> 24, k = (sl & 0xFFFFFFu) * 8 + (y & 7u);
    frame[i] = bands[((size_t)r * stride_rows + k) * W + x];
}

// frames compared pixel for pixel (rtbvh_compare_frames): *diff += pixels whose 16 bytes differ
__global__ __launch_bounds__(BLOCK) void k_count_diff(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                      size_t n, unsigned long long* __restrict__ diff) {
    unsigned long long cnt = 0;
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) {
        const uint4 x = a[i], y = b[i];
        cnt += (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane_id() == 0 && cnt) atomicAdd(diff, cnt);
}

// the same for 32-bit words (intensities)
__global__ __launch_bounds__(BLOCK) void k_count_diff32(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                        size_t n, unsigned long long* __restrict__ diff) {
    unsigned long long cnt = 0;
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) cnt += a[i] != b[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane_id() == 0 && cnt) atomicAdd(diff, cnt);
}

template <bool COUNT, int K>
void launch_primary_t(const TraceArgs& a, RayQ* q, uint32_t* qcount, bool emit, dim3 grid, hipStream_t s) {
    if (a.limited) hipLaunchKernelGGL((k_primary<COUNT, K, true>), grid, dim3(BLOCK), 0, s, a, q, qcount, (int)emit);
    else hipLaunchKernelGGL((k_primary<COUNT, K, false>), grid, dim3(BLOCK), 0, s, a, q, qcount, (int)emit);
}
template <int K>
void launch_primary_c(const TraceArgs& a, RayQ* q, uint32_t* qcount, bool count, bool emit, dim3 grid, hipStream_t s) {
    if (count) launch_primary_t<true, K>(a, q, qcount, emit, grid, s);
    else launch_primary_t<false, K>(a, q, qcount, emit, grid, s);
}

template <bool COUNT, int MODE>
void launch_bounce_trav_t(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const uint32_t* perm,
                          float2* hitrec, uint32_t* next, uint32_t blocks, bool cert, uint32_t* defer, hipStream_t s,
                          const BounceShade* es) {
    const int lim = MODE == 2 ? a.stack_limit4b : a.stack_limit;
    // early shading (certified passes, es): the hit records start "not written yet", shading workgroups follow the walk's
    const bool early = RTBVH_EARLY_SHADE && MODE == 2 && cert && es;
    const uint32_t nshade = early ? (es->P + ESHADE_RAYS - 1) / ESHADE_RAYS : 0u;
    if (early) hipLaunchKernelGGL(k_hit_init, dim3(1024), dim3(BLOCK), 0, s, hitrec, qin_count);
#define RTBVH_BTE(L, G, C, E)                                                                                          \
    hipLaunchKernelGGL((k_bounce_trav<COUNT, MODE, L, G, C, E>), dim3(blocks + nshade), dim3(BLOCK), 0, s, a.inner,         \
                       a.qnode,                                                                                        \
                       a.leaf, a.T, qin, qin_count, perm, hitrec, next, a.counters, a.overflow, lim, defer, a.topo,    \
                       a.nb ? a.nbox : nullptr, blocks, a, early ? es->qout : nullptr, early ? es->qout_count : nullptr, \
                       early ? (int)es->emit : 0, early ? es->redo : nullptr, early ? es->redo_count : nullptr)
#define RTBVH_BT(L, G, C) RTBVH_BTE(L, G, C, false)
    // the guard only for a tree that may have cycles (CPUTests delta), or for COUNT's census
    const bool guard = COUNT || !a.acyclic;
    if (MODE == 2 && cert && early) {
        if (guard) RTBVH_BTE(false, true, MODE == 2, MODE == 2);
        else RTBVH_BTE(false, false, MODE == 2, MODE == 2);
    } else if (MODE == 2 && cert) {   // (the certified walk: no stack limit, a clz64 tree -- api.hip enqueue_trace)
        if (guard) RTBVH_BT(false, true, MODE == 2);
        else RTBVH_BT(false, false, MODE == 2);
    } else if (a.limited) { if (guard) RTBVH_BT(true, true, false); else RTBVH_BT(true, false, false); }
    else { if (guard) RTBVH_BT(false, true, false); else RTBVH_BT(false, false, false); }
#undef RTBVH_BT
#undef RTBVH_BTE
}

}  // namespace

void launch_primary(const TraceArgs& a, RayQ* q, uint32_t* qcount, bool count, bool emit, PrimaryKind kind,
                    hipStream_t s) {
    const uint32_t my_bands = a.my_bands;
    const uint32_t launch_bands = my_bands > a.band0 ? (my_bands - a.band0 + a.bstep - 1) / a.bstep : 0;
    if (launch_bands == 0 || a.W == 0) return;
    dim3 grid((a.W + 31) / 32, launch_bands);
    switch (kind) {
        case PrimaryKind::LANE_NEAREST: launch_primary_c<1>(a, q, qcount, count, emit, grid, s); break;
        case PrimaryKind::PACKET_REFERENCE: launch_primary_c<2>(a, q, qcount, count, emit, grid, s); break;
        case PrimaryKind::PACKET_NEAREST: launch_primary_c<3>(a, q, qcount, count, emit, grid, s); break;
        case PrimaryKind::PACKET_WIDE:
            if (a.acyclic) launch_primary_c<5>(a, q, qcount, count, emit, grid, s);
            else launch_primary_c<4>(a, q, qcount, count, emit, grid, s);
            break;
        default:   // LANE_REFERENCE: on the topology and node boxes when the trace says so (a certified one)
            if (a.nb) launch_primary_c<6>(a, q, qcount, count, emit, grid, s);
            else launch_primary_c<0>(a, q, qcount, count, emit, grid, s);
            break;
    }
}

void launch_zero(const ZeroList& z, hipStream_t s) {
    size_t most = 0;
    for (int k = 0; k < ZeroList::N; k++) most = most > z.words[k] ? most : z.words[k];
    if (most == 0) return;
    size_t blocks = (most + BLOCK - 1) / BLOCK;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_zero, dim3((uint32_t)blocks, ZeroList::N), dim3(BLOCK), 0, s, z);
}

void launch_pb_pass(const TraceArgs& a, const PrimBins& pb, uint32_t rows, RayQ* q, uint32_t* qcount, bool count,
                    bool emit, bool zeroed, hipStream_t s, const BuildArgs* tail, const Redo* redo, bool small_tiles) {
    if (rows == 0 || a.W == 0 || a.T == 0) return;
    const uint32_t keys = pb.ntx * pb.nty * PB_NZ;
    if (!zeroed) (void)hipMemsetAsync(pb.off, 0, ((size_t)keys + 1) * sizeof(uint32_t), s);
    if (!zeroed && a.pb_list) (void)hipMemsetAsync(a.pb_list, 0, (size_t)PB_LISTS * PB_LIST_STRIDE * sizeof(uint32_t), s);
    const dim3 lg((a.T + PB_LEAVES - 1) / PB_LEAVES);
    if (tail) launch_pb_count_top(*tail, a, pb.off, pb.cur, pb.bins, pb.cap, pb.ntx, lg.x, s);
    else hipLaunchKernelGGL((k_pb_bin<false>), lg, dim3(BLOCK), 0, s, a, pb.off, pb.cur, pb.bins, pb.cap, pb.ntx);
    const uint32_t sb = (keys + PB_SCAN - 1) / PB_SCAN;
    hipLaunchKernelGGL(k_pb_sums, dim3(sb), dim3(PB_SCAN), 0, s, pb.off, pb.sums, keys);
    hipLaunchKernelGGL(k_pb_scan, dim3(sb), dim3(PB_SCAN), 0, s, pb.off, pb.cur, pb.sums, keys);
    hipLaunchKernelGGL((k_pb_bin<true>), lg, dim3(BLOCK), 0, s, a, pb.off, pb.cur, pb.bins, pb.cap, pb.ntx);
    const dim3 grid(pb.ntx, pb.nty);
    uint32_t* rl = redo ? redo->list : nullptr;
    uint32_t* rc = redo ? redo->count : nullptr;
    const bool rec = a.refl_rec || a.refr_rec;
#define RTBVH_PBR(C, R, F)                                                                                          \
    do {                                                                                                            \
        if (rec || !(F))                                                                                            \
            hipLaunchKernelGGL((k_primary_binned<C, R, F, true>), grid, dim3(PB_RASTER_BLOCK), 0, s, a, pb.off,     \
                               pb.bins, pb.cap, pb.ntx, rows, pb.keys, q, qcount, (int)emit, rl, rc);               \
        else if (small_tiles)                                                                                       \
            hipLaunchKernelGGL((k_primary_binned<C, R, F, false, PB_RASTER_BLOCK_SMALL>), grid,                      \
                               dim3(PB_RASTER_BLOCK_SMALL), 0, s, a, pb.off, pb.bins, pb.cap, pb.ntx, rows, pb.keys, q, \
                               qcount, (int)emit, rl, rc);                                                          \
        else                                                                                                        \
            hipLaunchKernelGGL((k_primary_binned<C, R, F, false>), grid, dim3(PB_RASTER_BLOCK), 0, s, a, pb.off,    \
                               pb.bins, pb.cap, pb.ntx, rows, pb.keys, q, qcount, (int)emit, rl, rc);               \
    } while (0)
#define RTBVH_PBS(C, R)                                                                                              \
    hipLaunchKernelGGL((k_pb_shade<C, R>), grid, dim3(PB_SHADE_BLOCK), 0, s, a, pb.off, pb.cap, pb.ntx, rows, pb.keys, q, \
                       qcount, (int)emit, rl, rc)
#if RTBVH_PB_FUSE
    if (count) { if (redo) RTBVH_PBR(true, true, true); else RTBVH_PBR(true, false, true); }
    else { if (redo) RTBVH_PBR(false, true, true); else RTBVH_PBR(false, false, true); }
#else
    if (count) RTBVH_PBR(true, false, false); else RTBVH_PBR(false, false, false);
    if (count) { if (redo) RTBVH_PBS(true, true); else RTBVH_PBS(true, false); }
    else { if (redo) RTBVH_PBS(false, true); else RTBVH_PBS(false, false); }
#endif
#undef RTBVH_PBR
#undef RTBVH_PBS
    if (redo) {   // the flagged pixels, in the reference order
        const dim3 rg(REDO_BLOCKS);
        if (count) hipLaunchKernelGGL((k_primary_redo<true>), rg, dim3(BLOCK), 0, s, a, rl, rc, q, qcount, (int)emit);
        else hipLaunchKernelGGL((k_primary_redo<false>), rg, dim3(BLOCK), 0, s, a, rl, rc, q, qcount, (int)emit);
    }
}

void launch_pb_gate(const TraceArgs& a, const PrimBins& pb, RayQ* q, uint32_t* qcount, bool count, bool emit,
                    hipStream_t s, bool reference) {
    if (a.W == 0 || a.T == 0) return;
    // the tiles whose bins overflowed: the per-lane nearest-first walk (every other block returns at
    // once); a binary walk, which reads no leaf pseudo-records (a binned build writes none).  A certified
    // trace takes the reference order there (exact by construction)
    TraceArgs g = a;
    g.pb_gate = pb.off;
    g.pb_cap = pb.cap;
    g.pb_ntx = pb.ntx;
    launch_primary(g, q, qcount, count, emit, reference ? PrimaryKind::LANE_REFERENCE : PrimaryKind::LANE_NEAREST, s);
}

void launch_primary_binned(const TraceArgs& a, const PrimBins& pb, uint32_t rows, RayQ* q, uint32_t* qcount,
                           bool count, bool emit, bool zeroed, hipStream_t s) {
    if (rows == 0) return;
    launch_pb_pass(a, pb, rows, q, qcount, count, emit, zeroed, s);
    launch_pb_gate(a, pb, q, qcount, count, emit, s, false);
}

void launch_bounce(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const uint32_t* perm, RayQ* qout,
                   uint32_t* qout_count, bool count, bool emit, bool nearest, hipStream_t s) {
    const uint32_t blocks = 2048;   // 8 waves/SIMD x 1024 SIMDs / 4 waves per block; grid-stride over the queue
#define RTBVH_BNC(C, N)                                                                                          \
    do {                                                                                                           \
        if (a.limited)                                                                                             \
            hipLaunchKernelGGL((k_bounce<C, N, true>), dim3(blocks), dim3(BLOCK), 0, s, a, qin, qin_count, perm, qout, \
                               qout_count, (int)emit);                                                           \
        else                                                                                                       \
            hipLaunchKernelGGL((k_bounce<C, N, false>), dim3(blocks), dim3(BLOCK), 0, s, a, qin, qin_count, perm,     \
                               qout, qout_count, (int)emit);                                                     \
    } while (0)
    if (count) { if (nearest) RTBVH_BNC(true, true); else RTBVH_BNC(true, false); }
    else { if (nearest) RTBVH_BNC(false, true); else RTBVH_BNC(false, false); }
#undef RTBVH_BNC
}

void launch_bounce_keys(const RayQ* q, const uint32_t* count, const float* box, uint32_t P, uint32_t* keys,
                        uint32_t* vals, hipStream_t s) {
    hipLaunchKernelGGL(k_bounce_keys, dim3((P + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, q, count, box, P, keys, vals);
}

void launch_bounce_traverse(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const uint32_t* perm,
                            bool count, BounceWalk walk, float2* hitrec, uint32_t* next, uint32_t blocks,
                            hipStream_t s, bool cert, uint32_t* defer, const BounceShade* es) {
    if (blocks == 0) blocks = 2048;
#define RTBVH_TRAV(C, M) launch_bounce_trav_t<C, M>(a, qin, qin_count, perm, hitrec, next, blocks, cert, defer, s, es)
    switch (walk) {
        case BounceWalk::NEAREST: if (count) RTBVH_TRAV(true, 1); else RTBVH_TRAV(false, 1); break;
        case BounceWalk::WIDE_QUANTIZED: if (count) RTBVH_TRAV(true, 2); else RTBVH_TRAV(false, 2); break;
        default: if (count) RTBVH_TRAV(true, 0); else RTBVH_TRAV(false, 0); break;
    }
#undef RTBVH_TRAV
}

void launch_bounce_shade(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const float2* hitrec,
                         RayQ* qout, uint32_t* qout_count, bool count, bool emit, uint32_t P, hipStream_t s,
                         const Redo* redo) {
    if (P == 0) return;
    uint32_t* rl = redo ? redo->list : nullptr;
    uint32_t* rc = redo ? redo->count : nullptr;
    const dim3 g((P + BLOCK - 1) / BLOCK);
#define RTBVH_BS(C, R)                                                                                             \
    hipLaunchKernelGGL((k_bounce_shade<C, R>), g, dim3(BLOCK), 0, s, a, qin, qin_count, hitrec, qout, qout_count, \
                       (int)emit, rl, rc)
    if (count) { if (redo) RTBVH_BS(true, true); else RTBVH_BS(true, false); }
    else { if (redo) RTBVH_BS(false, true); else RTBVH_BS(false, false); }
#undef RTBVH_BS
    if (redo) {   // the flagged rays (and the walk's deferred rays left over), in the reference order
        if (count) hipLaunchKernelGGL((k_bounce_redo<true>), dim3(REDO_BLOCKS), dim3(BLOCK), 0, s, a, qin, rl, rc, qout,
                                      qout_count, (int)emit, redo->defer, redo->dnext);
        else hipLaunchKernelGGL((k_bounce_redo<false>), dim3(REDO_BLOCKS), dim3(BLOCK), 0, s, a, qin, rl, rc, qout,
                                qout_count, (int)emit, redo->defer, redo->dnext);
    }
}

void launch_assemble(const float4* bands, const uint32_t* slots, uint32_t stride_rows, uint32_t W, uint32_t H,
                     uint32_t nranks, float4* frame, hipStream_t s) {
    const size_t n = (size_t)W * H;
    hipLaunchKernelGGL(k_assemble, dim3((uint32_t)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, bands, slots,
                       stride_rows, W, H, nranks, frame);
}

void launch_present(const float4* color, uint32_t W, uint32_t H, uint32_t* out, hipStream_t s) {
    const size_t n = (size_t)W * H;
    if (n) hipLaunchKernelGGL(k_present, dim3((uint32_t)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, color, W, H, out);
}

// the camera upload (sync_camera): the 32 floats travel as the kernel's by-value argument, so the copy is
// one dispatch in stream order -- no DMA engine, no staging of the pageable host matrices
__global__ __launch_bounds__(64) void k_set_camera(CameraWords m, float* __restrict__ cam) {
    if (threadIdx.x < 32) cam[threadIdx.x] = m.w[threadIdx.x];
}

void launch_set_camera(const float* wvp, const float* wv, float* cam, hipStream_t s) {
    CameraWords m;
    for (int i = 0; i < 16; i++) {
        m.w[i] = wvp[i];
        m.w[16 + i] = wv[i];
    }
    hipLaunchKernelGGL(k_set_camera, dim3(1), dim3(64), 0, s, m, cam);
}

void launch_count_diff(const float4* a, const float4* b, size_t n, unsigned long long* diff, hipStream_t s) {
    if (n == 0) return;
    size_t blocks = (n + BLOCK - 1) / BLOCK;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_count_diff, dim3((uint32_t)blocks), dim3(BLOCK), 0, s, reinterpret_cast<const uint4*>(a),
                       reinterpret_cast<const uint4*>(b), n, diff);
}

void launch_count_diff32(const float* a, const float* b, size_t n, unsigned long long* diff, hipStream_t s) {
    if (n == 0) return;
    size_t blocks = (n + BLOCK - 1) / BLOCK;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_count_diff32, dim3((uint32_t)blocks), dim3(BLOCK), 0, s, reinterpret_cast<const uint32_t*>(a),
                       reinterpret_cast<const uint32_t*>(b), n, diff);
}

}  // namespace rtbvh
