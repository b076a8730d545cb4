// margin.h -- the rounding margin of Moller-Trumbore (rayTriangleCollision, RayTraceTraversal.hlsl:41-86)
// that makes the certified walks exhaustive ("The per-ray certificate").  Shared by the
// kernels (build.hip: the primary rays' depth keys; trace.hip: the bounce walk's expanded entries) and
// the CPU checker tools/margin_check.cpp, so the checker tests these very functions.
//
// The bound.  Let the float test accept (o, d; p0, e1 = RN(p1 - p0), e2 = RN(p2 - p0)) with |det| >= 0.01
// and return t.  Then the real point o + t d lies within
//     rho(t) = 35.4 u L A E^2 (A t + 1.31 E) + u (4 A t + 6 E)           (u = 2^-24)
// (2-norm) of the triangle conv(p0, p1, p2), hence of every box that contains the triangle, where
// E >= max(|e1|, |e2|), A >= |d|, L >= 1 / |det|, provided (C): 28.3 L A u E (A t + 2 E) <= 0.2.
// (Forward error analysis of each dot and cross product, gamma_n bounds, the computed u, v, t against
// Cramer's rule on the same float inputs; DESIGN.md 3 has the steps.)  Everything below rounds that
// bound UP: the 1.01 factor covers the roundings of computing and applying it.
#pragma once
#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define RTBVH_HD __host__ __device__
#else
#define RTBVH_HD
#endif

namespace rtbvh {

constexpr float MT_U = 0x1p-24f;
constexpr float MT_LAMBDA = 100.01f;        // >= 1 / |det| of any accepted test: |det| >= EPSILON = 0.01f
constexpr float MT_A = 1.f + 0x1p-18f;      // >= |d| of a ray whose d.d <= MT_DD (bounce rays are normalized)
constexpr float MT_DD = 1.f + 0x1p-18f;
constexpr float MT_FLOOR = 1e-37f;          // absolute floor: the gradual-underflow terms of the products

// rho(t) = r1 * t + r0, valid for t <= tcap (condition (C)); tcap < 0: no t is covered
struct MtMargin {
    float r1, r0, tcap;
};
RTBVH_HD inline MtMargin mt_margin(float E, float L, float A) {
    MtMargin m;
    const float K = 35.4f * MT_U * L * A * E * E;   // (underflow only drops terms the 1.01 covers)
    m.r1 = 1.01f * A * (K + 4.f * MT_U);
    m.r0 = 1.01f * E * (1.31f * K + 6.f * MT_U) + MT_FLOOR;
    // (C): c (A t + 2 E) <= 0.2 with c = 28.3 L A u E; for a tiny E the product c is formed on E 2^64 and
    // 0.2 / c scaled back (powers of two: exact), so neither c's gradual underflow nor 0.2 / c's overflow
    // moves the range up (capped at 2^127: below the true range when that is past the float range)
    const bool tiny = E < 0x1p-60f;
    const float c = 28.3f * L * A * MT_U * (tiny ? E * 0x1p64f : E);
    const float r = tiny ? fminf(0.2f / c * 0x1p64f, 0x1p127f) : 0.2f / c;
    m.tcap = c > 0.f ? (r - 2.f * E) / A * 0.999f : INFINITY;
    if (!(E >= 0.f && E < INFINITY && m.r1 < 0.5f && m.r0 < INFINITY)) m.tcap = -1.f;   // (NaN: not covered)
    return m;
}

// ---- per-node margins (the certified bounce walk) ----------------------------------------
// rho grows with E and tcap falls with it, so a box may use the largest edge bound E_n of the leaves BELOW
// it instead of the scene's: every candidate x in the box has E_x <= E_n, hence rho_x(t) <= rho_n(t) and
// tcap(E_x) >= tcap(E_n).  Each QNode carries its subtree's E_n (rounded up) and tcap(E_n) (rounded down)
// as 16-bit codes (the high half of an fp32) in the low bits of its scl[1] / scl[2] words -- the grid steps
// are powers of two, their mantissas are otherwise zero (build.hip qnode_words).  The walk grows the node's
// boxes by
//     rho_n(t) = E_n^2 (P t + Q E_n) + U1 t + U0 E_n + FLOOR      (>= mt_margin(E_n).r1 t + r0)
// and never prunes a box by distance once its bound passes tcap(E_n) (the box's key is capped there).
RTBVH_HD inline uint32_t mt_f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
RTBVH_HD inline float mt_u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
RTBVH_HD inline uint32_t mt_code_up(float x) { return (mt_f2u(x) + 0xFFFFu) >> 16; }   // x >= 0: decodes >= x
RTBVH_HD inline uint32_t mt_code_down(float x) { return x >= 0.f ? mt_f2u(x) >> 16 : 0xBF80u; }   // <= x; -1
RTBVH_HD inline float mt_code_val(uint32_t w) { return mt_u2f(w << 16); }   // (the low 16 bits of w)
// 1 / x rounded down (x > 0 finite): the hardware reciprocal (within 1 ulp) on the device, the division
// on the host, either times 1 - 2^-21
RTBVH_HD inline float mt_rcp_down(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x) * (1.f - 0x1p-21f);
#else
    return 1.f / x * (1.f - 0x1p-21f);
#endif
}
// tcap of mt_margin(E, MT_LAMBDA, MT_A) from below, without a division (the build quantizes a node per thread).
// A tiny E is scaled as in mt_margin: c on E 2^64 (no gradual underflow of c, which would round it DOWN and
// the range up), 0.2 / c scaled back and capped at 2^127 (no overflow to inf past the true range)
RTBVH_HD inline float mt_tcap_down(float E) {
    if (!(E >= 0.f && E < INFINITY)) return -1.f;
    const bool tiny = E < 0x1p-60f;
    const float c = 28.3f * MT_LAMBDA * MT_A * MT_U * (tiny ? E * 0x1p64f : E) * (1.f + 0x1p-20f);   // >= mt_margin's c
    if (!(c > 0.f)) return INFINITY;
    const float q = 0.2f * mt_rcp_down(c);
    const float r = tiny ? fminf(q * 0x1p64f, 0x1p127f) : q;
    return (r - 2.f * E * (1.f + 0x1p-20f)) * ((1.f - 0x1p-20f) / MT_A) * 0.999f;
}
// a node's codes from the largest edge bound of its leaves (inf: a non-finite triangle below; tcap -1)
RTBVH_HD inline void mt_node_codes(float E, uint32_t& ce, uint32_t& ct) {
    ce = mt_code_up(E >= 0.f ? E : INFINITY);   // (NaN: inf)
    // (mt_margin's other conditions, r1 < 0.5 and r0 finite, hold for every E whose tcap is >= 0: E < ~24)
    ct = mt_code_down(mt_tcap_down(mt_code_val(ce)));
}
struct MtNodeK {
    float P, Q, U1, U0;
};
// the coefficients of rho_n for the bounce walk (L = MT_LAMBDA, A = MT_A), each rounded up past the few
// roundings of evaluating rho_n (the 1.01 of mt_margin already covers computing and applying the bound)
RTBVH_HD inline MtNodeK mt_node_consts() {
    constexpr float up = 1.f + 0x1p-18f;
    MtNodeK k;
    k.P = 1.01f * 35.4f * MT_U * MT_LAMBDA * MT_A * MT_A * up;
    k.Q = 1.01f * 1.31f * 35.4f * MT_U * MT_LAMBDA * MT_A * up;
    k.U1 = 4.04f * MT_U * MT_A * up;
    k.U0 = 6.06f * MT_U * up;
    return k;
}
// rho_n(t) as the walk evaluates it: per node the line rho_n(t) = s t + c, s = E^2 P + U1, c = E^2 Q E + U0 E
// + FLOOR (each a few roundings, inside the constants' margin), then one fma per bound t
struct MtNodeRho {
    float s, c;
};
RTBVH_HD inline MtNodeRho mt_node_prep(const MtNodeK& k, float E) {
    const float E2 = E * E;
    return MtNodeRho{fmaf(E2, k.P, k.U1), fmaf(E2, k.Q * E, fmaf(k.U0, E, MT_FLOOR))};
}
RTBVH_HD inline float mt_node_eval(const MtNodeRho& n, float t) { return fmaf(n.s, t, n.c); }
RTBVH_HD inline float mt_node_rho(const MtNodeK& k, float E, float t) { return mt_node_eval(mt_node_prep(k, E), t); }

// the global edge bound of a triangle: max(|e1|, |e2|) rounded up (inf for a non-finite triangle).  Below
// 2^-50 a component's square can underflow (to a denormal that rounds by more than the 2^-20, or to 0): then
// the bound is sqrt(3) max |component|, rounded up, plus the smallest denormal (E >= |e| must hold
// for the tiniest triangles too)
RTBVH_HD inline float mt_edge_bound(float e1x, float e1y, float e1z, float e2x, float e2y, float e2z) {
    const float a = e1x * e1x + e1y * e1y + e1z * e1z, b = e2x * e2x + e2y * e2y + e2z * e2z;
    const float m = sqrtf(fmaxf(a, b)) * (1.f + 0x1p-20f);
    if (m != m) return INFINITY;
    const float mx = fmaxf(fmaxf(fmaxf(fabsf(e1x), fabsf(e1y)), fmaxf(fabsf(e1z), fabsf(e2x))),
                           fmaxf(fabsf(e2y), fabsf(e2z)));
    if (mx < 0x1p-50f) return mx * 1.7320510f * (1.f + 0x1p-20f) + 0x1p-149f;
    return m;
}

// The depth key of a leaf for the orthographic primary rays (d = (0, 0, 1), so |d| = 1 and the
// determinant of the test, `dx` as the kernels compute it for that d, is the same for every pixel):
// every pixel ray whose test accepts this triangle returns t >= the key.  +inf when no primary ray
// can be accepted (|dx| < 0.01, or NaN), -inf when no bound is available (the leaf is never pruned).
RTBVH_HD inline float mt_primary_zkey(float dx, float E, float lo_z, float hi_z) {
    if (!(fabsf(dx) >= 0.01f)) return INFINITY;
    if (!(fabsf(lo_z) < INFINITY && fabsf(hi_z) < INFINITY && E < INFINITY)) return -INFINITY;
    const float L = 1.f / fabsf(dx) * (1.f + 0x1p-20f);
    const MtMargin m = mt_margin(E, L, 1.f);
    // a candidate's t lies within rho(t) of [lo_z, hi_z] (its point is (o.x, o.y, t)): t <= th
    const float th = (fmaxf(hi_z, 0.f) + m.r0) / (1.f - m.r1) * (1.f + 0x1p-20f);
    if (!(th <= m.tcap)) return -INFINITY;
    const float rho = (m.r1 * th + m.r0) * (1.f + 0x1p-20f);
    return nextafterf(lo_z - rho, -INFINITY);   // below the rounded difference
}

}  // namespace rtbvh
