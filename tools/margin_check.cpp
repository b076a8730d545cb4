// margin_check -- randomized check, on the CPU, of the rounding margin behind the certified walks
// (raytracebvh_amd/csrc/margin.h; DESIGN.md 3 "The per-ray certificate").
//
// For random rays and triangles -- C5-like scenes, grazing rays whose determinant sits just above the
// 0.01 rejection, flat (axis-plane) and coplanar triangles, near-edge and near-vertex hits, the
// orthographic primary rays, several magnitude regimes -- every test that Moller-Trumbore accepts
// (the fp32 arithmetic of trace.hip ray_triangle_flat, RayTraceTraversal.hlsl:41-86) must satisfy:
//  * dist: the real point o + t d lies within rho(t) of the triangle's box (margin.h mt_margin, with the
//    triangle's own edge bound and L = 100.01 as the walk uses, and with L = 1/|det| as the build uses);
//  * walk: the bounce walk's expanded slack test (trace.hip qaxis with the margin, qbox_fast) on a
//    quantized box containing the triangle passes at any bound best >= t, whenever the exact box passes
//    the reference slab test -- so the certified walk never prunes a box holding a hit it must see;
//  * zkey: for the primary rays, the leaf's depth key (margin.h mt_primary_zkey) is <= t;
//  * node: the per-node margin of the certified bounce walk (margin.h mt_node_codes / mt_node_rho, round 5):
//    for a node whose leaves' largest edge bound E_n >= the triangle's own, the decoded E_n >= E_n, the
//    decoded range tcap_n <= mt_margin(E_n).tcap, rho_n(t) >= mt_margin(E_n)'s rho(t) at every t <= tcap_n,
//    and the real point lies within rho_n(t) of the box whenever t <= tcap_n; and the walk's expanded
//    slack test with the node's margin at any bound best in [t, tcap_n] passes.
// Restates the device arithmetic with the same fp32 operations (-ffp-contract=off).  Reports the worst
// ratio of the real distance to the margin (how tight the bound is).  Built with -DMARGIN_SCALE=1e-3f
// (a margin 1000x too small) it must find violations: the check bites.  Used by tests/test_margin.py.
//   g++ -O2 -ffp-contract=off -I../raytracebvh_amd/csrc -o margin_check margin_check.cpp && ./margin_check 1000000 1
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "margin.h"

#ifndef MARGIN_SCALE
#define MARGIN_SCALE 1.0f
#endif

using namespace rtbvh;

namespace {

float bits_f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
uint32_t f_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

struct Rng {   // splitmix64
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double u01() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double ud(double lo, double hi) { return lo + (hi - lo) * u01(); }
};

struct V { float x, y, z; };
V mk(float x, float y, float z) { return V{x, y, z}; }
V sub(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

// trace.hip ray_triangle_flat (the reference's accept predicate and floats); dx out
float ray_triangle(V o, V d, V p0, V e1, V e2, float& dx) {
    const V tmp = cross(d, e2);
    dx = dot(e1, tmp);
    const float idx = 1.f / dx;
    const V rt = sub(o, p0);
    const float u = dot(rt, tmp) * idx;
    const V q = cross(rt, e1);
    const float v = dot(d, q) * idx;
    const float t = dot(e2, q) * idx;
    float r = 0.01f < t ? t : -1.f;
    if (fabsf(dx) < 0.01f || u < 0.f || 1.f < u || v < 0.f || 1.f < u + v) r = -1.f;
    return r;
}

// trace.hip ray_box (fminf / fmaxf drop NaN), no bound
bool slab(const float o[3], const float inv[3], const float lo[3], const float hi[3]) {
    float mn = 0, mx = 0;
    for (int a = 0; a < 3; a++) {
        const float t0 = (lo[a] - o[a]) * inv[a], t1 = (hi[a] - o[a]) * inv[a];
        const float n = fminf(t0, t1), x = fmaxf(t0, t1);
        mn = a == 0 ? n : fmaxf(mn, n);
        mx = a == 0 ? x : fminf(mx, x);
    }
    return 0 <= mx && mn <= mx;
}

// build.hip quantize_axis (as tools/slack_check.cpp)
float pow2f(int e) { return bits_f((uint32_t)(e + 127) << 23); }
bool quantize_axis(const float lo[4], const float hi[4], float& org, float& scl, uint32_t q_lo[4], uint32_t q_hi[4]) {
    float o = lo[0], m = hi[0];
    for (int c = 1; c < 4; c++) { o = fminf(o, lo[c]); m = fmaxf(m, hi[c]); }
    const float ext = m - o;
    if (!(fabsf(o) <= 0x1p100f && fabsf(m) <= 0x1p100f && ext <= 0x1p100f)) return false;
    int e = -120;
    if (ext > 0.f) {
        const int E = (int)((f_bits(ext) >> 23) & 255u) - 127;
        e = E - 8 > -120 ? E - 8 : -120;
    }
    while (fmaf(255.f, pow2f(e), o) < m) ++e;
    const float s = pow2f(e), rs = pow2f(-e);
    for (int c = 0; c < 4; c++) {
        uint32_t l = (uint32_t)fminf(fmaxf(floorf((lo[c] - o) * rs), 0.f), 255.f);
        uint32_t h = (uint32_t)fminf(fmaxf(ceilf((hi[c] - o) * rs), 0.f), 255.f);
        if (l > 0 && fmaf((float)l, s, o) > lo[c]) --l;
        if (h < 255 && fmaf((float)h, s, o) < hi[c]) ++h;
        q_lo[c] = l;
        q_hi[c] = h;
    }
    org = o;
    scl = s;
    return true;
}

// trace.hip qnode_fast_ray, qaxis (certified: the near side widened by the margin rr), qbox_fast
bool fast_ray(const float o[3], const float inv[3]) {
    const float mi = fmaxf(fmaxf(fabsf(inv[0]), fabsf(inv[1])), fabsf(inv[2]));
    const float mo = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fabsf(o[2]));
    return mi <= 0x1p20f && mo <= 0x1p90f;
}
struct QAxis { uint32_t nw, fw; float b, an, af; };
QAxis qaxis(float org, float scl, uint32_t lw, uint32_t hw, float o, float inv, float rr) {
    QAxis r;
    const bool neg = inv < 0.f;
    r.nw = neg ? hw : lw;
    r.fw = neg ? lw : hw;
    const float m = fmaf(scl, 256.f, fabsf(org) + fabsf(o));
    const float e = m * fabsf(inv);
    const float a = (org - o) * inv;
    const float mn = fmaf(m, 0x1p-20f, rr);
    r.an = fmaf(-mn, fabsf(inv), a);
    r.af = fmaf(e, 0x1p-20f, a);
    r.b = scl * inv;
    return r;
}
float qt(uint32_t w, int c, float b, float a) { return fmaf((float)((w >> (8 * c)) & 255u), b, a); }
bool qbox_fast(const QAxis& x, const QAxis& y, const QAxis& z, int c, float best) {
    const float mn = fmaxf(fmaxf(qt(x.nw, c, x.b, x.an), qt(y.nw, c, y.b, y.an)), qt(z.nw, c, z.b, z.an));
    const float mx = fminf(fminf(qt(x.fw, c, x.b, x.af), qt(y.fw, c, y.b, y.af)), qt(z.fw, c, z.b, z.af));
    return 0 <= mx && mn <= mx && mn <= best;
}

// unit direction (float), optionally close to a plane with normal n (|d . n| ~ g)
V unit(double x, double y, double z) {
    const double n = std::sqrt(x * x + y * y + z * z);
    return mk((float)(x / n), (float)(y / n), (float)(z / n));
}

struct Stats {
    long tests = 0, accepted = 0, dist_checked = 0, dist_viol = 0, dist_viol_tight = 0, walk_checked = 0,
         walk_viol = 0, zkey_checked = 0, zkey_viol = 0, uncovered = 0, node_checked = 0, node_viol = 0,
         node_walk_checked = 0, node_walk_viol = 0;
    double max_ratio = 0, max_ratio_tight = 0;
};

// real distance (inf-norm) of o + t d from the box [lo, hi]
long double box_dist(V o, V d, float t, const float lo[3], const float hi[3]) {
    const long double p[3] = {(long double)o.x + (long double)t * d.x, (long double)o.y + (long double)t * d.y,
                              (long double)o.z + (long double)t * d.z};
    long double m = 0;
    for (int a = 0; a < 3; a++) {
        long double q = 0;
        if (p[a] < lo[a]) q = lo[a] - p[a];
        else if (p[a] > hi[a]) q = p[a] - hi[a];
        if (q > m) m = q;
    }
    return m;
}

void check(Stats& s, Rng& rng, V o, V d, V p0, V p1, V p2, bool primary) {
    const V e1 = sub(p1, p0), e2 = sub(p2, p0);
    float dx;
    ++s.tests;
    const float t = ray_triangle(o, d, p0, e1, e2, dx);
    if (t == -1.f) return;
    ++s.accepted;
    const float lo[3] = {fminf(fminf(p0.x, p1.x), p2.x), fminf(fminf(p0.y, p1.y), p2.y), fminf(fminf(p0.z, p1.z), p2.z)};
    const float hi[3] = {fmaxf(fmaxf(p0.x, p1.x), p2.x), fmaxf(fmaxf(p0.y, p1.y), p2.y), fmaxf(fmaxf(p0.z, p1.z), p2.z)};
    const float E = mt_edge_bound(e1.x, e1.y, e1.z, e2.x, e2.y, e2.z);
    const float dd = dot(d, d);
    const long double dist = box_dist(o, d, t, lo, hi);
    // the walk's margin (L = 100.01, A = MT_A): the bounce rays
    if (dd <= MT_DD) {
        const MtMargin m = mt_margin(E, MT_LAMBDA, MT_A);
        if (t <= m.tcap) {
            const float rho = (m.r1 * t + m.r0) * MARGIN_SCALE;
            ++s.dist_checked;
            const double ratio = (double)(dist / (long double)rho);
            if (ratio > s.max_ratio) s.max_ratio = ratio;
            if (dist > rho) ++s.dist_viol;
            // the walk's expanded test on a quantized node whose child 0 is this box (the others random)
            const float o3[3] = {o.x, o.y, o.z};
            const float inv[3] = {1.f / d.x, 1.f / d.y, 1.f / d.z};
            if (fast_ray(o3, inv) && slab(o3, inv, lo, hi)) {
                float clo[3][4], chi[3][4], org[3], scl[3];
                uint32_t ql[3][4], qh[3][4];
                bool ok = true;
                for (int a = 0; a < 3; a++) {
                    clo[a][0] = lo[a];
                    chi[a][0] = hi[a];
                    for (int c = 1; c < 4; c++) {
                        const float w = (hi[a] - lo[a]) + 1.f;
                        const float u0 = lo[a] + (float)rng.ud(-4.0, 4.0) * w, u1 = u0 + (float)rng.u01() * w;
                        clo[a][c] = u0;
                        chi[a][c] = u1;
                    }
                    ok = quantize_axis(clo[a], chi[a], org[a], scl[a], ql[a], qh[a]) && ok;
                }
                if (ok) {
                    uint32_t lw[3] = {0, 0, 0}, hw[3] = {0, 0, 0};
                    for (int a = 0; a < 3; a++)
                        for (int c = 0; c < 4; c++) { lw[a] |= ql[a][c] << (8 * c); hw[a] |= qh[a][c] << (8 * c); }
                    // the walk's bound: best >= t (the hit itself, or a worse one found first)
                    const float best = rng.next() % 2 ? t : t * (float)(1.0 + rng.u01());
                    if (best <= m.tcap) {
                        const float rr = (m.r1 * best + m.r0) * MARGIN_SCALE;
                        const QAxis X = qaxis(org[0], scl[0], lw[0], hw[0], o.x, inv[0], rr);
                        const QAxis Y = qaxis(org[1], scl[1], lw[1], hw[1], o.y, inv[1], rr);
                        const QAxis Z = qaxis(org[2], scl[2], lw[2], hw[2], o.z, inv[2], rr);
                        ++s.walk_checked;
                        if (!qbox_fast(X, Y, Z, 0, best)) ++s.walk_viol;
                    }
                }
            }
        } else {
            ++s.uncovered;
        }
    }
    // the per-node margin: a node above this triangle, whose largest edge bound is E or larger
    if (dd <= MT_DD) {
        const float En = rng.next() % 3 ? E : E * (float)(1.0 + 3.0 * rng.u01());
        uint32_t ce, ct;
        mt_node_codes(En, ce, ct);
        const float Eq = mt_code_val(ce), tcn = mt_code_val(ct);
        const MtMargin mn = mt_margin(En, MT_LAMBDA, MT_A);
        const MtNodeK nk = mt_node_consts();
        ++s.node_checked;
        // (a negative range covers no t > EPSILON either way: the codes keep -1)
        bool bad = !(Eq >= En) || !(tcn <= mn.tcap || (tcn < 0.f && mn.tcap < 0.f));
        if (t <= tcn) {
            const float rn = mt_node_rho(nk, Eq, t) * MARGIN_SCALE;
            if (!(rn >= mn.r1 * t + mn.r0) && MARGIN_SCALE == 1.0f) bad = true;
            if (dist > rn) bad = true;
            // the walk's expanded test with the node's margin at a bound best in [t, tcap_n]
            const float o3[3] = {o.x, o.y, o.z};
            const float inv[3] = {1.f / d.x, 1.f / d.y, 1.f / d.z};
            if (fast_ray(o3, inv) && slab(o3, inv, lo, hi)) {
                float org[3], scl[3];
                uint32_t lw[3] = {0, 0, 0}, hw[3] = {0, 0, 0};
                bool ok = true;
                for (int a = 0; a < 3; a++) {
                    float clo[4] = {lo[a], lo[a], lo[a], lo[a]}, chi[4] = {hi[a], hi[a], hi[a], hi[a]};
                    const float w = (hi[a] - lo[a]) + 1.f;
                    clo[3] = lo[a] - (float)rng.u01() * 8.f * w;   // a sibling stretching the grid
                    uint32_t ql[4], qh[4];
                    ok = quantize_axis(clo, chi, org[a], scl[a], ql, qh) && ok;
                    for (int c = 0; c < 4; c++) { lw[a] |= ql[c] << (8 * c); hw[a] |= qh[c] << (8 * c); }
                }
                float best = rng.next() % 2 ? t : t * (float)(1.0 + rng.u01());
                if (ok && best <= tcn) {
                    const float rr = mt_node_rho(nk, Eq, best) * MARGIN_SCALE;
                    const QAxis X = qaxis(org[0], scl[0], lw[0], hw[0], o.x, inv[0], rr);
                    const QAxis Y = qaxis(org[1], scl[1], lw[1], hw[1], o.y, inv[1], rr);
                    const QAxis Z = qaxis(org[2], scl[2], lw[2], hw[2], o.z, inv[2], rr);
                    ++s.node_walk_checked;
                    if (!qbox_fast(X, Y, Z, 0, best)) ++s.node_walk_viol;
                }
            }
        }
        if (bad) ++s.node_viol;
    }
    // the build's per-triangle margin (L = 1/|det|): the primary rays' depth keys
    {
        const float L = 1.f / fabsf(dx) * (1.f + 0x1p-20f);
        const MtMargin m = mt_margin(E, L, dd <= MT_DD ? MT_A : sqrtf(dd) * 1.001f);
        if (t <= m.tcap) {
            const float rho = (m.r1 * t + m.r0) * MARGIN_SCALE;
            const double ratio = (double)(dist / (long double)rho);
            if (ratio > s.max_ratio_tight) s.max_ratio_tight = ratio;
            if (dist > rho) ++s.dist_viol_tight;
        }
    }
    if (primary) {
        float zk = mt_primary_zkey(dx, E, lo[2], hi[2]);
        if (zk > -INFINITY && zk < INFINITY && MARGIN_SCALE != 1.0f) zk = lo[2] - (lo[2] - zk) * MARGIN_SCALE;
        ++s.zkey_checked;
        if (!(zk <= t)) ++s.zkey_viol;
    }
}

double scale_of(Rng& r) {
    switch (r.next() % 6) {
        case 0: return 1.0;
        case 1: return 4.0;
        case 2: return 0.05;
        case 3: return std::ldexp(1.0, (int)(r.next() % 16) - 8);
        default: return 1.0;
    }
}

}  // namespace

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    Rng rng{argc > 2 ? (uint64_t)atoll(argv[2]) : 1};
    Stats s;
    for (long it = 0; it < n; it++) {
        const int regime = (int)(rng.next() % 6);
        const double sc = scale_of(rng);
        // a triangle: C5-like clip-space offsets, scaled; flat in one axis now and then
        const double cx = rng.ud(-400, 400), cy = rng.ud(-250, 250), cz = rng.ud(1, 250);
        double v[3][3];
        for (int k = 0; k < 3; k++) {
            v[k][0] = cx + sc * 4.29 * rng.ud(-0.5, 0.5);
            v[k][1] = cy + sc * 2.41 * rng.ud(-0.5, 0.5);
            v[k][2] = cz + sc * 1.0 * rng.ud(-0.5, 0.5);
        }
        if (regime == 2) {   // flat: a plane of constant x, y or z (boxes with a zero extent)
            const int ax = (int)(rng.next() % 3);
            for (int k = 1; k < 3; k++) v[k][ax] = v[0][ax];
        }
        if (regime == 5) {   // large triangles (edges of tens of units)
            for (int k = 1; k < 3; k++)
                for (int a = 0; a < 3; a++) v[k][a] = v[0][a] + rng.ud(-12, 12);
        }
        const V p0 = mk((float)v[0][0], (float)v[0][1], (float)v[0][2]);
        const V p1 = mk((float)v[1][0], (float)v[1][1], (float)v[1][2]);
        const V p2 = mk((float)v[2][0], (float)v[2][1], (float)v[2][2]);
        // a point on (or just off) the triangle: barycentrics near an edge or a vertex now and then
        for (int k = 0; k < 6; k++) {
            double a = rng.u01(), b = rng.u01();
            if (a + b > 1) { a = 1 - a; b = 1 - b; }
            const uint64_t pick = rng.next() % 4;
            if (pick == 0) a = rng.ud(-1e-6, 1e-6);
            else if (pick == 1) b = 1 - a + rng.ud(-1e-6, 1e-6);
            const double X[3] = {v[0][0] + a * (v[1][0] - v[0][0]) + b * (v[2][0] - v[0][0]),
                                 v[0][1] + a * (v[1][1] - v[0][1]) + b * (v[2][1] - v[0][1]),
                                 v[0][2] + a * (v[1][2] - v[0][2]) + b * (v[2][2] - v[0][2])};
            if (regime == 4) {   // the orthographic primary rays: o on the quarter-pixel grid, d = +z
                const V o = mk((float)(std::floor(X[0] * 4.0 + rng.ud(-1, 1)) / 4.0),
                               (float)(std::floor(X[1] * 4.0 + rng.ud(-1, 1)) / 4.0), 0.f);
                check(s, rng, o, mk(0.f, 0.f, 1.f), p0, p1, p2, true);
                continue;
            }
            // direction: random, or grazing (|d . n| just above what |det| >= 0.01 allows)
            const double e1[3] = {v[1][0] - v[0][0], v[1][1] - v[0][1], v[1][2] - v[0][2]};
            const double e2[3] = {v[2][0] - v[0][0], v[2][1] - v[0][1], v[2][2] - v[0][2]};
            double nn[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            const double nl = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
            V d;
            if (regime == 1 || regime == 3 || (regime == 2 && rng.next() % 2)) {
                // in-plane direction + a small normal part: |det| = |n| |d . n^| in [0.01, 0.05]
                double w[3] = {rng.u01() - 0.5, rng.u01() - 0.5, rng.u01() - 0.5};
                const double wn = (w[0] * nn[0] + w[1] * nn[1] + w[2] * nn[2]) / (nl * nl);
                for (int q = 0; q < 3; q++) w[q] -= wn * nn[q];
                const double wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                const double g = (rng.next() % 2 ? 1 : -1) * rng.ud(0.0099, 0.05) / nl;
                d = unit(w[0] / wl + g * nn[0] / nl, w[1] / wl + g * nn[1] / nl, w[2] / wl + g * nn[2] / nl);
            } else {
                d = unit(rng.u01() - 0.5, rng.u01() - 0.5, rng.u01() - 0.5);
            }
            // origin: t0 back along the ray (bounce rays hit within a few units; some far)
            const double t0 = rng.next() % 3 ? rng.ud(0.02, 8) * sc : rng.ud(0.02, 300);
            const V o = mk((float)(X[0] - t0 * d.x), (float)(X[1] - t0 * d.y), (float)(X[2] - t0 * d.z));
            check(s, rng, o, d, p0, p1, p2, false);
        }
    }
    // the division-free range of the node codes (margin.h mt_tcap_down) against mt_margin's, on a sweep of
    // edge bounds 2^-12 .. 2^6 (every 2^-14 step of the exponent)
    for (int k = -12 * 16384; k <= 6 * 16384; k++) {
        const float E = std::ldexp(1.0f + 0.0f, 0) * (float)std::exp2((double)k / 16384.0);
        const MtMargin m = mt_margin(E, MT_LAMBDA, MT_A);
        const float tc = mt_tcap_down(E);
        ++s.node_checked;
        if (m.tcap >= 0.f ? !(tc <= m.tcap) : !(tc < 0.f)) ++s.node_viol;
    }
    // ... and both ranges against condition (C) in exact arithmetic (long double), over every edge bound from
    // the smallest denormal to 2^6 (2^-8 steps of the exponent): the tiny ones, whose c underflows and whose
    // 0.2 / c overflows in float, included; with the code the walk decodes (mt_node_codes) as well
    for (int k = -149 * 256; k <= 6 * 256; k++) {
        const float E = (float)std::exp2((double)k / 256.0);
        if (!(E > 0.f)) continue;
        const long double c = 28.3L * 100.01L * (1.0L + 0x1p-18L) * 0x1p-24L * (long double)E;
        const long double real = (0.2L / c - 2.0L * E) / (1.0L + 0x1p-18L);
        const MtMargin m = mt_margin(E, MT_LAMBDA, MT_A);
        const float tc = mt_tcap_down(E);
        uint32_t ce, ct;
        mt_node_codes(E, ce, ct);
        const float Ec = mt_code_val(ce), tn = mt_code_val(ct);
        const long double cc = 28.3L * 100.01L * (1.0L + 0x1p-18L) * 0x1p-24L * (long double)Ec;
        const long double realc = (0.2L / cc - 2.0L * Ec) / (1.0L + 0x1p-18L);
        s.node_checked += 3;
        // (a negative range covers no t: any negative value says the same)
        const auto ok = [](float v, long double r) { return r >= 0 ? (long double)v <= r : v < 0.f; };
        if (!ok(tc, real)) ++s.node_viol;
        if (!ok(m.tcap, real)) ++s.node_viol;
        if (!(Ec >= E && ok(tn, realc))) ++s.node_viol;
    }
    // the edge bound against the exact 2-norm of random edges at every scale down to the denormals
    for (int k = 0; k < 200000; k++) {
        const int ex = -149 + (int)(rng.next() % 200);
        float e[6];
        long double n1 = 0, n2 = 0;
        for (int q = 0; q < 6; q++) {
            e[q] = (float)(std::ldexp(rng.u01() - 0.5, ex + 1));
            (q < 3 ? n1 : n2) += (long double)e[q] * e[q];
        }
        const float E = mt_edge_bound(e[0], e[1], e[2], e[3], e[4], e[5]);
        ++s.node_checked;
        if (!((long double)E >= std::sqrt(std::max(n1, n2)))) ++s.node_viol;
    }
    printf("{\"tests\": %ld, \"accepted\": %ld, \"dist_checked\": %ld, \"dist_violations\": %ld, "
           "\"dist_violations_tight\": %ld, \"walk_checked\": %ld, \"walk_violations\": %ld, \"zkey_checked\": %ld, "
           "\"zkey_violations\": %ld, \"uncovered\": %ld, \"max_ratio\": %.6g, \"max_ratio_tight\": %.6g, "
           "\"node_checked\": %ld, \"node_violations\": %ld, \"node_walk_checked\": %ld, \"node_walk_violations\": %ld}\n",
           s.tests, s.accepted, s.dist_checked, s.dist_viol, s.dist_viol_tight, s.walk_checked, s.walk_viol,
           s.zkey_checked, s.zkey_viol, s.uncovered, s.max_ratio, s.max_ratio_tight, s.node_checked, s.node_viol,
           s.node_walk_checked, s.node_walk_viol);
    return (s.dist_viol || s.dist_viol_tight || s.walk_viol || s.zkey_viol || s.node_viol || s.node_walk_viol) ? 1 : 0;
}
