// slack_check -- randomized check of the bounce walk's slack QNode test on the CPU.
//
// For random quantized nodes (four child boxes quantized as build.hip quantize_axis does) and random
// rays, every box the reference slab test hits on the EXACT child box (RayTraceTraversal.hlsl:92-104,
// trace.hip ray_box) must be hit by the slack test (trace.hip qaxis / qbox_fast), at an entry
// distance <= the exact one.  Restates the device arithmetic with the same fp32 operations
// (fmaf, -ffp-contract=off); counts violations.  Used by tests/test_slack_box.py.
//   g++ -O2 -ffp-contract=off -o slack_check slack_check.cpp && ./slack_check 2000000 1
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#ifndef SLACK   // the relative slack of trace.hip qaxis (a smaller one is the test's negative control)
#define SLACK 0x1p-20f
#endif

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
    float uf(float lo, float hi) { return (float)(lo + (hi - lo) * u01()); }
};

// build.hip quantize_axis: origin, power-of-two step, per-box bytes whose decoded corners contain the box
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

// trace.hip ray_box: the reference slab test (fminf/fmaxf drop NaN)
bool ray_box(const float o[3], const float inv[3], const float lo[3], const float hi[3], float best, float& tmin) {
    float mn = -INFINITY, mx = INFINITY;
    for (int a = 0; a < 3; a++) {
        const float t0 = (lo[a] - o[a]) * inv[a], t1 = (hi[a] - o[a]) * inv[a];
        const float n = fminf(t0, t1), x = fmaxf(t0, t1);
        mn = a == 0 ? n : fmaxf(mn, n);
        mx = a == 0 ? x : fminf(mx, x);
    }
    tmin = mn;
    return 0 <= mx && mn <= mx && mn <= best;
}

// trace.hip qnode_fast_ray / qaxis / qbox_fast
bool fast_ray(const float o[3], const float inv[3]) {
    const float mi = fmaxf(fmaxf(fabsf(inv[0]), fabsf(inv[1])), fabsf(inv[2]));
    const float mo = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fabsf(o[2]));
    return mi <= 0x1p20f && mo <= 0x1p90f;
}
struct QAxis { uint32_t nw, fw; float b, an, af; };
QAxis qaxis(float org, float scl, uint32_t lw, uint32_t hw, float o, float inv) {
    QAxis r;
    const bool neg = inv < 0.f;
    r.nw = neg ? hw : lw;
    r.fw = neg ? lw : hw;
    const float m = fmaf(scl, 256.f, fabsf(org) + fabsf(o));
    const float e = m * fabsf(inv);
    const float a = (org - o) * inv;
    r.an = fmaf(e, -SLACK, a);
    r.af = fmaf(e, SLACK, a);
    r.b = scl * inv;
    return r;
}
float qt(uint32_t w, int c, float b, float a) { return fmaf((float)((w >> (8 * c)) & 255u), b, a); }
bool qbox_fast(const QAxis& x, const QAxis& y, const QAxis& z, int c, float best, float& tmin) {
    const float mn = fmaxf(fmaxf(qt(x.nw, c, x.b, x.an), qt(y.nw, c, y.b, y.an)), qt(z.nw, c, z.b, z.an));
    const float mx = fminf(fminf(qt(x.fw, c, x.b, x.af), qt(y.fw, c, y.b, y.af)), qt(z.fw, c, z.b, z.af));
    tmin = mn;
    return 0 <= mx && mn <= mx && mn <= best;
}

// a coordinate of one of several magnitude regimes
float coord(Rng& r, int regime) {
    switch (regime) {
        case 0: return r.uf(-1.f, 1.f);
        case 1: return r.uf(-500.f, 500.f);
        case 2: return r.uf(-1e6f, 1e6f);
        case 3: return 1e4f + r.uf(-1e-2f, 1e-2f);           // far from the origin, tiny boxes
        default: return (float)std::ldexp(r.u01() - 0.5, (int)(r.next() % 160) - 80);   // any scale
    }
}

}  // namespace

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    Rng rng{argc > 2 ? (uint64_t)atoll(argv[2]) : 1};
    long tested = 0, exact_hits = 0, missed = 0, later = 0, fast_rays = 0;
    for (long it = 0; it < n; it++) {
        const int regime = (int)(rng.next() % 5);
        // four child boxes
        float lo[3][4], hi[3][4];
        for (int a = 0; a < 3; a++) {
            const float base = coord(rng, regime);
            const float span = regime == 3 ? 1e-3f : fabsf(coord(rng, regime)) + 1e-30f;
            for (int c = 0; c < 4; c++) {
                float u = base + span * (float)rng.u01(), v = base + span * (float)rng.u01();
                if (rng.next() % 16 == 0) v = u;   // flat boxes
                lo[a][c] = fminf(u, v);
                hi[a][c] = fmaxf(u, v);
            }
        }
        float org[3], scl[3];
        uint32_t ql[3][4], qh[3][4];
        bool ok = true;
        for (int a = 0; a < 3; a++) ok = quantize_axis(lo[a], hi[a], org[a], scl[a], ql[a], qh[a]) && ok;
        if (!ok) continue;   // the exact record pair path
        uint32_t lw[3] = {0, 0, 0}, hw[3] = {0, 0, 0};
        for (int a = 0; a < 3; a++)
            for (int c = 0; c < 4; c++) { lw[a] |= ql[a][c] << (8 * c); hw[a] |= qh[a][c] << (8 * c); }
        // rays: origins inside, on a plane of, or around the boxes; directions random, some near an axis
        for (int k = 0; k < 8; k++) {
            float o[3], d[3];
            const int c0 = (int)(rng.next() % 4);
            for (int a = 0; a < 3; a++) {
                const uint64_t pick = rng.next() % 6;
                if (pick == 0) o[a] = lo[a][c0];
                else if (pick == 1) o[a] = hi[a][c0];
                else if (pick == 2) o[a] = lo[a][c0] + (hi[a][c0] - lo[a][c0]) * (float)rng.u01();
                else o[a] = lo[a][c0] + (hi[a][c0] - lo[a][c0] + 1e-30f) * (float)((rng.u01() - 0.5) * 40.0);
            }
            double dd[3], nrm = 0;
            for (int a = 0; a < 3; a++) { dd[a] = rng.u01() - 0.5; nrm += dd[a] * dd[a]; }
            const int axis = (int)(rng.next() % 4);
            if (axis < 3) for (int a = 0; a < 3; a++) if (a != axis) dd[a] *= std::ldexp(1.0, -(int)(rng.next() % 22));
            nrm = 0;
            for (int a = 0; a < 3; a++) nrm += dd[a] * dd[a];
            for (int a = 0; a < 3; a++) d[a] = (float)(dd[a] / std::sqrt(nrm));
            float inv[3];
            for (int a = 0; a < 3; a++) inv[a] = 1.f / d[a];
            if (!fast_ray(o, inv)) continue;
            ++fast_rays;
            const float best = rng.next() % 2 ? INFINITY : (float)(rng.u01() * 2.0 * fabsf(coord(rng, regime)));
            QAxis X = qaxis(org[0], scl[0], lw[0], hw[0], o[0], inv[0]);
            QAxis Y = qaxis(org[1], scl[1], lw[1], hw[1], o[1], inv[1]);
            QAxis Z = qaxis(org[2], scl[2], lw[2], hw[2], o[2], inv[2]);
            for (int c = 0; c < 4; c++) {
                const float blo[3] = {lo[0][c], lo[1][c], lo[2][c]}, bhi[3] = {hi[0][c], hi[1][c], hi[2][c]};
                float te, tf;
                ++tested;
                if (!ray_box(o, inv, blo, bhi, best, te)) continue;
                ++exact_hits;
                if (!qbox_fast(X, Y, Z, c, best, tf)) ++missed;
                else if (!(tf <= te)) ++later;
            }
        }
    }
    printf("{\"nodes\": %ld, \"fast_rays\": %ld, \"box_tests\": %ld, \"exact_hits\": %ld, \"missed\": %ld, "
           "\"later_entry\": %ld}\n", n, fast_rays, tested, exact_hits, missed, later);
    return (missed || later) ? 1 : 0;
}
