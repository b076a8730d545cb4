/*
 * rtbvh_oracle.cpp -- CPU ORACLE (test infrastructure only; see rtbvh_oracle.h).
 *
 * Plain restatement of the reference's LBVH build + traversal.  Every function
 * names the reference lines it follows.  No SIMD intrinsics, no FMA
 * (-ffp-contract=off), fminf/fmaxf for HLSL min/max.
 */
#include "rtbvh_oracle.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {
int g_threads = 1;   // orc_trace_ex row parallelism (orc_set_threads)
}  // namespace

namespace {

inline float fmin_h(float a, float b) { return fminf(a, b); }   // HLSL min: NaN-dropping
inline float fmax_h(float a, float b) { return fmaxf(a, b); }

struct f3 { float x, y, z; };
inline f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
inline f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 mul(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
inline f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline f3 vmin(f3 a, f3 b) { return mk(fmin_h(a.x, b.x), fmin_h(a.y, b.y), fmin_h(a.z, b.z)); }
inline f3 vmax(f3 a, f3 b) { return mk(fmax_h(a.x, b.x), fmax_h(a.y, b.y), fmax_h(a.z, b.z)); }
// HLSL normalize(v): v * rsqrt(dot(v,v)); restated with correctly rounded ops.
inline f3 normalize(f3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return mul(v, inv); }
// HLSL reflect(i, n) = i - 2 * dot(i, n) * n
inline f3 reflect(f3 i, f3 n) { float t = 2.0f * dot(i, n); return sub(i, mul(n, t)); }
inline float magnitude(f3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }  // RayTraceHelper.hlsl:6

struct f4 { float x, y, z, w; };
inline f4 mk4(float x, float y, float z, float w) { f4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
inline float sat(float v) { return fmin_h(fmax_h(v, 0.0f), 1.0f); }
// HLSL lerp(a, b, s) = a + s * (b - a)
inline float lerpf(float a, float b, float s) { return a + s * (b - a); }

// mul(float4(p, 1), M) with M row-major (row-vector convention): out_j = sum_k v_k M[k][j]
inline f3 xform_point(const float* M, f3 p) {
    f3 r;
    r.x = ((p.x * M[0] + p.y * M[4]) + p.z * M[8]) + M[12];
    r.y = ((p.x * M[1] + p.y * M[5]) + p.z * M[9]) + M[13];
    r.z = ((p.x * M[2] + p.y * M[6]) + p.z * M[10]) + M[14];
    return r;
}
// mul(n, (float3x3)M)  (RayTraceTraversal.hlsl:30-31)
inline f3 xform_normal(const float* M, f3 n) {
    f3 r;
    r.x = (n.x * M[0] + n.y * M[4]) + n.z * M[8];
    r.y = (n.x * M[1] + n.y * M[5]) + n.z * M[9];
    r.z = (n.x * M[2] + n.y * M[6]) + n.z * M[10];
    return r;
}

inline f3 vpos(const orc_scene* s, uint32_t vi) {
    const orc_vertex& v = s->verts[vi];
    return mk(v.position[0], v.position[1], v.position[2]);
}

// quantise one axis: CPUTests (Morton Code/main.cpp:84-92, ShaderSim/main.cpp:226-237)
inline uint32_t quantise_cputests(float p) {
    p *= 1024.f;
    if (p < 0) p = 0;
    else if (p >= 1024) p = 1023;
    if (p != p) return 0;          // NaN: x86-64 cvttss2si yields 0 after the u32 truncation
    return (uint32_t)p;
}
// quantise one axis: HLSL clamp(p, 0, 1023) (MortonCodes.hlsl:42-47); clamp = min(max())
inline uint32_t quantise_hlsl(float p) {
    p *= 1024.f;
    p = fmin_h(fmax_h(p, 0.0f), 1023.0f);
    return (uint32_t)p;
}

}  // namespace

extern "C" {

/* bitTwiddling, MortonCodes.hlsl:13-31 (== expand, Morton Code/main.cpp:56-73) */
uint32_t orc_expand_bits(uint32_t var) {
    static const uint32_t masks[] = {0x09249249u, 0x030c30c3u, 0x0300f00fu, 0x030000ffu, 0x000003ffu};
    uint32_t shift = 16;
    for (uint32_t i = 4; 0 < i; i--) {
        var &= masks[i];
        var |= var << shift;
        shift >>= 1;
    }
    return var & masks[0];
}

/* calcMorton, Morton Code/main.cpp:75-98: code[2] | code[1] << 1 | code[0] << 2 */
uint32_t orc_morton_point_cputests(float x, float y, float z) {
    return orc_expand_bits(quantise_cputests(z)) | orc_expand_bits(quantise_cputests(y)) << 1 |
           orc_expand_bits(quantise_cputests(x)) << 2;
}

/* calcMortonCode, MortonCodes.hlsl:33-52: code[0] | code[1] << 1 | code[2] << 2 */
uint32_t orc_morton_point_hlsl(float x, float y, float z) {
    return orc_expand_bits(quantise_hlsl(x)) | orc_expand_bits(quantise_hlsl(y)) << 1 |
           orc_expand_bits(quantise_hlsl(z)) << 2;
}

/* ShaderSim/main.cpp:269-301: mesh vertex AABB, true centroid (x0+x1+x2)/3 */
void orc_morton_tris_cputests(const orc_scene* s, uint32_t* codes) {
    f3 mn = mk(9999999e10f, 9999999e10f, 9999999e10f), mx = mk(-9999999e10f, -9999999e10f, -9999999e10f);
    // (all-cores variant: per-thread partial boxes; min/max are exact, so the box is the same)
#pragma omp parallel num_threads(g_threads) if (g_threads > 1)
    {
        f3 lo = mn, hi = mx;
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)s->num_verts; i++) {
            f3 p = vpos(s, (uint32_t)i);
            lo = vmin(p, lo);
            hi = vmax(p, hi);
        }
#pragma omp critical
        {
            mn = vmin(lo, mn);
            mx = vmax(hi, mx);
        }
    }
    const uint32_t ntri = s->num_indices / 3;
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
    for (uint32_t t = 0; t < ntri; t++) {
        f3 a = vpos(s, s->indices[3 * t]), b = vpos(s, s->indices[3 * t + 1]), c = vpos(s, s->indices[3 * t + 2]);
        float xv = a.x + b.x + c.x, yv = a.y + b.y + c.y, zv = a.z + b.z + c.z;
        codes[t] = orc_morton_point_cputests((xv / 3.f - mn.x) / (mx.x - mn.x),
                                             (yv / 3.f - mn.y) / (mx.y - mn.y),
                                             (zv / 3.f - mn.z) / (mx.z - mn.z));
    }
}

/* MortonCodes.hlsl:70-106 incl. the `avg = minUnion(bbMin, vertData)` bug (:98) */
void orc_morton_tris_hlsl(const orc_scene* s, const float wvp[16], const float smin[3],
                          const float smax[3], uint32_t* codes) {
    const uint32_t ntri = s->num_indices / 3;
    for (uint32_t t = 0; t < ntri; t++) {
        f3 v = xform_point(wvp, vpos(s, s->indices[3 * t]));
        f3 bmin = v, avg = v;
        for (int k = 1; k < 3; k++) {
            v = xform_point(wvp, vpos(s, s->indices[3 * t + k]));
            bmin = vmin(bmin, v);
            avg = vmin(bmin, v);
        }
        avg = mk(avg.x / 3.f, avg.y / 3.f, avg.z / 3.f);
        codes[t] = orc_morton_point_hlsl((avg.x - smin[0]) / (smax[0] - smin[0]),
                                         (avg.y - smin[1]) / (smax[1] - smin[1]),
                                         (avg.z - smin[2]) / (smax[2] - smin[2]));
    }
}

/* prefixSum, RadixBVHCombo/main.cpp:249-284 (== RadixSortP1.hlsl:7-49): exclusive */
void orc_blelloch_scan256(uint32_t* data) {
    const uint32_t DS = 256;
    for (uint32_t up = 1; up < DS; up <<= 1)
        for (uint32_t id = 0; id < DS >> 1; id++) {
            uint32_t l = id * (up << 1) + up - 1, r = id * (up << 1) + (up << 1) - 1;
            if (r < DS) data[r] += data[l];
        }
    data[DS - 1] = 0;
    for (uint32_t dn = DS >> 1; 0 < dn; dn >>= 1)
        for (uint32_t id = 0; id < DS >> 1; id++) {
            uint32_t base = id * (dn << 1), i1 = base + dn - 1, i2 = base + (dn << 1) - 1;
            if (i2 < DS) {
                uint32_t tmp = data[i1];
                data[i1] = data[i2];
                data[i2] = tmp + data[i2];
            }
        }
}

/* 32 split passes, RadixBVHCombo/main.cpp:369-480 (GPU: RadixSortP1.hlsl:51-106,
 * RadixSortP2.hlsl:3-65).  The serial O(G) sum of group zero-counts that every
 * group repeats (RadixSortP2.hlsl:16-22, combo :399-412) is restated as one
 * running sum: identical numPrecOnes / netOnes values. */
void orc_split_sort(const uint32_t* keys, uint32_t n, uint32_t* perm) {
    const uint32_t DS = 256;
    const uint32_t G = (n + DS - 1) / DS, np = G * DS;
    std::vector<uint32_t> k(np, 0xFFFFFFFFu), idx(np), k2(np), idx2(np), flags(np), zeros(G), prec(G);
    for (uint32_t i = 0; i < n; i++) k[i] = keys[i];
    for (uint32_t i = 0; i < np; i++) idx[i] = i;
    // (all-cores variant, orc_set_threads > 1: the flags, the groups' scans and the scatter
    // run in parallel -- one thread per element / group, as the GPU dispatch does)
    for (uint32_t r = 0; r < 32; r++) {
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
        for (uint32_t i = 0; i < np; i++) flags[i] = !(k[i] & (1u << r));        // RadixSortP1.hlsl:78
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
        for (uint32_t g = 0; g < G; g++) {
            uint32_t* f = &flags[g * DS];
            uint32_t last = f[DS - 1];                                            // :84-85
            orc_blelloch_scan256(f);
            zeros[g] = last + f[DS - 1];                                          // :94-95
        }
        uint32_t net = 0;
        for (uint32_t g = 0; g < G; g++) {
            prec[g] = net;                                                        // RadixSortP2.hlsl:16-22
            net += zeros[g];
        }
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
        for (uint32_t i = 0; i < np; i++) {
            uint32_t g = i / DS, pos0 = flags[i];
            uint32_t present = i - pos0 - prec[g] + net;                         // RadixSortP2.hlsl:45-48
            uint32_t dest = (k[i] & (1u << r)) ? present : pos0 + prec[g];        // :50-53
            k2[dest] = k[i];
            idx2[dest] = idx[i];
        }
        k.swap(k2);
        idx.swap(idx2);
    }
    for (uint32_t i = 0; i < n; i++) perm[i] = idx[i];
}

void orc_lsd_sort(const uint32_t* keys, uint32_t n, uint32_t* perm) {
    std::vector<uint32_t> k(keys, keys + n), idx(n), k2(n), idx2(n);
    for (uint32_t i = 0; i < n; i++) idx[i] = i;
    for (uint32_t shift = 0; shift < 32; shift += 8) {
        uint32_t cnt[257] = {0};
        for (uint32_t i = 0; i < n; i++) cnt[((k[i] >> shift) & 255u) + 1]++;
        for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
        for (uint32_t i = 0; i < n; i++) {
            uint32_t d = (k[i] >> shift) & 255u, o = cnt[d]++;
            k2[o] = k[i];
            idx2[o] = idx[i];
        }
        k.swap(k2);
        idx.swap(idx2);
    }
    for (uint32_t i = 0; i < n; i++) perm[i] = idx[i];
}

}  // extern "C"

namespace {

const int kDeBruijn[32] = {0, 31, 9,  30, 3,  8,  13, 29, 2,  5,  7,  21, 12, 24, 28, 19,
                           1, 10, 4,  14, 6,  22, 25, 20, 11, 15, 23, 26, 16, 27, 17, 18};

// leadingZero, BVHConstructP1.hlsl:39-53
int32_t leading_zero_hlsl(uint32_t data) {
    if (data == 0) return 32;
    data |= data >> 1; data |= data >> 2; data |= data >> 4; data |= data >> 8; data |= data >> 16;
    data++;
    return kDeBruijn[(uint32_t)(data * 0x076be629u) >> 27];
}
// leadingPrefix, RadixBVHCombo/main.cpp:136-151 (index tie-break WITHOUT the +32)
int32_t leading_prefix_cputests(uint32_t d1, uint32_t d2, uint32_t i1, uint32_t i2) {
    uint32_t data = d1 == d2 ? i1 ^ i2 : d1 ^ d2;
    data |= data >> 1; data |= data >> 2; data |= data >> 4; data |= data >> 8; data |= data >> 16;
    data++;
    return data ? kDeBruijn[(uint32_t)(data * 0x076be629u) >> 27] : 32;
}
// leadingPrefix, BVHConstructP1.hlsl:61-72 (== clz64 of index-augmented keys)
int32_t leading_prefix_hlsl(uint32_t d1, uint32_t d2, uint32_t i1, uint32_t i2) {
    int32_t lpr = leading_zero_hlsl(d1 ^ d2);
    if (lpr == 32) lpr += leading_zero_hlsl(i1 ^ i2);
    return lpr;
}

}  // namespace

extern "C" {

/* leadingPrefixBounds, BVHConstructP1.hlsl:78-84 / RadixBVHCombo/main.cpp:157-162 */
int32_t orc_delta(int mode, const uint32_t* codes, uint32_t n, uint32_t i, int64_t j) {
    if (j < 0 || j >= (int64_t)n) return -1;
    if (mode == ORC_DELTA_CPUTESTS) return leading_prefix_cputests(codes[i], codes[j], i, (uint32_t)j);
    return leading_prefix_hlsl(codes[i], codes[j], i, (uint32_t)j);
}

/* getChildren + main, BVHConstructP1.hlsl:99-188 (RadixBVHCombo/main.cpp:168-237,508-530) */
void orc_karras(int mode, const uint32_t* c, uint32_t n, uint32_t* parent, uint32_t* cl, uint32_t* cr) {
    const uint32_t total = 2 * n - 1;
    for (uint32_t k = 0; k < total; k++) { parent[k] = 0xFFFFFFFFu; cl[k] = 0xFFFFFFFFu; cr[k] = 0xFFFFFFFFu; }
    // (all-cores variant: one iteration per internal node, as BVHConstructP1's threads; every
    // node has one parent, so the writes of two iterations never meet)
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
    for (int64_t i = 0; i < (int64_t)n - 1; i++) {
        int64_t d = orc_delta(mode, c, n, (uint32_t)i, i + 1) < orc_delta(mode, c, n, (uint32_t)i, i - 1) ? -1 : 1;
        int32_t min_lz = orc_delta(mode, c, n, (uint32_t)i, i - d);
        int64_t bound_len = 2;
        for (; min_lz < orc_delta(mode, c, n, (uint32_t)i, i + bound_len * d); bound_len <<= 1) {}
        int64_t delta = bound_len, delta_sum = 0;
        do {
            delta = (delta + 1) >> 1;
            if (min_lz < orc_delta(mode, c, n, (uint32_t)i, i + (delta_sum + delta) * d)) delta_sum += delta;
        } while (1 < delta);
        int64_t bound_start = i + delta_sum * d;
        int32_t lz = orc_delta(mode, c, n, (uint32_t)i, bound_start);
        delta = delta_sum;
        int64_t tmp = 0;
        do {
            delta = (delta + 1) >> 1;
            if (lz < orc_delta(mode, c, n, (uint32_t)i, i + (tmp + delta) * d)) tmp += delta;
        } while (1 < delta);
        int64_t loc = i + tmp * d + std::min<int64_t>(d, 0);
        uint32_t left = (std::min(i, bound_start) == loc) ? (uint32_t)loc : (uint32_t)(loc + n);
        uint32_t right = (std::max(i, bound_start) == loc + 1) ? (uint32_t)(loc + 1) : (uint32_t)(loc + 1 + n);
        cl[n + i] = left;
        cr[n + i] = right;
        parent[left] = (uint32_t)(n + i);
        parent[right] = (uint32_t)(n + i);
    }
    if (n > 1) parent[n] = 0xFFFFFFFFu;   // BVHConstructP1.hlsl:186-187 (the root; n == 1: leaf 0, set above)
}

/* BVHConstructP2.hlsl:8-37 emulated thread by thread (RadixBVHCombo/main.cpp:535-574) */
uint32_t orc_refit(uint32_t n, const uint32_t* parent, const uint32_t* cl, const uint32_t* cr,
                   float* bmin, float* bmax) {
    if (n < 2) return 0;
    if (g_threads > 1) {   // all-cores variant: the GPU's one thread per leaf with an atomic ticket per node
        std::vector<uint32_t> ticket(n, 0);
        uint32_t longest = 0;
#pragma omp parallel for num_threads(g_threads) schedule(static) reduction(max : longest)
        for (uint32_t t = 0; t < n; t++) {
            uint32_t node = parent[t], loops = 0;
            // acq_rel: the first arriver's child box is visible to the second (InterlockedAdd + the
            // fence BVHConstructP2.hlsl lacks); min/max are exact, so the order does not matter
            uint32_t value = __atomic_fetch_add(&ticket[node - n], 1u, __ATOMIC_ACQ_REL);
            while (value) {
                uint32_t a = cl[node], b = cr[node];
                for (int k = 0; k < 3; k++) {
                    bmin[3 * node + k] = fmin_h(bmin[3 * a + k], bmin[3 * b + k]);
                    bmax[3 * node + k] = fmax_h(bmax[3 * a + k], bmax[3 * b + k]);
                }
                node = parent[node];
                if (node == 0xFFFFFFFFu) break;
                value = __atomic_fetch_add(&ticket[node - n], 1u, __ATOMIC_ACQ_REL);
                loops++;
            }
            longest = std::max(longest, loops);
        }
        return longest;
    }
    std::vector<uint32_t> transfer(n, 0);
    uint32_t longest = 0;
    for (uint32_t t = 0; t < n; t++) {
        uint32_t node = parent[t];
        uint32_t value = transfer[node - n]++;
        uint32_t loops = 0;
        while (value) {
            uint32_t a = cl[node], b = cr[node];
            for (int k = 0; k < 3; k++) {
                bmin[3 * node + k] = fmin_h(bmin[3 * a + k], bmin[3 * b + k]);
                bmax[3 * node + k] = fmax_h(bmax[3 * a + k], bmax[3 * b + k]);
            }
            node = parent[node];
            if (node == 0xFFFFFFFFu) break;
            value = transfer[node - n]++;
            loops++;
        }
        longest = std::max(longest, loops);
    }
    return longest;
}

int orc_build(const orc_scene* s, const float wvp[16], int morton_mode, int delta_mode,
              const float smin[3], const float smax[3], int sort_mode, orc_node* out) {
    const uint32_t n = s->num_indices / 3;
    if (n == 0) return 1;
    std::vector<uint32_t> codes(n), perm(n), sorted(n);
    if (morton_mode == ORC_MORTON_HLSL) orc_morton_tris_hlsl(s, wvp, smin, smax, codes.data());
    else orc_morton_tris_cputests(s, codes.data());
    if (sort_mode == 0) orc_split_sort(codes.data(), n, perm.data());
    else orc_lsd_sort(codes.data(), n, perm.data());
    for (uint32_t i = 0; i < n; i++) sorted[i] = codes[perm[i]];
    const uint32_t total = 2 * n - 1;
    std::vector<uint32_t> parent(total), cl(total), cr(total);
    std::vector<float> bmin(3 * (size_t)total, 0.f), bmax(3 * (size_t)total, 0.f);
    orc_karras(delta_mode, sorted.data(), n, parent.data(), cl.data(), cr.data());
    // leaf AABB in clip space: MortonCodes.hlsl:84-99, 115-116
#pragma omp parallel for num_threads(g_threads) if (g_threads > 1) schedule(static)
    for (uint32_t i = 0; i < n; i++) {
        uint32_t t = perm[i];
        f3 v = xform_point(wvp, vpos(s, s->indices[3 * t]));
        f3 lo = v, hi = v;
        for (int k = 1; k < 3; k++) {
            v = xform_point(wvp, vpos(s, s->indices[3 * t + k]));
            lo = vmin(lo, v);
            hi = vmax(hi, v);
        }
        bmin[3 * i] = lo.x; bmin[3 * i + 1] = lo.y; bmin[3 * i + 2] = lo.z;
        bmax[3 * i] = hi.x; bmax[3 * i + 1] = hi.y; bmax[3 * i + 2] = hi.z;
    }
    orc_refit(n, parent.data(), cl.data(), cr.data(), bmin.data(), bmax.data());
    for (uint32_t k = 0; k < total; k++) {
        orc_node& o = out[k];
        o.parent = parent[k];
        o.child_l = cl[k];
        o.child_r = cr[k];
        o.code = k < n ? sorted[k] : 0u;
        for (int a = 0; a < 3; a++) { o.bb_min[a] = bmin[3 * (size_t)k + a]; o.bb_max[a] = bmax[3 * (size_t)k + a]; }
        o.index = k < n ? 3 * perm[k] : 0u;
    }
    return 0;
}

}  // extern "C"

namespace {

struct Tri { f3 p[3]; f3 nrm[3]; float uv[3][2]; };
struct Ray { f3 o, d, inv; };

struct Ctx {
    const orc_scene* s;
    const orc_node* nodes;
    uint32_t n;
    const float* wvp;
    const float* wv;
    uint64_t int_visits, leaf_visits, overflow, max_depth;
};

// getUpdateVerts, RayTraceTraversal.hlsl:25-35
void fetch_tri(const Ctx& c, uint32_t index, Tri& t) {
    for (int k = 0; k < 3; k++) {
        const orc_vertex& v = c.s->verts[c.s->indices[index + k]];
        t.p[k] = xform_point(c.wvp, mk(v.position[0], v.position[1], v.position[2]));
        t.nrm[k] = xform_normal(c.wv, mk(v.normal[0], v.normal[1], v.normal[2]));
        t.uv[k][0] = v.texcoord[0];
        t.uv[k][1] = v.texcoord[1];
    }
}

// rayTriangleCollision, RayTraceTraversal.hlsl:41-86 (EPSILON .01 as float)
float ray_triangle(const Ray& r, const f3* p) {
    const float EPS = 0.01f;
    f3 e1 = sub(p[1], p[0]), e2 = sub(p[2], p[0]);
    f3 tmp = cross(r.d, e2);
    float dx = dot(e1, tmp);
    if (fabsf(dx) < EPS) return -1.f;
    float idx = 1.f / dx;
    f3 rt = sub(r.o, p[0]);
    float u = dot(rt, tmp) * idx;
    if (u < .0f || 1.f < u) return -1.f;
    tmp = cross(rt, e1);
    float v = dot(r.d, tmp) * idx;
    if (v < .0f || 1.f < u + v) return -1.f;
    float t = dot(e2, tmp) * idx;
    if (EPS < t) return t;
    return -1.f;
}

// rayBoxCollision, RayTraceTraversal.hlsl:92-104
bool ray_box(const Ray& r, const float* bmin, const float* bmax, bool hit, float dist) {
    f3 dmin = mulv(sub(mk(bmin[0], bmin[1], bmin[2]), r.o), r.inv);
    f3 dmax = mulv(sub(mk(bmax[0], bmax[1], bmax[2]), r.o), r.inv);
    f3 mnv = vmin(dmin, dmax), mxv = vmax(dmin, dmax);
    float mn = fmax_h(fmax_h(mnv.x, mnv.y), mnv.z);
    float mx = fmin_h(fmin_h(mxv.x, mxv.y), mxv.z);
    return 0 <= mx && mn <= mx && (!hit || mn <= dist);
}

struct Hit { bool hit; float dist; uint32_t tri; Tri t; };

// findCollision, RayTraceTraversal.hlsl:106-193 (stack 66 entries instead of 32;
// depth of a clz64 Karras tree is <= 64 so it cannot overflow)
void find_collision(Ctx& c, const Ray& r, Hit& h) {
    h.hit = false;
    h.dist = 0;
    h.tri = 0;
    const int STACK = 66;
    int32_t stack[STACK];
    int sp = 0;
    stack[0] = -1;
    int32_t node = (int32_t)c.n;   // root
    if (c.n == 1) node = 0;        // a single leaf is its own root
    Tri tt;
    do {
        const orc_node& nd = c.nodes[node];
        if ((int32_t)nd.child_l == -1 && (int32_t)nd.child_r == -1) {
            c.leaf_visits++;
            fetch_tri(c, nd.index, tt);
            float d = ray_triangle(r, tt.p);
            if (d != -1 && (!h.hit || d < h.dist)) {
                h.tri = nd.index / 3;
                h.hit = true;
                h.t = tt;
                h.dist = d;
            }
            node = stack[sp--];
            continue;
        }
        c.int_visits++;
        const orc_node& L = c.nodes[nd.child_l];
        const orc_node& R = c.nodes[nd.child_r];
        bool lh = ray_box(r, L.bb_min, L.bb_max, h.hit, h.dist);
        bool rh = ray_box(r, R.bb_min, R.bb_max, h.hit, h.dist);
        if (!lh && !rh) {
            node = stack[sp--];
        } else {
            if (lh && rh) {
                if (sp + 1 >= STACK) { c.overflow++; node = stack[sp--]; continue; }
                stack[++sp] = (int32_t)nd.child_r;
                if ((uint64_t)sp > c.max_depth) c.max_depth = (uint64_t)sp;
            }
            node = lh ? (int32_t)nd.child_l : (int32_t)nd.child_r;
        }
    } while (sp != -1);
}

// getNromalTexCoord, RayTraceHelper.hlsl:12-35
void normal_texcoord(const Tri& t, f3 pt, float uv[2], f3& n) {
    f3 v0 = sub(t.p[0], pt), v1 = sub(t.p[1], pt), v2 = sub(t.p[2], pt);
    float a0 = magnitude(cross(sub(t.p[0], t.p[1]), sub(t.p[0], t.p[2])));
    float a1 = magnitude(cross(v1, v2)) / a0;
    float a2 = magnitude(cross(v2, v0)) / a0;
    float a3 = magnitude(cross(v0, v1)) / a0;
    uv[0] = (t.uv[0][0] * a1 + t.uv[1][0] * a2) + t.uv[2][0] * a3;
    uv[1] = (t.uv[0][1] * a1 + t.uv[1][1] * a2) + t.uv[2][1] * a3;
    n = add(add(mul(t.nrm[0], a1), mul(t.nrm[1], a2)), mul(t.nrm[2], a3));
}

// diffuseTex[k].SampleLevel(compSample, uv, 0), RayTraceRender.hlsl:22-26, with the
// sampler of Image.cpp:154-169 (MIN_MAG_MIP_LINEAR, WRAP) on R8G8B8A8_UNORM_SRGB
// texels (Image.cpp:9).  Restated (parity unpinned: no DevIL, no D3D filter): texels
// decoded sRGB -> linear (IEC 61966-2-1 in double, rounded to float; alpha / 255),
// x = u*W - 0.5, y = v*H - 0.5, wrap, bilinear as lerp(lerp(t00, t10, fx), lerp(t01, t11, fx), fy).
struct SrgbTable {
    float v[256];
    SrgbTable() {
        for (int i = 0; i < 256; i++) {
            const double c = i / 255.0;
            v[i] = (float)(c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4));
        }
    }
};
const float* srgb_table() {
    static const SrgbTable tab;   // thread-safe one-time init
    return tab.v;
}
f4 texel(const orc_texture& t, uint32_t x, uint32_t y) {
    const uint8_t* p = t.rgba8 + ((size_t)y * t.width + x) * 4;
    const float* tab = srgb_table();
    return mk4(tab[p[0]], tab[p[1]], tab[p[2]], (float)p[3] / 255.f);
}
uint32_t wrap_index(float f, uint32_t n) {
    if (!(std::fabs(f) < 2147483648.f)) f = 0.f;
    int64_t i = (int64_t)f % (int64_t)n;
    return (uint32_t)(i < 0 ? i + n : i);
}
f4 sample_texture(const orc_texture& t, float u, float v) {
    const float x = u * (float)t.width - 0.5f, y = v * (float)t.height - 0.5f;
    const float x0 = std::floor(x), y0 = std::floor(y);
    const float fx = x - x0, fy = y - y0;
    const uint32_t ix = wrap_index(x0, t.width), iy = wrap_index(y0, t.height);
    const uint32_t ix1 = ix + 1 == t.width ? 0u : ix + 1, iy1 = iy + 1 == t.height ? 0u : iy + 1;
    const f4 t00 = texel(t, ix, iy), t10 = texel(t, ix1, iy), t01 = texel(t, ix, iy1), t11 = texel(t, ix1, iy1);
    const f4 top = mk4(lerpf(t00.x, t10.x, fx), lerpf(t00.y, t10.y, fx), lerpf(t00.z, t10.z, fx), lerpf(t00.w, t10.w, fx));
    const f4 bot = mk4(lerpf(t01.x, t11.x, fx), lerpf(t01.y, t11.y, fx), lerpf(t01.z, t11.z, fx), lerpf(t01.w, t11.w, fx));
    return mk4(lerpf(top.x, bot.x, fy), lerpf(top.y, bot.y, fy), lerpf(top.z, bot.z, fy), lerpf(top.w, bot.w, fy));
}

// renderPixel * specular, RayTraceRender.hlsl:16-29 + RayTraceLaunch.hlsl:57-59.
// A material with texNum != -1 but no texture bound samples white.
f4 shade(const Ctx& c, uint32_t tri, const float uv[2], bool* textured) {
    const orc_material& m = c.s->materials[c.s->mat_indices[tri]];
    f4 tex = mk4(1, 1, 1, 1);
    *textured = m.tex_num != -1;
    if (*textured && (uint32_t)m.tex_num < c.s->num_textures)
        tex = sample_texture(c.s->textures[m.tex_num], uv[0], uv[1]);
    f4 col = mk4(sat(m.ambient[0] + m.diffuse[0] * tex.x), sat(m.ambient[1] + m.diffuse[1] * tex.y),
                 sat(m.ambient[2] + m.diffuse[2] * tex.z), sat(m.ambient[3] + m.diffuse[3] * tex.w));
    return mk4(col.x * m.specular[0], col.y * m.specular[1], col.z * m.specular[2], col.w * m.specular[3]);
}

inline Ray make_ray(f3 o, f3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    r.inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    return r;
}

// HLSL refract(i, n, eta) as the intrinsic is documented: cosi = dot(-i, n),
// cost2 = 1 - eta*eta*(1 - cosi*cosi), t = eta*i + (eta*cosi - sqrt(|cost2|))*n,
// result t * (cost2 > 0).  Used by RayTraceLaunch.hlsl:76-78 (parity unpinned:
// no reference test covers refraction).
inline f3 refract_hlsl(f3 i, f3 n, float eta) {
    const float cosi = dot(mk(-i.x, -i.y, -i.z), n);
    const float cost2 = 1.0f - eta * eta * (1.0f - cosi * cosi);
    const float s = eta * cosi - sqrtf(fabsf(cost2));
    const f3 t = add(mul(i, eta), mul(n, s));
    const float keep = cost2 > 0.0f ? 1.0f : 0.0f;
    return mul(t, keep);
}

// RayPresent (RayTraceGlobal.hlsl:30-35): intensity, origin, direction, invDirection, color
inline void put_record(float* r, float intensity, const Ray* ray, f4 color) {
    r[0] = intensity;
    if (ray) {
        r[1] = ray->o.x; r[2] = ray->o.y; r[3] = ray->o.z;
        r[4] = ray->d.x; r[5] = ray->d.y; r[6] = ray->d.z;
        r[7] = ray->inv.x; r[8] = ray->inv.y; r[9] = ray->inv.z;
    } else {
        for (int k = 1; k < 10; k++) r[k] = 0.f;
    }
    r[10] = color.x; r[11] = color.y; r[12] = color.z; r[13] = color.w;
}

}  // namespace

extern "C" {

int orc_trace(const orc_scene* s, const orc_node* nodes, uint32_t n, const float wvp[16],
              const float wv[16], uint32_t W, uint32_t H, uint32_t bounces, uint32_t row_begin,
              uint32_t row_end, uint32_t row_step, float* rgba, float* intensity_out,
              uint64_t* counters) {
    return orc_trace_ex(s, nodes, n, wvp, wv, W, H, bounces, row_begin, row_end, row_step, rgba, intensity_out,
                        counters, nullptr, nullptr);
}

int orc_trace_ex(const orc_scene* s, const orc_node* nodes, uint32_t n, const float wvp[16],
                 const float wv[16], uint32_t W, uint32_t H, uint32_t bounces, uint32_t row_begin,
                 uint32_t row_end, uint32_t row_step, float* rgba, float* intensity_out,
                 uint64_t* counters, float* refl_rec, float* refr_rec) {
    if (n == 0 || row_step == 0) return 1;
    uint64_t total[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const float hw = (float)(W >> 1), hh = (float)(H >> 1);
    const uint32_t last = row_end < H ? row_end : H;
    const int64_t nrows = row_begin < last ? ((int64_t)last - row_begin + row_step - 1) / row_step : 0;
    // rows are independent: OpenMP over rows when orc_set_threads(n > 1) (the all-cores CPU
    // baseline); each thread sums its own counters, merged at the end (same totals)
#pragma omp parallel num_threads(g_threads)
    {
    uint64_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma omp for schedule(dynamic, 1)
    for (int64_t out_row = 0; out_row < nrows; out_row++) {
        const uint32_t y = row_begin + (uint32_t)out_row * row_step;
        for (uint32_t x = 0; x < W; x++) {
            Ctx c{s, nodes, n, wvp, wv, 0, 0, 0, 0};
            // RayTraceLaunch.hlsl:23-30
            Ray ray = make_ray(mk(((float)x - hw) / 4.f, ((float)y - hh) / 4.f, 0), mk(0, 0, 1));
            Hit h;
            find_collision(c, ray, h);
            cnt[0]++;
            f4 color;
            float intensity;
            Ray bray;
            bool have_bray = false;
            const size_t o = (size_t)out_row * W + x;
            if (h.hit) {
                cnt[4]++;
                f3 hit = add(ray.o, mul(ray.d, h.dist));                          // getHitLoc :15-19
                const orc_material& m = s->materials[s->mat_indices[h.tri]];
                intensity = m.shininess / 1000.f * 1;                             // :48
                float uv[2];
                f3 nrm;
                normal_texcoord(h.t, hit, uv, nrm);
                bool tx;
                color = shade(c, h.tri, uv, &tx);
                cnt[5] += tx;
                if (intensity != 0) {
                    bray = make_ray(add(hit, mul(nrm, .001f)), normalize(reflect(ray.d, nrm)));  // :61-67
                    have_bray = true;
                }
                if (refr_rec) {   // :70-80; the ray stays zero when the intensity is 0 (unset in HLSL)
                    const float ri = (1.f - m.alpha) * 1;
                    Ray rr;
                    if (ri != 0) rr = make_ray(sub(hit, mul(nrm, .001f)), normalize(refract_hlsl(ray.d, nrm, m.optical_density)));
                    put_record(refr_rec + 14 * o, ri, ri != 0 ? &rr : nullptr, mk4(1.f, 1.f, 1.f, 1.f));
                }
            } else {
                color = mk4(.5f, .5f, .5f, 1.f);                                   // :85 clearRayPresent
                intensity = 0;
                if (refr_rec) put_record(refr_rec + 14 * o, 0.f, nullptr, color);
            }
            // RayTraceReflection.hlsl:17-60, `bounces` passes (Graphics.cpp:795)
            for (uint32_t b = 0; b < bounces && 0 < intensity; b++) {
                cnt[1]++;
                find_collision(c, bray, h);
                if (h.hit) {
                    cnt[4]++;
                    f3 hit = add(bray.o, mul(bray.d, h.dist));
                    const orc_material& m = s->materials[s->mat_indices[h.tri]];
                    float uv[2];
                    f3 nrm;
                    normal_texcoord(h.t, hit, uv, nrm);
                    bool tx;
                    f4 sc = shade(c, h.tri, uv, &tx);
                    cnt[5] += tx;
                    color = mk4(lerpf(color.x, sc.x, intensity), lerpf(color.y, sc.y, intensity),
                                lerpf(color.z, sc.z, intensity), lerpf(color.w, sc.w, intensity));
                    intensity *= m.shininess / 1000.f * 1;
                    bray = make_ray(add(hit, mul(nrm, .0001f)), normalize(reflect(bray.d, nrm)));
                    have_bray = true;
                } else {
                    color = mk4(lerpf(color.x, .5f, intensity), lerpf(color.y, .5f, intensity),
                                lerpf(color.z, .5f, intensity), lerpf(color.w, 1.f, intensity));
                    intensity = 0;
                }
            }
            if (refl_rec) put_record(refl_rec + 14 * o, intensity, have_bray ? &bray : nullptr, color);
            if (rgba) { rgba[4 * o] = color.x; rgba[4 * o + 1] = color.y; rgba[4 * o + 2] = color.z; rgba[4 * o + 3] = color.w; }
            if (intensity_out) intensity_out[o] = intensity;
            cnt[2] += c.int_visits;
            cnt[3] += c.leaf_visits;
            cnt[6] += c.overflow;
            if (c.max_depth > cnt[7]) cnt[7] = c.max_depth;
        }
    }
#pragma omp critical
    {
        for (int k = 0; k < 7; k++) total[k] += cnt[k];
        if (cnt[7] > total[7]) total[7] = cnt[7];
    }
    }
    if (counters) for (int k = 0; k < 8; k++) counters[k] = total[k];
    return 0;
}

void orc_sample_texture(const orc_texture* t, float u, float v, float out[4]) {
    const f4 r = sample_texture(*t, u, v);
    out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}

/* Graphics.cpp:44-53 with XMMatrixLookAtLH / XMMatrixPerspectiveFovLH restated
 * (DirectXMath formulas; libm sinf/cosf instead of XMScalarSinCos: unpinned). */
void orc_camera_reference(uint32_t W, uint32_t H, float wvp[16], float wv[16]) {
    f3 eye = mk(0.0f, 5.0f, -100.0f), at = mk(0, 0, 0), up = mk(0, 1.f, 0);   // Graphics.h:200-204
    f3 dir = sub(at, eye);
    f3 r2 = mul(dir, 1.0f / sqrtf(dot(dir, dir)));
    f3 cx = cross(up, r2);
    f3 r0 = mul(cx, 1.0f / sqrtf(dot(cx, cx)));
    f3 r1 = cross(r2, r0);
    f3 ne = mk(-eye.x, -eye.y, -eye.z);
    float view[16] = {r0.x, r1.x, r2.x, 0, r0.y, r1.y, r2.y, 0, r0.z, r1.z, r2.z, 0,
                      dot(r0, ne), dot(r1, ne), dot(r2, ne), 1};
    float fov = 3.14159265358979323846f / 4, aspect = (float)H / (float)W, zn = 0.1f, zf = 1000.0f;
    float sn = sinf(0.5f * fov), cs = cosf(0.5f * fov);
    float hgt = cs / sn, wdt = hgt / aspect, range = zf / (zf - zn);
    float proj[16] = {wdt, 0, 0, 0, 0, hgt, 0, 0, 0, 0, range, 1, 0, 0, -range * zn, 0};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            wvp[4 * i + j] = ((view[4 * i] * proj[j] + view[4 * i + 1] * proj[4 + j]) +
                              view[4 * i + 2] * proj[8 + j]) + view[4 * i + 3] * proj[12 + j];
    memcpy(wv, view, sizeof(view));
}

uint64_t orc_fnv1a64(const void* data, uint64_t nbytes) {
    const uint8_t* p = (const uint8_t*)data;
    uint64_t h = 1469598103934665603ull;
    for (uint64_t i = 0; i < nbytes; i++) { h ^= p[i]; h *= 1099511628211ull; }
    return h;
}

void orc_set_threads(int n) { g_threads = n > 0 ? n : 1; }

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

}  // extern "C"
