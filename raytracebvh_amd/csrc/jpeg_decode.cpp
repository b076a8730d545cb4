// jpeg_decode.cpp -- native baseline JPEG decoding for the scene's diffuse textures.
//
// The reference loads map_Kd textures with DevIL (Image.cpp:35-61; Test.mtl:12 binds
// Balls.jpg), which decodes JPEG with the IJG library.  This is an independent decoder of
// the subset the reference's meshes need -- baseline sequential DCT (SOF0/SOF1), 8-bit,
// Huffman coding, 1 or 3 components, any sampling factors up to 2, restart intervals -- that
// computes what libjpeg's default decompression computes:
//   * the "islow" integer IDCT (13-bit constants, 2 extra bits in pass 1, the range-limit
//     table of jdmaster.c prepare_range_limit_table),
//   * "fancy" triangle-filter upsampling of subsampled chroma (h2v1 / h2v2 / h1v2, edge
//     rows and columns replicated),
//   * YCbCr -> RGB with the 16-bit fixed-point tables of jdcolor.c.
// Pinned bit for bit against PIL (libjpeg-turbo) on the reference's Balls.jpg and on
// synthetic images of every supported sampling (tests/test_host.py).  Rows are returned in
// file order (top row first), as DevIL hands JPEG rows to Image.cpp:48-49.
// Malformed input returns RTBVH_ERR_IO; every read is bounds-checked (fuzzed under
// ASan/UBSan, tools/sanitize_host.cpp).
#include "../../include/rtbvh.h"

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <new>
#include <vector>

namespace {

struct Huff {
    // canonical code tables: for code length l (1..16), codes [mincode[l], maxcode[l]] map to
    // values[valptr[l] + code - mincode[l]]
    int32_t mincode[17], maxcode[18], valptr[17];
    uint8_t values[256];
    bool present = false;
};

struct Comp {
    int id, h, v, tq, td = 0, ta = 0;
    int bw, bh;                  // blocks across / down in the padded component plane
    std::vector<uint8_t> plane;  // bw*8 x bh*8 samples
    int pred = 0;
};

constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint32_t acc = 0;
    int n = 0;
    bool marker = false;   // hit a marker: feed zeros (as libjpeg does at the end of a segment)
    int fill() {
        while (n <= 24) {
            uint32_t byte = 0;
            if (!marker && p < end) {
                byte = *p;
                if (byte == 0xFF) {
                    if (p + 1 < end && p[1] == 0x00) {
                        p += 2;
                    } else {
                        marker = true;
                        byte = 0;
                    }
                } else {
                    ++p;
                }
            }
            acc |= byte << (24 - n);
            n += 8;
        }
        return 0;
    }
    int bit() {
        if (n < 1) fill();
        const int b = (int)(acc >> 31);
        acc <<= 1;
        --n;
        return b;
    }
    int get(int k) {   // k <= 16
        if (k == 0) return 0;
        if (n < k) fill();
        const int v = (int)(acc >> (32 - k));
        acc <<= k;
        n -= k;
        return v;
    }
    void reset() {   // byte-align and skip the RSTn marker
        acc = 0;
        n = 0;
        marker = false;
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
        if (p + 1 < end) p += 2;
    }
};

bool decode_huff(Bits& b, const Huff& h, int& out) {
    int code = 0;
    for (int l = 1; l <= 16; l++) {
        code = (code << 1) | b.bit();
        if (code <= h.maxcode[l]) {
            const int idx = h.valptr[l] + code - h.mincode[l];
            if (idx < 0 || idx > 255) return false;
            out = h.values[idx];
            return true;
        }
    }
    return false;
}

inline int extend(int v, int t) { return t == 0 ? 0 : (v < (1 << (t - 1)) ? v - (1 << t) + 1 : v); }

// jidctint.c jpeg_idct_islow
constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
                  F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }

struct RangeLimit {   // jdmaster.c prepare_range_limit_table, the post-IDCT part (index & 1023)
    uint8_t post[1024];
    uint8_t simple[3 * 256];   // clamp to [0, 255] for x in [-256, 511] (colour conversion)
    RangeLimit() {
        for (int i = 0; i < 1024; i++) {
            int v;
            if (i < 128) v = i + 128;
            else if (i < 512) v = 255;
            else if (i < 896) v = 0;
            else v = i - 896;
            post[i] = (uint8_t)v;
        }
        for (int i = 0; i < 768; i++) simple[i] = (uint8_t)(i < 256 ? 0 : i < 512 ? i - 256 : 255);
    }
    uint8_t clamp(int x) const { return simple[x < -256 ? 0 : x > 511 ? 767 : x + 256]; }
};
// jdcolor.c build_ycc_rgb_table: built once, thread-safe (a function-local static)
struct YccTables {
    int cr_r[256], cb_b[256];
    int32_t cr_g[256], cb_g[256];
    YccTables() {
        const int32_t F1402 = (int32_t)(1.40200 * 65536 + 0.5), F1772 = (int32_t)(1.77200 * 65536 + 0.5);
        const int32_t F0714 = (int32_t)(0.71414 * 65536 + 0.5), F0344 = (int32_t)(0.34414 * 65536 + 0.5);
        for (int i = 0, x = -128; i < 256; i++, x++) {
            cr_r[i] = (int)((F1402 * x + 32768) >> 16);
            cb_b[i] = (int)((F1772 * x + 32768) >> 16);
            cr_g[i] = -F0714 * x;
            cb_g[i] = -F0344 * x + 32768;
        }
    }
};
const YccTables& ycc_tables() {
    static const YccTables t;
    return t;
}

const RangeLimit& range_limit() {
    static const RangeLimit r;
    return r;
}

void idct_islow(const int16_t* coef /* natural order */, const uint16_t* q, uint8_t* out, int stride) {
    int32_t ws[64];
    for (int c = 0; c < 8; c++) {
        const int16_t* in = coef + c;
        const uint16_t* qq = q + c;
        if (!in[8] && !in[16] && !in[24] && !in[32] && !in[40] && !in[48] && !in[56]) {
            const int32_t dc = (int32_t)in[0] * qq[0] * (1 << PASS1_BITS);
            for (int r = 0; r < 8; r++) ws[8 * r + c] = dc;
            continue;
        }
        int64_t z2 = (int32_t)in[16] * qq[16], z3 = (int32_t)in[48] * qq[48];
        int64_t z1 = (z2 + z3) * F0541;
        int64_t tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
        z2 = (int32_t)in[0] * qq[0];
        z3 = (int32_t)in[32] * qq[32];
        int64_t tmp0 = (z2 + z3) * (1 << CONST_BITS), tmp1 = (z2 - z3) * (1 << CONST_BITS);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = (int32_t)in[56] * qq[56];
        tmp1 = (int32_t)in[40] * qq[40];
        tmp2 = (int32_t)in[24] * qq[24];
        tmp3 = (int32_t)in[8] * qq[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1175;
        tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
        z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        const int n = CONST_BITS - PASS1_BITS;
        ws[c] = descale(tmp10 + tmp3, n);
        ws[56 + c] = descale(tmp10 - tmp3, n);
        ws[8 + c] = descale(tmp11 + tmp2, n);
        ws[48 + c] = descale(tmp11 - tmp2, n);
        ws[16 + c] = descale(tmp12 + tmp1, n);
        ws[40 + c] = descale(tmp12 - tmp1, n);
        ws[24 + c] = descale(tmp13 + tmp0, n);
        ws[32 + c] = descale(tmp13 - tmp0, n);
    }
    const uint8_t* rl = range_limit().post;
    const int n2 = CONST_BITS + PASS1_BITS + 3;
    for (int r = 0; r < 8; r++) {
        const int32_t* w = ws + 8 * r;
        uint8_t* o = out + (size_t)r * stride;
        if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
            const uint8_t v = rl[descale(w[0], PASS1_BITS + 3) & 1023];
            for (int c = 0; c < 8; c++) o[c] = v;
            continue;
        }
        int64_t z2 = w[2], z3 = w[6];
        int64_t z1 = (z2 + z3) * F0541;
        int64_t tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
        int64_t tmp0 = ((int64_t)w[0] + w[4]) * (1 << CONST_BITS), tmp1 = ((int64_t)w[0] - w[4]) * (1 << CONST_BITS);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F1175;
        tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
        z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
        o[0] = rl[descale(tmp10 + tmp3, n2) & 1023];
        o[7] = rl[descale(tmp10 - tmp3, n2) & 1023];
        o[1] = rl[descale(tmp11 + tmp2, n2) & 1023];
        o[6] = rl[descale(tmp11 - tmp2, n2) & 1023];
        o[2] = rl[descale(tmp12 + tmp1, n2) & 1023];
        o[5] = rl[descale(tmp12 - tmp1, n2) & 1023];
        o[3] = rl[descale(tmp13 + tmp0, n2) & 1023];
        o[4] = rl[descale(tmp13 - tmp0, n2) & 1023];
    }
}

// jdsample.c fancy upsampling of one component to the full image size (W x H), from its
// downsampled plane (dw x dh valid samples, row stride `stride`); hs, vs in {1, 2}
void upsample(const Comp& c, int dw, int dh, int hs, int vs, int W, int H, std::vector<uint8_t>& out) {
    out.assign((size_t)W * H, 0);
    const int stride = c.bw * 8;
    auto at = [&](int x, int y) -> int { return c.plane[(size_t)y * stride + x]; };
    // horizontal 2x of a row of column sums (h2v1_fancy_upsample / h2v2 inner loop)
    std::vector<int> row((size_t)dw), tmp((size_t)2 * dw);
    for (int oy = 0; oy < H; oy++) {
        if (vs == 1) {
            const int y = oy < dh ? oy : dh - 1;
            if (hs == 1) {
                for (int x = 0; x < W; x++) out[(size_t)oy * W + x] = (uint8_t)at(x < dw ? x : dw - 1, y);
                continue;
            }
            // h2v1: out[2i] = (3 in[i] + in[i-1] + 1) >> 2, out[2i+1] = (3 in[i] + in[i+1] + 2) >> 2
            for (int i = 0; i < dw; i++) {
                const int cur = at(i, y);
                if (dw == 1) {
                    tmp[0] = tmp[1] = cur;
                    break;
                }
                tmp[2 * i] = i == 0 ? cur : (cur * 3 + at(i - 1, y) + 1) >> 2;
                tmp[2 * i + 1] = i == dw - 1 ? cur : (cur * 3 + at(i + 1, y) + 2) >> 2;
            }
            for (int x = 0; x < W; x++) out[(size_t)oy * W + x] = (uint8_t)tmp[x < 2 * dw ? x : 2 * dw - 1];
            continue;
        }
        // vs == 2: output row oy comes from input row y = oy / 2 and its neighbour above (even
        // oy) or below (odd oy), edges replicated
        const int y = (oy >> 1) < dh ? (oy >> 1) : dh - 1;
        const int yn = (oy & 1) ? (y + 1 < dh ? y + 1 : dh - 1) : (y > 0 ? y - 1 : 0);
        for (int i = 0; i < dw; i++) row[i] = at(i, y) * 3 + at(i, yn);
        if (hs == 1) {   // h1v2_fancy_upsample: (3 * near + far + 1 or 2) >> 2
            const int bias = (oy & 1) ? 2 : 1;
            for (int x = 0; x < W; x++) out[(size_t)oy * W + x] = (uint8_t)((row[x < dw ? x : dw - 1] + bias) >> 2);
            continue;
        }
        // h2v2_fancy_upsample
        if (dw == 1) {
            tmp[0] = tmp[1] = (row[0] * 4 + 8) >> 4;
        } else {
            for (int i = 0; i < dw; i++) {
                const int cs = row[i];
                if (i == 0) {
                    tmp[0] = (cs * 4 + 8) >> 4;
                    tmp[1] = (cs * 3 + row[1] + 7) >> 4;
                } else if (i == dw - 1) {
                    tmp[2 * i] = (cs * 3 + row[i - 1] + 8) >> 4;
                    tmp[2 * i + 1] = (cs * 4 + 7) >> 4;
                } else {
                    tmp[2 * i] = (cs * 3 + row[i - 1] + 8) >> 4;
                    tmp[2 * i + 1] = (cs * 3 + row[i + 1] + 7) >> 4;
                }
            }
        }
        for (int x = 0; x < W; x++) out[(size_t)oy * W + x] = (uint8_t)tmp[x < 2 * dw ? x : 2 * dw - 1];
    }
}

bool decode(const uint8_t* data, size_t size, uint32_t& W_out, uint32_t& H_out, std::vector<uint8_t>& rgba) {
    if (size < 4 || data[0] != 0xFF || data[1] != 0xD8) return false;
    uint16_t qt[4][64];
    bool qt_present[4] = {};
    Huff hdc[4], hac[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, restart = 0, hmax = 1, vmax = 1;
    bool frame = false;
    size_t pos = 2;
    auto u16 = [&](size_t at) { return (int)data[at] << 8 | data[at + 1]; };
    while (pos + 4 <= size) {
        if (data[pos] != 0xFF) return false;
        const int m = data[pos + 1];
        if (m == 0xFF) { ++pos; continue; }   // fill bytes
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) { pos += 2; continue; }
        if (m == 0xD9) break;
        const int len = u16(pos + 2);
        if (len < 2 || pos + 2 + (size_t)len > size) return false;
        const uint8_t* seg = data + pos + 4;
        const int sl = len - 2;
        if (m == 0xDB) {   // DQT
            int k = 0;
            while (k < sl) {
                const int pq = seg[k] >> 4, tq = seg[k] & 15;
                if (tq > 3 || pq > 1 || k + 1 + 64 * (pq + 1) > sl) return false;
                for (int i = 0; i < 64; i++)
                    qt[tq][kZigzag[i]] = pq ? (uint16_t)(seg[k + 1 + 2 * i] << 8 | seg[k + 2 + 2 * i]) : seg[k + 1 + i];
                qt_present[tq] = true;
                k += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xC4) {   // DHT
            int k = 0;
            while (k < sl) {
                if (k + 17 > sl) return false;
                const int tc = seg[k] >> 4, th = seg[k] & 15;
                if (tc > 1 || th > 3) return false;
                Huff& h = tc ? hac[th] : hdc[th];
                int total = 0;
                for (int l = 1; l <= 16; l++) total += seg[k + l];
                if (total > 256 || k + 17 + total > sl) return false;
                memcpy(h.values, seg + k + 17, (size_t)total);
                int code = 0, vp = 0;
                for (int l = 1; l <= 16; l++) {
                    const int cnt = seg[k + l];
                    h.valptr[l] = vp;
                    h.mincode[l] = code;
                    code += cnt;
                    vp += cnt;
                    h.maxcode[l] = cnt ? code - 1 : -1;
                    code <<= 1;
                }
                h.maxcode[17] = 0x7FFFFFFF;
                h.present = true;
                k += 17 + total;
            }
        } else if (m == 0xC0 || m == 0xC1) {   // SOF0 / SOF1: baseline / extended sequential Huffman
            if (sl < 6 || seg[0] != 8) return false;
            H = u16(pos + 5);
            W = u16(pos + 7);
            const int nc = seg[5];
            if (W <= 0 || H <= 0 || W > 65535 || H > 65535 || (nc != 1 && nc != 3) || sl < 6 + 3 * nc) return false;
            comps.assign(nc, Comp{});
            for (int c = 0; c < nc; c++) {
                comps[c].id = seg[6 + 3 * c];
                comps[c].h = seg[7 + 3 * c] >> 4;
                comps[c].v = seg[7 + 3 * c] & 15;
                comps[c].tq = seg[8 + 3 * c];
                if (comps[c].h < 1 || comps[c].h > 2 || comps[c].v < 1 || comps[c].v > 2 || comps[c].tq > 3)
                    return false;
                hmax = comps[c].h > hmax ? comps[c].h : hmax;
                vmax = comps[c].v > vmax ? comps[c].v : vmax;
            }
            frame = true;
        } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return false;   // progressive / lossless / arithmetic: not the reference's files
        } else if (m == 0xDD) {
            if (sl < 2) return false;
            restart = u16(pos + 4);
        } else if (m == 0xDA) {   // SOS: decode the (single, interleaved or not) scan
            if (!frame || sl < 1) return false;
            const int ns = seg[0];
            if (ns < 1 || ns > (int)comps.size() || sl < 1 + 2 * ns + 3) return false;
            std::vector<int> sc(ns);
            for (int s = 0; s < ns; s++) {
                const int cid = seg[1 + 2 * s];
                int ci = -1;
                for (int c = 0; c < (int)comps.size(); c++)
                    if (comps[c].id == cid) ci = c;
                if (ci < 0) return false;
                comps[ci].td = seg[2 + 2 * s] >> 4;
                comps[ci].ta = seg[2 + 2 * s] & 15;
                if (comps[ci].td > 3 || comps[ci].ta > 3 || !hdc[comps[ci].td].present || !hac[comps[ci].ta].present ||
                    !qt_present[comps[ci].tq])
                    return false;
                sc[s] = ci;
            }
            const int mcux = (W + 8 * hmax - 1) / (8 * hmax), mcuy = (H + 8 * vmax - 1) / (8 * vmax);
            for (auto& c : comps) {
                if (c.plane.empty()) {
                    c.bw = mcux * c.h;
                    c.bh = mcuy * c.v;
                    c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
                }
                c.pred = 0;
            }
            Bits bits{data + pos + 2 + len, data + size};
            int16_t blk[64];
            auto block = [&](Comp& c, int bx, int by) -> bool {
                memset(blk, 0, sizeof(blk));
                int t;
                if (!decode_huff(bits, hdc[c.td], t) || t > 11) return false;
                c.pred += extend(bits.get(t), t);   // |diff| < 2^11 per block
                if (c.pred < -32768 || c.pred > 32767) return false;   // no 16-bit DC: malformed
                blk[0] = (int16_t)c.pred;
                for (int k = 1; k < 64;) {
                    int rs;
                    if (!decode_huff(bits, hac[c.ta], rs)) return false;
                    const int r = rs >> 4, s = rs & 15;
                    if (s == 0) {
                        if (r != 15) break;   // EOB
                        k += 16;
                        continue;
                    }
                    k += r;
                    if (k > 63) return false;
                    blk[kZigzag[k]] = (int16_t)extend(bits.get(s), s);
                    ++k;
                }
                if (bx < 0 || by < 0 || bx >= c.bw || by >= c.bh) return true;
                const int stride = c.bw * 8;
                idct_islow(blk, qt[c.tq], &c.plane[(size_t)by * 8 * stride + (size_t)bx * 8], stride);
                return true;
            };
            int todo = restart;
            if (ns == 1) {   // non-interleaved: the component's own blocks, ceil(comp size / 8)
                Comp& c = comps[sc[0]];
                const int cw = (W * c.h + hmax - 1) / hmax, ch = (H * c.v + vmax - 1) / vmax;
                const int nbx = (cw + 7) / 8, nby = (ch + 7) / 8;
                for (int by = 0; by < nby; by++)
                    for (int bx = 0; bx < nbx; bx++) {
                        if (restart && todo == 0) {
                            bits.reset();
                            c.pred = 0;
                            todo = restart;
                        }
                        if (!block(c, bx, by)) return false;
                        --todo;
                    }
            } else {
                for (int my = 0; my < mcuy; my++)
                    for (int mx = 0; mx < mcux; mx++) {
                        if (restart && todo == 0) {
                            bits.reset();
                            for (auto& c : comps) c.pred = 0;
                            todo = restart;
                        }
                        for (int s = 0; s < ns; s++) {
                            Comp& c = comps[sc[s]];
                            for (int v = 0; v < c.v; v++)
                                for (int h = 0; h < c.h; h++)
                                    if (!block(c, mx * c.h + h, my * c.v + v)) return false;
                        }
                        --todo;
                    }
            }
            // resume at the next marker after the entropy-coded data
            const uint8_t* p = bits.p;
            while (p + 1 < data + size && !(p[0] == 0xFF && p[1] != 0x00 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
            pos = (size_t)(p - data);
            continue;
        }
        pos += 2 + (size_t)len;
    }
    if (!frame || comps.empty()) return false;
    for (auto& c : comps)
        if (c.plane.empty()) return false;
    std::vector<std::vector<uint8_t>> full(comps.size());
    for (size_t k = 0; k < comps.size(); k++) {
        const Comp& c = comps[k];
        const int hs = hmax / c.h, vs = vmax / c.v;
        if (hmax % c.h || vmax % c.v) return false;
        const int dw = (W * c.h + hmax - 1) / hmax, dh = (H * c.v + vmax - 1) / vmax;
        upsample(c, dw, dh, hs, vs, W, H, full[k]);
    }
    // jdcolor.c ycc_rgb_convert (SCALEBITS 16); grayscale: R = G = B = Y
    const YccTables& yt = ycc_tables();
    const RangeLimit& rl = range_limit();
    rgba.assign((size_t)W * H * 4, 255);
    for (size_t i = 0; i < (size_t)W * H; i++) {
        uint8_t* o = &rgba[4 * i];
        const int y = full[0][i];
        if (comps.size() == 1) {
            o[0] = o[1] = o[2] = (uint8_t)y;
            continue;
        }
        const int cb = full[1][i], cr = full[2][i];
        o[0] = rl.clamp(y + yt.cr_r[cr]);
        o[1] = rl.clamp(y + (int)((yt.cb_g[cb] + yt.cr_g[cr]) >> 16));
        o[2] = rl.clamp(y + yt.cb_b[cb]);
    }
    W_out = (uint32_t)W;
    H_out = (uint32_t)H;
    return true;
}

bool read_file(const char* path, std::vector<uint8_t>& b) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    b.assign((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return true;
}

}  // namespace

extern "C" {

rtbvh_status rtbvh_texture_decode_jpeg(const uint8_t* data, size_t size, rtbvh_texture* out) {
    if (!data || !out) return RTBVH_ERR_INVALID_ARG;
    out->width = out->height = 0;
    out->rgba8 = nullptr;
    try {
        std::vector<uint8_t> rgba;
        uint32_t W = 0, H = 0;
        if (!decode(data, size, W, H, rgba)) return RTBVH_ERR_IO;
        uint8_t* buf = static_cast<uint8_t*>(malloc(rgba.size()));
        if (!buf) return RTBVH_ERR_OOM;
        memcpy(buf, rgba.data(), rgba.size());
        out->width = W;
        out->height = H;
        out->rgba8 = buf;
        return RTBVH_OK;
    } catch (const std::bad_alloc&) {
        return RTBVH_ERR_OOM;
    }
}

rtbvh_status rtbvh_texture_load_jpeg(const char* path, rtbvh_texture* out) {
    if (!path || !out) return RTBVH_ERR_INVALID_ARG;
    out->width = out->height = 0;
    out->rgba8 = nullptr;
    std::vector<uint8_t> b;
    try {
        if (!read_file(path, b)) return RTBVH_ERR_IO;
    } catch (const std::bad_alloc&) {
        return RTBVH_ERR_OOM;
    }
    return rtbvh_texture_decode_jpeg(b.data(), b.size(), out);
}

rtbvh_status rtbvh_texture_load(const char* path, rtbvh_texture* out) {
    if (!path || !out) return RTBVH_ERR_INVALID_ARG;
    out->width = out->height = 0;
    out->rgba8 = nullptr;
    std::ifstream f(path, std::ios::binary);
    if (!f) return RTBVH_ERR_IO;
    unsigned char magic[2] = {0, 0};
    f.read(reinterpret_cast<char*>(magic), 2);
    if (magic[0] == 'B' && magic[1] == 'M') return rtbvh_texture_load_bmp(path, out);
    if (magic[0] == 0xFF && magic[1] == 0xD8) return rtbvh_texture_load_jpeg(path, out);
    return RTBVH_ERR_IO;
}

}  // extern "C"
