#pragma once
// pb_bin.h -- the binned primary pass's two bin passes (trace.hip k_pb_bin), as a block function
// over a block index, so that build.hip can run them in one launch beside the build's crossing
// nodes' QNodes (rtbvh_compute_bvh: k_pb_count_late).  Included inside each file's
// anonymous namespace, after its BLOCK constant.
// k of band b in this rank's deal (its compact rows k*8 .. k*8+7), or -1 when another rank has it
__device__ __forceinline__ int pb_band_pos(const TraceArgs& a, uint32_t b) {
    if (a.band_slots) {
        const uint32_t s = a.band_slots[b];
        return (s >> 24) == a.rank ? (int)(s & 0xFFFFFFu) : -1;
    }
    return b % a.nranks == a.rank ? (int)(b / a.nranks) : -1;
}
// the rank's compact rows among image rows [y0, y1] (an order-preserving map, so a range [c0, c1]); pos(b) is
// pb_band_pos(a, b), from the block's LDS copy of the deal (pb_bin_block)
template <class Pos>
__device__ __forceinline__ void pb_rows(const TraceArgs& a, int y0, int y1, int& c0, int& c1, const Pos& pos) {
    if (a.nranks == 1 || y0 > y1) { c0 = y0; c1 = y1; return; }
    c0 = 1; c1 = 0;
    const int b0 = y0 >> 3, b1 = y1 >> 3;
    int b = b0;
    for (; b <= b1; b++) {
        const int k = pos((uint32_t)b);
        if (k >= 0) { c0 = b == b0 ? k * 8 + (y0 & 7) : k * 8; break; }
    }
    if (b > b1) return;   // none of the bands is the rank's
    for (b = b1; b >= b0; b--) {
        const int k = pos((uint32_t)b);
        if (k >= 0) { c1 = b == b1 ? k * 8 + (y1 & 7) : k * 8 + 7; break; }
    }
}

// pass 1 (FILL false): leaf j's footprint -- its pixel columns and the rank's compact rows, min.z,
// the general bit -- and its count in every (screen tile, depth bucket) bin it covers; pass 2 (FILL
// true): the footprint with j into those bins at the scanned offsets (16-B entries: the binned pass
// streams them with no dependent fetch).  A workgroup takes PB_LEAVES consecutive sorted leaves --
// neighbours in space, sharing their bins -- and counts them per bin in an LDS table first, so the
// global atomics are one per bin and workgroup instead of one per wave and bin; in pass 2 the
// table's returned bases and LDS cursors place every entry.  A bin the full table cannot hold takes
// a global atomic of its own (correct either way).
// (PB_LEAVES, rtbvh_internal.h: leaves per workgroup, 4 per thread)
constexpr uint32_t PB_HASH = 1024;        // LDS table slots
// N > 1: the deal's band positions copied to LDS per block (frames of up to 8 * PB_LDS_BANDS rows; taller ones
// read the deal from memory): pb_rows walks a footprint's bands one by one, and from memory each step was a
// dependent L2 load (the count pass of an N = 8 rank took longer than N = 1's, which bins 8x the entries)
constexpr uint32_t PB_LDS_BANDS = 2048;
constexpr uint32_t PB_EMPTY = 0xFFFFFFFFu;
__device__ __forceinline__ int pb_slot_of(uint32_t* h_key, uint32_t key, bool insert) {
    uint32_t h = (key * 2654435761u) >> 22;   // 10 bits
    for (int probe = 0; probe < 32; probe++) {
        const uint32_t k = insert ? atomicCAS(&h_key[h], PB_EMPTY, key) : h_key[h];
        if (k == key || (insert && k == PB_EMPTY)) return (int)h;
        if (!insert && k == PB_EMPTY) return -1;
        h = (h + 1) & (PB_HASH - 1);
    }
    return -1;
}
// (both passes derive the frame's footprint from the build's: storing it in the first pass for the
// second was +-0, C5 A/B 0.952 / 0.952 ms, for 16 B per leaf of memory)
template <bool FILL>
__device__ __forceinline__ void pb_bin_block(const TraceArgs& a, uint32_t bid, uint32_t* __restrict__ off,
                                             uint32_t* __restrict__ cur, uint4* __restrict__ bins, uint32_t cap,
                                             uint32_t ntx) {
    __shared__ uint32_t h_key[PB_HASH], h_cnt[PB_HASH], h_base[FILL ? PB_HASH : 1];
    __shared__ uint16_t s_band[PB_LDS_BANDS];   // N > 1: pb_band_pos of every band, 0xFFFF for another rank's
    // N > 1 (a.pb_list): the count pass appends the rank's leaves to one of PB_LISTS lists (count block bid to
    // list bid % PB_LISTS: one atomic per block on its list's counter), and fill block bid takes the 1024
    // entries at (bid / PB_LISTS) * 1024 of list bid % PB_LISTS -- blocks past a list's end return at once
    uint32_t* const list = a.pb_list;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t lk = bid % PB_LISTS, rcap = pb_list_cap(a.T);
    uint32_t* const lcnt = list ? list + PB_LIST_STRIDE * lk : nullptr;
    uint32_t* const lent = list ? list + PB_LISTS * PB_LIST_STRIDE + (size_t)lk * rcap : nullptr;
    const uint32_t nlist = FILL && list ? min(*lcnt, rcap) : 0u;
    const uint32_t lbase = (bid / PB_LISTS) * PB_LEAVES;
    if (FILL && list && lbase >= nlist) return;   // (uniform over the block)
    for (uint32_t i = threadIdx.x; i < PB_HASH; i += BLOCK) { h_key[i] = PB_EMPTY; h_cnt[i] = 0; }
    const uint32_t nbands = (a.H + 7) >> 3;
    const bool lds_bands = a.nranks > 1 && nbands <= PB_LDS_BANDS;
    if (lds_bands)
        for (uint32_t b = threadIdx.x; b < nbands; b += BLOCK) {
            const int k = pb_band_pos(a, b);
            s_band[b] = k < 0 ? (uint16_t)0xFFFFu : (uint16_t)k;
        }
    __syncthreads();
    constexpr uint32_t LPT = PB_LEAVES / BLOCK;
    uint4 f[LPT];
    uint32_t zb[LPT], jj[LPT];
    const float zlo = a.rootbox[6], zhi = a.rootbox[7];   // the leaves' depth range (= the root box's)
#pragma unroll
    for (uint32_t i = 0; i < LPT; i++) {
        uint32_t j = bid * PB_LEAVES + i * BLOCK + threadIdx.x;
        if (FILL && list) {
            const uint32_t e = lbase + i * BLOCK + threadIdx.x;
            j = e < nlist ? lent[e] : a.T;
        }
        jj[i] = j;
        f[i] = make_uint4(1, 1, 0, 0);   // empty: x0 = 1 > x1 = 0
        if (j < a.T) {
            {   // the build's footprint (pixel offsets from the frame centre) on this frame and rank
                const uint4 l = a.lfp[j];
                const int hw = (int)(a.W >> 1), hh = (int)(a.H >> 1);
                const int x0 = max((int)(int16_t)(l.x & 0xFFFFu) + hw, 0), x1 = min((int)(int16_t)(l.x >> 16) + hw, (int)a.W - 1);
                const int y0 = max((int)(int16_t)(l.y & 0xFFFFu) + hh, 0), y1 = min((int)(int16_t)(l.y >> 16) + hh, (int)a.H - 1);
                int c0 = 1, c1 = 0;
                if (x0 <= x1) {
                    if (lds_bands)
                        pb_rows(a, y0, y1, c0, c1, [&](uint32_t b) {
                            const uint32_t v = s_band[b];
                            return v == 0xFFFFu ? -1 : (int)v;
                        });
                    else
                        pb_rows(a, y0, y1, c0, c1, [&](uint32_t b) { return pb_band_pos(a, b); });
                }
                if (x0 <= x1 && c0 <= c1)
                    f[i] = make_uint4((uint32_t)x0 | (uint32_t)x1 << 16, (uint32_t)c0 | (uint32_t)c1 << 16, l.z, l.w);
            }
        }
        // the depth bucket of min.z in the root box's depth range (general boxes first: they always test)
        const float u = (__uint_as_float(f[i].z) - zlo) / (zhi - zlo) * (float)PB_NZ;
        zb[i] = f[i].w ? 0u : (uint32_t)fminf(fmaxf(u, 0.f), (float)(PB_NZ - 1));   // NaN: 0
    }
    if (!FILL && list) {   // the rank's leaves (a footprint in its rows) appended to list lk: one atomic a block
        __shared__ uint32_t s_wn[BLOCK / 64], s_base;
        uint32_t mine = 0;
#pragma unroll
        for (uint32_t i = 0; i < LPT; i++) mine += (f[i].x & 0xFFFFu) <= (f[i].x >> 16) ? 1u : 0u;
        uint32_t x = mine;   // inclusive scan over the wave
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t y = __shfl_up(x, dd, 64);
            if ((int)lane >= dd) x += y;
        }
        if (lane == 63) s_wn[wv] = x;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (uint32_t k = 0; k < BLOCK / 64; k++) { const uint32_t v = s_wn[k]; s_wn[k] = t; t += v; }
            s_base = t ? atomicAdd(lcnt, t) : 0u;
        }
        __syncthreads();
        uint32_t at = s_base + s_wn[wv] + x - mine;
#pragma unroll
        for (uint32_t i = 0; i < LPT; i++)
            if ((f[i].x & 0xFFFFu) <= (f[i].x >> 16)) lent[at++] = jj[i];
    }
    // the (leaf, bin) pairs of item i, visited by `body(key)`
    const auto pairs = [&](uint32_t i, auto&& body) {
        const uint32_t x0 = f[i].x & 0xFFFFu, x1 = f[i].x >> 16, c0 = f[i].y & 0xFFFFu, c1 = f[i].y >> 16;
        if (x0 > x1 || c0 > c1) return;
        for (uint32_t ty = c0 / PB_TILE; ty <= c1 / PB_TILE; ty++)
            for (uint32_t tx = x0 / PB_TILE; tx <= x1 / PB_TILE; tx++) body((ty * ntx + tx) * PB_NZ + zb[i]);
    };
    // counts per bin in the table (or straight to the global count when the table is full)
#pragma unroll
    for (uint32_t i = 0; i < LPT; i++)
        pairs(i, [&](uint32_t key) {
            const int sl = pb_slot_of(h_key, key, true);
            if (sl >= 0) atomicAdd(&h_cnt[sl], 1u);
            else if (!FILL) atomicAdd(&off[key], 1u);
        });
    __syncthreads();
    for (uint32_t sl = threadIdx.x; sl < PB_HASH; sl += BLOCK) {
        const uint32_t key = h_key[sl];
        if (key == PB_EMPTY) continue;
        if (!FILL) {
            atomicAdd(&off[key], h_cnt[sl]);
        } else {
            h_base[sl] = off[key] + atomicAdd(&cur[key], h_cnt[sl]);
            h_cnt[sl] = 0;
        }
    }
    if (!FILL) return;
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < LPT; i++) {
        const uint32_t j = jj[i];
        const uint4 entry = make_uint4(f[i].x, f[i].y, f[i].z, j | (f[i].w ? LEAF_BIT : 0u));
        pairs(i, [&](uint32_t key) {
            const int sl = pb_slot_of(h_key, key, false);
            const uint32_t e = sl >= 0 ? h_base[sl] + atomicAdd(&h_cnt[sl], 1u) : off[key] + atomicAdd(&cur[key], 1u);
            if (e < cap) bins[e] = entry;
        });
    }
}
