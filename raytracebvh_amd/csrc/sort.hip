// sort.hip -- stable LSD radix sort of (key, value) pairs for gfx950.
//
// Replaces RadixSortP1.hlsl (1-bit flags + a 256-wide Blelloch scan per
// group) and RadixSortP2.hlsl (a serial O(G) sum of group counts by thread 0,
// then a scatter of whole 44-B nodes), run 32 times by Graphics.cpp:735-754.
// Here: RADIX_BITS-bit digits (8: 4 passes for 30-bit codes; 10: 3), 8-B (key, value)
// payloads, and per pass a reduce-then-scan over 4096-key tiles:
//   upsweep   tile digit histogram in LDS         -> counts[digit][tile]
//   scan      one workgroup per digit row          -> exclusive tile offsets + digit totals
//   downsweep stable wave64 ranking (8 ballots per key, per-wave LDS digit
//             counters), LDS staging so each digit's run is written contiguously.
// No inter-workgroup communication inside a launch (kernel boundaries order the
// three phases), so nothing here depends on XCD placement.
#include "rtbvh_internal.h"

namespace rtbvh {
namespace {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_exclusive_scan256(uint32_t v, uint32_t* s_wave /*[4]*/, uint32_t* total) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += t;
    }
    if (lane == 63) s_wave[w] = incl;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        uint32_t x = s_wave[k];
        if (k < w) wpre += x;
        tot += x;
    }
    __syncthreads();
    if (total) *total = tot;
    return wpre + incl - v;
}

__global__ __launch_bounds__(SORT_BLOCK) void k_upsweep(const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift,
                                                        uint32_t* __restrict__ counts, uint32_t ntiles) {
    __shared__ uint32_t hist[4][RADIX];
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    for (uint32_t k = tid; k < 4 * RADIX; k += SORT_BLOCK) (&hist[0][0])[k] = 0;
    __syncthreads();
    const uint32_t tile = blockIdx.x;
    const size_t base = (size_t)tile * SORT_TILE;
    if (base + SORT_TILE <= n) {
        const uint4* k4 = reinterpret_cast<const uint4*>(keys + base);
#pragma unroll
        for (uint32_t it = 0; it < SORT_ITEMS / 4; it++) {
            uint4 v = k4[it * SORT_BLOCK + tid];
            atomicAdd(&hist[w][(v.x >> shift) & (RADIX - 1)], 1u);
            atomicAdd(&hist[w][(v.y >> shift) & (RADIX - 1)], 1u);
            atomicAdd(&hist[w][(v.z >> shift) & (RADIX - 1)], 1u);
            atomicAdd(&hist[w][(v.w >> shift) & (RADIX - 1)], 1u);
        }
    } else {
        for (uint32_t it = 0; it < SORT_ITEMS; it++) {
            size_t i = base + it * SORT_BLOCK + tid;
            if (i < n) atomicAdd(&hist[w][(keys[i] >> shift) & (RADIX - 1)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = tid; d < RADIX; d += SORT_BLOCK)
        counts[(size_t)d * ntiles + tile] = hist[0][d] + hist[1][d] + hist[2][d] + hist[3][d];
}

// one workgroup per digit: exclusive scan of counts[digit][0..ntiles) in place
__global__ __launch_bounds__(SORT_BLOCK) void k_scan_rows(uint32_t* __restrict__ counts, uint32_t ntiles,
                                                          uint32_t* __restrict__ digit_totals) {
    __shared__ uint32_t s_wave[4];
    uint32_t* row = counts + (size_t)blockIdx.x * ntiles;
    const uint32_t tid = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < ntiles; base += SORT_BLOCK * 8) {
        // each thread owns 8 consecutive entries of this chunk
        uint32_t v[8], sum = 0;
        const uint32_t b0 = base + tid * 8;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            v[k] = (b0 + k < ntiles) ? row[b0 + k] : 0u;
            sum += v[k];
        }
        uint32_t tot;
        uint32_t pre = block_exclusive_scan256(sum, s_wave, &tot) + carry;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (b0 + k < ntiles) row[b0 + k] = pre;
            pre += v[k];
        }
        carry += tot;
    }
    if (tid == 0) digit_totals[blockIdx.x] = carry;
}

__global__ __launch_bounds__(SORT_BLOCK) void k_downsweep(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                          uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                          uint32_t n, uint32_t shift, const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ digit_totals, uint32_t ntiles) {
    __shared__ uint32_t s_keys[SORT_TILE];
    __shared__ uint32_t s_vals[SORT_TILE];
    __shared__ uint32_t s_whist[4][RADIX];
    __shared__ uint32_t s_lstart[RADIX];
    __shared__ uint32_t s_gstart[RADIX];
    __shared__ uint32_t s_wave[4];

    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const size_t base = (size_t)tile * SORT_TILE;
    const uint32_t valid = (uint32_t)min((size_t)SORT_TILE, (size_t)n - base);

    // global start of each digit for this tile = sum of lower digits + this digit's earlier tiles
    // (thread tid owns digits [RPT tid, RPT tid + RPT))
    constexpr uint32_t RPT = RADIX / SORT_BLOCK;
    static_assert(RADIX % SORT_BLOCK == 0, "whole digits per thread");
    {
        uint32_t g[RPT], sum = 0;
#pragma unroll
        for (uint32_t r = 0; r < RPT; r++) { g[r] = digit_totals[RPT * tid + r]; sum += g[r]; }
        uint32_t gbase = block_exclusive_scan256(sum, s_wave, nullptr);
#pragma unroll
        for (uint32_t r = 0; r < RPT; r++) {
            s_gstart[RPT * tid + r] = gbase + counts[(size_t)(RPT * tid + r) * ntiles + tile];
            gbase += g[r];
        }
    }
    for (uint32_t k = tid; k < 4 * RADIX; k += SORT_BLOCK) (&s_whist[0][0])[k] = 0;
    __syncthreads();

    // wave w owns tile positions [w*1024, (w+1)*1024); item it of lane l = position w*1024 + it*64 + l
    uint32_t key[SORT_ITEMS], val[SORT_ITEMS], rank[SORT_ITEMS];
    const size_t wbase = base + (size_t)w * (SORT_TILE / 4);
#pragma unroll
    for (uint32_t it = 0; it < SORT_ITEMS; it++) {
        const uint32_t pos = w * (SORT_TILE / 4) + it * 64 + lane;
        const bool ok = pos < valid;
        key[it] = ok ? kin[wbase + it * 64 + lane] : 0xFFFFFFFFu;
        val[it] = ok ? vin[wbase + it * 64 + lane] : 0u;
    }
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (uint32_t it = 0; it < SORT_ITEMS; it++) {
        const uint32_t pos = w * (SORT_TILE / 4) + it * 64 + lane;
        // invalid items rank as digit RADIX-1 after every valid key of the tile
        const uint32_t d = pos < valid ? (key[it] >> shift) & (RADIX - 1) : RADIX - 1;
        uint64_t peers = ~0ull;
#pragma unroll
        for (uint32_t b = 0; b < RADIX_BITS; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t before = __popcll(peers & lt_mask);
        const uint32_t cnt = __popcll(peers);
        const uint32_t prev = s_whist[w][d];
        if (before == 0) s_whist[w][d] = prev + cnt;   // lowest lane of the peer group
        rank[it] = prev + before;
    }
    __syncthreads();
    // tile-local digit starts and per-wave offsets
    {
        uint32_t c[RPT][4], sum = 0;
#pragma unroll
        for (uint32_t r = 0; r < RPT; r++) {
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) { c[r][k] = s_whist[k][RPT * tid + r]; sum += c[r][k]; }
        }
        uint32_t lstart = block_exclusive_scan256(sum, s_wave, nullptr);   // (its barriers: all reads done)
#pragma unroll
        for (uint32_t r = 0; r < RPT; r++) {
            const uint32_t d = RPT * tid + r;
            s_lstart[d] = lstart;
            s_whist[0][d] = lstart;
            s_whist[1][d] = lstart + c[r][0];
            s_whist[2][d] = lstart + c[r][0] + c[r][1];
            s_whist[3][d] = lstart + c[r][0] + c[r][1] + c[r][2];
            lstart += c[r][0] + c[r][1] + c[r][2] + c[r][3];
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < SORT_ITEMS; it++) {
        const uint32_t pos = w * (SORT_TILE / 4) + it * 64 + lane;
        const uint32_t d = pos < valid ? (key[it] >> shift) & (RADIX - 1) : RADIX - 1;
        const uint32_t lpos = s_whist[w][d] + rank[it];
        s_keys[lpos] = key[it];
        s_vals[lpos] = val[it];
    }
    __syncthreads();
    for (uint32_t j = tid; j < valid; j += SORT_BLOCK) {
        const uint32_t k = s_keys[j];
        const uint32_t d = (k >> shift) & (RADIX - 1);
        const uint32_t g = s_gstart[d] + (j - s_lstart[d]);
        kout[g] = k;
        vout[g] = s_vals[j];
    }
}

}  // namespace

SortResult radix_sort_pairs(const uint32_t* kin, const uint32_t* vin, uint32_t* ka, uint32_t* va, uint32_t* kb,
                            uint32_t* vb, uint32_t n, uint32_t key_bits, uint32_t* scratch, hipStream_t s) {
    const uint32_t ntiles = sort_tiles(n);
    uint32_t* counts = scratch;
    uint32_t* totals = scratch + (size_t)RADIX * ntiles;
    const uint32_t passes = (key_bits + RADIX_BITS - 1) / RADIX_BITS;
    const uint32_t* ki = kin;
    const uint32_t* vi = vin;
    uint32_t *ko = ka, *vo = va;
    SortResult res{const_cast<uint32_t*>(kin), const_cast<uint32_t*>(vin)};
    if (n == 0) return res;
    for (uint32_t p = 0; p < passes; p++) {
        const uint32_t shift = p * RADIX_BITS;
        hipLaunchKernelGGL(k_upsweep, dim3(ntiles), dim3(SORT_BLOCK), 0, s, ki, n, shift, counts, ntiles);
        hipLaunchKernelGGL(k_scan_rows, dim3(RADIX), dim3(SORT_BLOCK), 0, s, counts, ntiles, totals);
        hipLaunchKernelGGL(k_downsweep, dim3(ntiles), dim3(SORT_BLOCK), 0, s, ki, vi, ko, vo, n, shift, counts,
                           totals, ntiles);
        res.keys = ko;
        res.vals = vo;
        ki = ko;
        vi = vo;
        if (ko == ka) { ko = kb; vo = vb; }
        else { ko = ka; vo = va; }
    }
    return res;
}

}  // namespace rtbvh
