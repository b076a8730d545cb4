// rtbvh_internal.h -- host-side launchers shared by the translation units of
// librtbvh.so.  Not part of the public ABI (that is include/rtbvh.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtbvh_device.h"

namespace rtbvh {

// waves per SIMD of the persistent bounce walk (its launch bounds; the full grid is 256 blocks
// of 4 waves per wave/SIMD over the 1,024 SIMDs)
#ifndef RTBVH_BOUNCE_WAVES
#define RTBVH_BOUNCE_WAVES 8
#endif
constexpr uint32_t BOUNCE_WAVES = RTBVH_BOUNCE_WAVES;

// ---- radix sort (sort.hip) --------------------------------------------------
constexpr uint32_t SORT_BLOCK = 256;
#ifndef RTBVH_SORT_ITEMS
#define RTBVH_SORT_ITEMS 16
#endif
constexpr uint32_t SORT_ITEMS = RTBVH_SORT_ITEMS;   // keys per thread of a tile (A/B: 8 / 16 / 32)
constexpr uint32_t SORT_TILE = SORT_BLOCK * SORT_ITEMS;   // 4096 keys per tile
#ifndef RTBVH_RADIX_BITS
#define RTBVH_RADIX_BITS 8
#endif
constexpr uint32_t RADIX_BITS = RTBVH_RADIX_BITS;   // digit width: 8 (4 passes of 30-bit codes) or 10 (3)
constexpr uint32_t RADIX = 1u << RADIX_BITS;
constexpr size_t BOUNDS_WORDS = 8 + 6 * 1024;
constexpr uint32_t ROOTBOX_WORDS = 16;   // BuildArgs::rootbox
constexpr uint32_t ZPART = 3;            // floats per refit workgroup in BuildArgs::zpart

inline uint32_t sort_tiles(uint32_t n) { return (n + SORT_TILE - 1) / SORT_TILE; }
// scratch words needed: RADIX * tiles (per-tile digit counts) + RADIX (digit totals)
inline size_t sort_scratch_words(uint32_t n) { return (size_t)RADIX * sort_tiles(n) + RADIX; }

// Stable LSD sort of (key, val) over bits [0, key_bits), 8-bit digits.  Pass 0
// reads (kin, vin) and writes (ka, va); later passes ping-pong A <-> B, so the
// input is preserved.  Returns where the sorted pairs are (A, or B, or the
// input itself when n == 0).  Result is in A for an odd pass count, else B.
struct SortResult { uint32_t* keys; uint32_t* vals; };
SortResult radix_sort_pairs(const uint32_t* kin, const uint32_t* vin, uint32_t* ka, uint32_t* va, uint32_t* kb,
                            uint32_t* vb, uint32_t n, uint32_t key_bits, uint32_t* scratch, hipStream_t s);

// ---- build (build.hip) ------------------------------------------------------
struct BuildArgs {
    const float4* opos;       // [V]
    const uint32_t* idx;      // [3T]
    const uint32_t* matidx;   // [T] (into the clip triangle's fourth float4 for the shading)
    uint32_t V, T;
    int morton_mode, delta_mode;
    const float* cam;         // [32] device: the camera of the frame, WVP then WV (row-major, row vectors;
                              //   rtbvh_set_camera), read by the kernels -- a captured frame keeps it
    float smin[3], smax[3];   // HLSL-mode scene box
    float* bounds;            // CPUTests mode: [0..5] scene box (min xyz, max xyz), [8..] 1024 x 6 partials
    uint32_t* keys;           // [T] Morton codes (triangle order) -> sort input
    uint32_t* vals;           // [T] triangle ids
    float4* tclip;            // [TCS * T]
    const uint32_t* sorted_keys;  // [T]
    const uint32_t* sorted_vals;  // [T]
    float4* leaf;             // [4T] 64-B sorted leaf records
    Inner* inner;             // [T-1] refit hand-off boxes of nodes spanning workgroups (touched for those only)
    uint4* topo;              // [T-1] Karras node i: child_l, child_r, leaf range [lo, hi] (16 B)
    Inner* rec;               // [2T-1] node records in slots (rtbvh_device.h)
    uint32_t* pleaf;          // [T]
    uint32_t* pint;           // [T-1]
    uint32_t* refit_cnt;      // [T-1]
    uint32_t* xlist;          // [T] k_refit workgroup b's crossing nodes at [b * RBLOCK, ...)
    uint32_t* xcnt;           // [T / RBLOCK + 1] their counts
    float* rootbox;           // [ROOTBOX_WORDS] the root box (min xyz, max xyz), the leaves' depth range and
                              //   [8] the largest leaf edge bound (k_zrange; margin.h)
    QNode* qnode;             // [2T-1] quantized 4-wide nodes in slots (rtbvh_device.h), from rec
    uint4* lfp;               // [T] leaf footprints on the primary pixel grid (rtbvh_device.h leaf_footprint)
    float* zpart;             // [ZPART * refit_blocks(T)] k_refit workgroup b's leaf depth range, edge bound
    uint32_t pseudo;          // write the leaves' pseudo-records (rec at pleaf[j]; only the packet walks read them)
    uint32_t rec_on;          // write the node records (rec; a certified-only context's build writes none: api.hip)
    uint32_t* qlate;          // [T] or null: k_refit_group's crossing nodes whose QNodes k_qnodes_late builds (count at 0)
    float* nbox;              // [6 (T-1)] or null: internal node k's box (min xyz, max xyz) -- what the certified
                              //   walks' reference-order re-traces and the crossing nodes' QNodes read without records
};
void launch_bounds(const BuildArgs& a, hipStream_t s);
void launch_morton(const BuildArgs& a, hipStream_t s);
// Karras topology (topo, pleaf, pint)
void launch_karras(const BuildArgs& a, hipStream_t s);
// leaf records + refit + node records + QNodes (zeroes the tickets it uses)
void launch_refit(const BuildArgs& a, hipStream_t s);
// ... in two parts: the leaves (k_refit: leaf records, footprints, the in-workgroup nodes; then the
// leaves' depth range rootbox[6..7]) -- all the binned primary pass reads -- and the crossing nodes
void launch_refit_leaves(const BuildArgs& a, hipStream_t s);
void launch_refit_tail(const BuildArgs& a, hipStream_t s);
// the leaves' pseudo-records alone, for a tree built without them (a.pseudo = 0)
void launch_pseudo(const BuildArgs& a, hipStream_t s);
// size of BuildArgs::xcnt for T leaves
uint32_t refit_blocks(uint32_t T);
// qnode[k] of every internal node from the record pairs
void launch_qnodes(const BuildArgs& a, hipStream_t s);
// the whole build in one workgroup for T <= small_build_max() (sorted pairs into
// a.sorted_keys / a.sorted_vals, which must be writable)
uint32_t small_build_max();
void launch_build_small(const BuildArgs& a, hipStream_t s);
// the Morton pass and the sort in one workgroup for T <= small_sort_max() (sorted pairs into
// a.sorted_keys / a.sorted_vals, which must be writable); the multi-kernel build's later stages follow
uint32_t small_sort_max();
void launch_morton_sort_small(const BuildArgs& a, hipStream_t s);
// the node records from the topology and the node boxes (a build that wrote none), and the node boxes from the
// records (one that wrote only records)
void launch_records(const BuildArgs& a, hipStream_t s);
void launch_nbox(const BuildArgs& a, hipStream_t s);
// reference-layout export (44-B Node), 2T-1 entries
void launch_export(const BuildArgs& a, void* out_nodes, hipStream_t s);
// Karras + refit from given sorted codes and leaf boxes (n x 6 floats, device)
void launch_from_codes(const BuildArgs& a, const float* leaf_boxes, hipStream_t s);

// ---- trace (trace.hip) ------------------------------------------------------
struct TraceArgs {
    const Inner* inner;       // node records in slots (BuildArgs::rec); the 4-wide walks read the same array
    // a certified trace's reference-order re-traces walk the topology and the node boxes instead (the context's
    // build may have written no records): nb set, topo = BuildArgs::topo, nbox = BuildArgs::nbox
    const uint4* topo;
    const float* nbox;
    bool nb;
    const float4* leaf;       // [4T] sorted leaf records (see build.hip)
    const float4* tclip;      // [3T] clip-space triangles in triangle order (hit shading)
    const float* verts;       // rtbvh_vertex AoS, 8 floats each
    const uint32_t* idx;
    const uint32_t* matidx;
    const Mat* mats;
    const uint32_t* texels;   // RGBA8 texels of every texture, concatenated (u32 per texel)
    const uint4* texinfo;     // per texture: {first texel, width, height, 0}
    const float* srgb;        // [256] sRGB -> linear (rtbvh_srgb_table)
    uint32_t ntex;
    uint32_t T, W, H, rank, nranks;
    uint32_t band0, bstep;    // this launch traces the rank's bands band0, band0 + bstep, ... (trace chains)
    uint32_t my_bands;        // the rank's bands under the deal (rtbvh_deal_bands)
    const uint32_t* band_list;   // the rank's bands in order (a weighted deal), or null: k * nranks + rank
    const uint32_t* band_slots;  // a weighted deal: band b is rank r's k-th band, slots[b] = r << 24 | k (or null)
    // k_primary behind k_primary_binned: the bins' tile offsets (null: k_primary traces every block),
    // their capacity and the tiles per row
    const uint32_t* pb_gate;
    uint32_t pb_cap, pb_ntx;
    const float* rootbox;     // [6] the BVH root's box (min xyz, max xyz): the bins' depth buckets
    const uint4* lfp;         // [T] leaf footprints (BuildArgs::lfp)
    const float* cam;         // [32] device: WVP, WV (BuildArgs::cam); the shading reads WV
    float4* color;            // output pixels (compacted band rows when nranks > 1)
    float* intensity;         // optional, same indexing as color
    unsigned long long* counters;   // [64] per trace: see flush_counts (trace.hip) and rtbvh_get_stats
    unsigned long long* overflow;   // stack overflows / guard trips, accumulated over every trace (never reset)
    int stack_limit, stack_limit4;  // stack entries the binary / 4-wide primary walks may use (<= STACK_SIZE / STACK4)
    int stack_limit4b;              // ... and the 4-wide bounce walk (<= STACK4B)
    bool limited;                   // a limit below a capacity: the kernels read the limits (else constants)
    bool acyclic;                   // built with the clz64 delta (a radix tree): the 4-wide primary walk
                                    //   needs no walk-length guard
    float* refl_rec;          // optional 14-float RayPresent records (reference reflectRay)
    float* refr_rec;          // optional refractRay records
    const QNode* qnode;       // [2T-1] quantized 4-wide nodes in slots (bounce walk mode 4)
    // N > 1, the binned pass's bins: the leaves whose footprint meets the rank's rows, in PB_LISTS lists (the
    // count pass appends them, the fill pass reads only them; null at N = 1, where every leaf is read):
    // counters PB_LIST_STRIDE words apart, then the lists, pb_list_cap(T) entries each (pb_bin.h)
    uint32_t* pb_list;
};
// primary-ray walks (trace.hip k_primary): per lane in reference order / nearest-first, wave
// packets in reference order / nearest-first, 4-wide wave packets (axis-parallel box test)
enum class PrimaryKind { LANE_REFERENCE, LANE_NEAREST, PACKET_REFERENCE, PACKET_NEAREST, PACKET_WIDE, BINNED };
// bounce walks of the persistent refill kernel (k_bounce_trav)
enum class BounceWalk { REFERENCE, NEAREST, WIDE_QUANTIZED };
void launch_primary(const TraceArgs& a, RayQ* q, uint32_t* qcount, bool count, bool emit, PrimaryKind kind,
                    hipStream_t s);
// A certified trace's re-trace list: the rays of one pass whose certificate failed, and their
// count (zeroed before the pass); the pass's re-trace kernel (reference order) runs over them, REDO_BLOCKS
// workgroups striding over the count on the device
// The certified bounce walk's deferred rays (trace.hip DEFER_*): a clean list of P words per buffer set (readers
// clear what they take) and the pass's work-counter words (its claim and count); null outside bounce passes
struct Redo {
    uint32_t* list;
    uint32_t* count;
    uint32_t* defer = nullptr;
    const uint32_t* dnext = nullptr;
};
constexpr uint32_t REDO_BLOCKS = 512;
// binned primary rays (trace.hip k_primary_binned): the rank's frame in PB_TILE x PB_TILE screen
// tiles (columns x compact band rows), every leaf listed in the tiles its box covers
constexpr uint32_t PB_TILE = 32;
constexpr uint32_t PB_NZ = 16;   // depth buckets per tile: a tile's bins are listed nearest bucket first
constexpr uint32_t PB_LEAVES = 1024;   // the bin passes' leaves per workgroup (pb_bin.h)
constexpr uint32_t PB_LISTS = 16, PB_LIST_STRIDE = 32;   // TraceArgs::pb_list: lists, counter spacing (words)
// entries per list: the leaves of every PB_LISTS-th count block
inline __host__ __device__ uint32_t pb_list_cap(uint32_t T) {
    return ((T + PB_LEAVES - 1) / PB_LEAVES + PB_LISTS - 1) / PB_LISTS * PB_LEAVES;
}
inline size_t pb_list_words(uint32_t T) { return (size_t)PB_LISTS * PB_LIST_STRIDE + (size_t)PB_LISTS * pb_list_cap(T); }
struct PrimBins {
    uint32_t* off;    // [tiles * PB_NZ + 1] leaves per (tile, depth bucket), then their offsets (exclusive
                      //   scan), [tiles * PB_NZ] the total
    uint32_t* cur;    // [tiles * PB_NZ] fill cursors
    uint4* bins;      // [cap] (footprint, leaf) entries, tile by tile, nearest depth bucket first
    unsigned long long* keys;   // [W x rows] the frame's (t, leaf) keys (k_primary_binned -> k_pb_shade)
    uint32_t* sums;   // [tiles * PB_NZ / 1024 + 1] the scan's block totals
    uint32_t cap, ntx, nty;
};
inline uint32_t pb_tiles_x(uint32_t W) { return (W + PB_TILE - 1) / PB_TILE; }
inline uint32_t pb_tiles_y(uint32_t rows) { return (rows + PB_TILE - 1) / PB_TILE; }
// footprints, bins, the binned kernel, then k_primary (the lane walk) behind it for any tile whose
// bins overflowed `cap`; rows = the rank's compact rows
void launch_primary_binned(const TraceArgs& a, const PrimBins& pb, uint32_t rows, RayQ* q, uint32_t* qcount,
                           bool count, bool emit, bool zeroed, hipStream_t s);
// ... in two parts: the binned pass (reads what launch_refit_leaves writes) and the packet walk of
// the overflowed tiles (the whole BVH)
// redo: a certified pass (the shading checks each hit's certificate; the flagged pixels are re-traced)
void launch_pb_pass(const TraceArgs& a, const PrimBins& pb, uint32_t rows, RayQ* q, uint32_t* qcount, bool count,
                    bool emit, bool zeroed, hipStream_t s, const BuildArgs* tail = nullptr, const Redo* redo = nullptr,
                    bool small_tiles = false);   // (512 threads a tile: a small pass one frame at a time)
// the count pass of launch_pb_pass with the climb of the build's crossing nodes in the same launch,
// then their QNodes (build.hip: the build's launch_refit_tail, moved into the frame)
void launch_pb_count_top(const BuildArgs& b, const TraceArgs& a, uint32_t* off, uint32_t* cur, uint4* bins, uint32_t cap,
                         uint32_t ntx, uint32_t leaf_blocks, hipStream_t s);
// reference: the overflowed tiles in the reference order (a certified trace), else nearest-first
void launch_pb_gate(const TraceArgs& a, const PrimBins& pb, RayQ* q, uint32_t* qcount, bool count, bool emit,
                    hipStream_t s, bool reference);
// up to N arrays of 32-bit words zeroed by one launch (null / 0 words: unused)
struct ZeroList {
    static constexpr int N = 5;
    uint32_t* ptr[N];
    size_t words[N];
};
void launch_zero(const ZeroList& z, hipStream_t s);
// one ray per lane bounce pass (reference order or nearest-first), shading included
void launch_bounce(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const uint32_t* perm, RayQ* qout,
                   uint32_t* qout_count, bool count, bool emit, bool nearest, hipStream_t s);
// bounce pass as persistent refill traversal (hit records) + shading kernel; `next` holds
// NEXT_SEGS zeroed work counters NEXT_STRIDE words apart (one per queue segment);
// `blocks` persistent workgroups (0: 2048)
#ifndef RTBVH_NEXT_SEGS
#define RTBVH_NEXT_SEGS 64
#endif
constexpr uint32_t NEXT_SEGS = RTBVH_NEXT_SEGS;
constexpr uint32_t NEXT_STRIDE = 32;                          // one 128-B line per counter
constexpr uint32_t NEXT_WORDS = 16 * NEXT_SEGS * NEXT_STRIDE;  // per buffer set: bounce passes 0..15
// the certified walk's deferred rays (trace.hip): claim and count words in the pass's first counter line
constexpr uint32_t DEFER_CLAIM = 1, DEFER_COUNT = 2;
constexpr uint32_t DEFER_VALID = 0x80000000u;
// cert: the certified 4-wide walk (WIDE_QUANTIZED, no stack limit, a clz64 tree), whose hit records flag
// the rays it cannot vouch for; the shading with a Redo checks each hit's certificate and re-traces
// the flagged rays in the reference order
// a certified pass's early shading (trace.hip RTBVH_EARLY_SHADE): the outputs k_bounce_shade writes, and the pass's
// largest ray count (the shading workgroups of the walk's launch cover it)
struct BounceShade {
    RayQ* qout;
    uint32_t* qout_count;
    bool emit;
    uint32_t* redo;
    uint32_t* redo_count;
    uint32_t P;
};
void launch_bounce_traverse(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const uint32_t* perm,
                            bool count, BounceWalk walk, float2* hitrec, uint32_t* next, uint32_t blocks,
                            hipStream_t s, bool cert = false, uint32_t* defer = nullptr, const BounceShade* es = nullptr);
void launch_bounce_shade(const TraceArgs& a, const RayQ* qin, const uint32_t* qin_count, const float2* hitrec,
                         RayQ* qout, uint32_t* qout_count, bool count, bool emit, uint32_t P, hipStream_t s,
                         const Redo* redo = nullptr);
// *diff += the number of the n float4 pixels of a and b whose bits differ
// the context's device camera (WVP then WV, 32 floats) written by one dispatch in stream order
struct CameraWords { float w[32]; };
void launch_set_camera(const float* wvp, const float* wv, float* cam, hipStream_t s);
void launch_count_diff(const float4* a, const float4* b, size_t n, unsigned long long* diff, hipStream_t s);
void launch_count_diff32(const float* a, const float* b, size_t n, unsigned long long* diff, hipStream_t s);
// frame from per-rank compact band buffers (stride_rows rows apart), see rtbvh_assemble_bands
void launch_assemble(const float4* bands, const uint32_t* slots, uint32_t stride_rows, uint32_t W, uint32_t H,
                     uint32_t nranks,
                     float4* frame, hipStream_t s);
// presentation pass (RayTraceBVHPS.hlsl): flipped rows, UNORM8 RGBA
void launch_present(const float4* color, uint32_t W, uint32_t H, uint32_t* out, hipStream_t s);
// coherence sort keys of a bounce queue: P entries (past *count: key 0xFFFFFFFF)
void launch_bounce_keys(const RayQ* q, const uint32_t* count, const float* box, uint32_t P, uint32_t* keys,
                        uint32_t* vals, hipStream_t s);

}  // namespace rtbvh
