// api.hip -- the C ABI of librtbvh.so (include/rtbvh.h): context, device
// buffers, stream ordering and the host sequence of Graphics::computeBVH
// (Graphics.cpp:667-831), re-done as one HIP stream of kernels with no per-frame
// queue/allocator/fence creation and no host round trip inside build or trace.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/rtbvh.h"
#include "rtbvh_internal.h"

using namespace rtbvh;

struct rtbvh_ctx {
    rtbvh_config cfg{};
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;

    // scene (set_scene)
    uint32_t V = 0, T = 0, nmat = 0;
    float4* d_opos = nullptr;
    float* d_verts = nullptr;
    uint32_t* d_idx = nullptr;
    uint32_t* d_matidx = nullptr;
    Mat* d_mats = nullptr;
    float wvp[16], wv[16];
    float* d_cam = nullptr;     // [32] the kernels' camera (BuildArgs::cam): WVP, WV, uploaded in stream order
    bool cam_dirty = false;     //   (sync_camera) when set_camera changed it
    bool have_scene = false, have_camera = false, built = false;
    bool built_clz64 = false;   // the BVH was built with the clz64 delta: a valid tree (no cycles)

    // build buffers (capacity cap_T)
    uint32_t cap_T = 0;
    uint32_t *d_codes = nullptr, *d_ids = nullptr, *d_ka = nullptr, *d_va = nullptr, *d_kb = nullptr, *d_vb = nullptr;
    uint32_t* d_sort_scratch = nullptr;
    float4 *d_tclip = nullptr, *d_leaf = nullptr;
    float4* d_band = nullptr;                // rtbvh_trace_tiles: this rank's bands; rank 0: all ranks'
    size_t cap_band = 0;                     //   (float4 capacity)
    Inner* d_inner = nullptr;                // box hand-off of refit nodes spanning workgroups
    uint4* d_topo = nullptr;                 // Karras node: child ids + leaf range
    Inner* d_rec = nullptr;                  // node records in slots (rtbvh_device.h), 2T-1
    QNode* d_qnode = nullptr;                // quantized 4-wide nodes in slots (rtbvh_device.h), 2T-1
    uint4* d_lfp = nullptr;                  // leaf footprints on the primary pixel grid (binned primary pass)
    uint32_t* d_texels = nullptr;            // textures (rtbvh_texture), concatenated RGBA8
    uint4* d_texinfo = nullptr;
    float* d_srgb = nullptr;
    uint32_t ntex = 0;
    float* d_refl_rec = nullptr;             // RTBVH_FLAG_REFRACT_RECORDS: reflectRay / refractRay
    float* d_refr_rec = nullptr;             //   RayPresent records, 14 floats per traced pixel
    size_t cap_rec = 0, rec_P = 0;           // record capacity; pixels of the last records trace
    uint32_t *d_pleaf = nullptr, *d_pint = nullptr, *d_cnt = nullptr;
    uint32_t *d_xlist = nullptr, *d_xcnt = nullptr;   // refit: crossing nodes per workgroup
    uint32_t* d_qlate = nullptr;                        // BuildArgs::qlate
    unsigned long long* d_ovf = nullptr;     // stack overflows + guard trips of every trace (never reset)
    unsigned long long* h_ovf = nullptr;     // pinned: a snapshot of *d_ovf copied at the end of each trace,
                                             //   one word per slot; ovf_seen: the value last reported
    unsigned long long ovf_seen = 0;
    float* d_bounds = nullptr;
    float* d_rootbox = nullptr;
    float* d_zpart = nullptr;
    // rtbvh_compute_bvh: the binned primary pass of the frame starts on `side` once the build's
    // leaves are written (ev_leaf, between k_zrange and k_refit_group) and joins the context stream
    // (ev_prim) before the walk of its overflowed tiles, which reads the whole BVH
    hipStream_t side = nullptr;
    hipEvent_t ev_leaf = nullptr, ev_prim = nullptr;
    bool pseudo_ok = false;      // the built tree has its leaf pseudo-records (read by the packet walks only)
    // the built tree's node records (the binary and packet walks') and node boxes (a certified trace's
    // reference-order re-traces): a certified-only context's build writes the boxes alone (records_skipped),
    // any other build the records alone; the other form is derived on first use (ensure_records / ensure_nbox)
    bool rec_ok = false, nbox_ok = false;
    bool build_nbox = false;     // the last build wrote node boxes, not records
    float* d_nbox = nullptr;     // [6 (T-1)] internal node boxes
    bool qnode_ok = false;       // the built tree has its QNodes (read by the 4-wide bounce walk only)
    // rtbvh_compute_bvh: the build leaves its crossing nodes (launch_refit_tail) to the frame's binned
    // pass, which runs them in its bin launches (launch_pb_bin_tail); any other first use of the tree
    // runs them first (flush_tail)
    bool tail_want = false, tail_pending = false;
    bool leaf_want = false;      // the next build records ev_leaf
    bool leaf_pending = false;   // ev_leaf recorded and nothing enqueued on the stream since
    SortResult sorted{nullptr, nullptr};

    // trace buffers (capacity cap_P pixels)
    size_t cap_P = 0;
    uint32_t W = 0, H = 0, bounces = 0, rank = 0, nranks = 1;
    float4* d_color = nullptr;
    float* d_intensity = nullptr;
    RayQ* d_q[2] = {nullptr, nullptr};
    uint32_t *d_bkin = nullptr, *d_bvin = nullptr, *d_bka = nullptr, *d_bva = nullptr, *d_bkb = nullptr,
             *d_bvb = nullptr, *d_bscratch = nullptr;   // bounce coherence sort
    uint32_t* d_qcount = nullptr;             // [32 x MAXSPLIT]: per pipeline, queue counts [0..15] and
                                              //   bounce work counters [16..31]
    float2* d_hit = nullptr;                  // per queued bounce ray: (t, leaf | INVALID)
    uint32_t* d_next = nullptr;               // [NEXT_WORDS x MAXSPLIT]: segmented bounce work counters
    // pipelines 1.. of a split trace (pipeline 0 = d_q / d_hit on the context stream): a
    // rank's bands dealt over `nsplit` independent primary -> bounce chains on their own
    // streams, so one chain's kernel tail overlaps the others' work
#ifndef RTBVH_MAXSPLIT
#define RTBVH_MAXSPLIT 4
#endif
    static constexpr uint32_t MAXSPLIT = RTBVH_MAXSPLIT;   // buffer sets: the context stream's + caller-stream slots
    RayQ* d_qs[MAXSPLIT][2] = {};
    float2* d_hits[MAXSPLIT] = {};
    size_t cap_split = 0;                     // rays per pipeline queue
    hipStream_t sub[MAXSPLIT] = {};
    hipEvent_t ev_fork = nullptr, ev_join[MAXSPLIT] = {};
    uint32_t nsplit = 1;                      // pipelines of the last trace
    // RTBVH_FLAG_BINNED_PRIMARY, per buffer set (chain / frames-in-flight slot): leaf footprints,
    // tile counts / offsets, fill cursors and the bins (trace.hip k_pb_bin)
    struct PbBufs {
        uint32_t *off = nullptr, *cur = nullptr, *sums = nullptr;
        uint4* bins = nullptr;
        unsigned long long* keys = nullptr;
        uint32_t cap_T = 0, cap_tiles = 0, cap_bins = 0;
        size_t cap_px = 0;
        uint32_t* list = nullptr;   // N > 1: the rank's leaves (TraceArgs::pb_list)
        size_t cap_list = 0;
    } pb[MAXSPLIT];
    unsigned long long* d_counters = nullptr; // [64]: see rtbvh_get_stats
    bool traced = false;
    bool frame_here = false;                 // d_color holds the last trace's whole frame
    bool intensity_here = false;             // d_intensity holds its intensities

    // hipEvent rings: per build 6 events (before bounds, after bounds/morton/sort/karras/refit),
    // per trace 3 (before primary, after primary, after bounces)
    static constexpr int RING = 32;
    hipEvent_t evb[RING][6] = {};
    hipEvent_t evt[RING][5] = {};   // trace start, primary done, end, first bounce traversal start/end
    bool evt_trav[RING] = {};
    uint32_t n_builds = 0, n_traces = 0;   // timed samples since reset
    // Frames in flight (rtbvh_trace_band_async on a caller stream other than the context's):
    // such a stream gets a trace-buffer set of its own -- slot k >= 1: d_qs[k], d_hits[k],
    // the queue counts at d_qcount + 32k and the counters at d_counters + 64k -- so traces on
    // different streams run concurrently over the one BVH.  They wait only for the last
    // build (ev_built); the next build waits for them (ev_slot).
    hipStream_t slot_stream[MAXSPLIT] = {};
    hipEvent_t ev_built = nullptr, ev_slot[MAXSPLIT] = {};
    bool slot_busy[MAXSPLIT] = {};
    uint32_t last_slot = 0;   // slot of the last trace (its counters are the stats)
    bool slots_used = false;  // a foreign-stream slot was used: trace chains are off
    // RTBVH_FLAG_GRAPH: the captured frame (build + trace) of rtbvh_compute_bvh and its key
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    uint64_t graph_key[5] = {};
    bool capturing = false;   // enqueueing into a capture: no event records
    uint64_t graph_captures = 0;
    // host-side trace state of the captured frame, restored after every replay
    struct TraceState {
        uint32_t W, H, bounces, nsplit;
        size_t rec_P;
        uint32_t walk, walk_state;
        bool cert;
    } graph_state{};
    // RTBVH_FLAG_AUTO_WALK above AUTO_WALK_MAX_TRIS: the certified fast walks: per buffer
    // set, the list of rays a pass re-traces in the reference order (their counts: d_qcount 16..31)
    uint32_t* d_redo[MAXSPLIT] = {};
    size_t cap_redo[MAXSPLIT] = {};
    uint32_t* d_defer[MAXSPLIT] = {};   // the certified bounce walk's deferred rays (trace.hip DEFER_*), kept clean
    size_t cap_defer[MAXSPLIT] = {};
    uint64_t cert_traces = 0;                         // certified traces so far
    uint32_t last_walk = 0;                           // walk flags of the last trace
    uint32_t last_walk_state = 0;                     // rtbvh_stats.walk_state of the last trace
    // RTBVH_FLAG_AUTO_WALK at <= AUTO_WALK_MAX_TRIS: the primary kind, the reference order's lanes or its
    // wave packets (the same frame), timed on this scene and frame size (enqueue_trace)
    uint64_t small_key = 0;
    uint32_t small_flags = 0;     // the flags the small-scene primary kind was timed under
    bool small_packet = false;
    hipEvent_t ev_small[2] = {};  // its timing events (created on first use, destroyed with the context)
    bool last_cert = false;                           // the last trace was certified (its re-trace counts)
    // tuning knobs of A/B runs, read once by rtbvh_create (RTBVH_BOUNCE_BLOCKS, RTBVH_OVERLAP,
    // RTBVH_SIDE_PRIORITY): a shipped context does not change its launches per frame
    uint32_t knob_bounce_blocks = 0;
    bool knob_overlap = false, knob_side_priority = true, knob_keep_records = false, knob_no_early_shade = false,
         knob_no_small_tiles = false;
    // the band deal of band traces (rtbvh_set_band_deal): rank 0's weight in 1/16 of another rank's
    uint32_t root_share = 16;
    struct DealTab {   // a weighted deal's device table: every rank's bands, then slots[b] = r << 24 | pos
        uint32_t H, nranks, share;
        uint32_t* d;
        std::vector<uint32_t> off;   // rank r's bands at d[off[r] .. off[r + 1])
        uint32_t* h;                 // its pinned staging copy (the upload is asynchronous; freed with d)
        hipEvent_t ready;            // recorded after the upload on the context stream
    };
    std::deque<DealTab> deals;       // the MAX_DEALS most recently used (H, nranks, share), most recent first
    static constexpr size_t MAX_DEALS = 8;
};

namespace {

std::string g_create_error;

rtbvh_status fail(rtbvh_ctx* c, rtbvh_status st, const std::string& msg) {
    if (c) c->err = msg;
    else g_create_error = msg;
    return st;
}

#define HIPC(ctx, expr)                                                                          \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail(ctx, _e == hipErrorOutOfMemory ? RTBVH_ERR_OOM : RTBVH_ERR_HIP,          \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                      \
    } while (0)

template <typename T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

template <typename T>
hipError_t dalloc(T*& p, size_t count) {
    dfree(p);
    if (count == 0) count = 1;
    return hipMalloc((void**)&p, count * sizeof(T));
}

// A captured frame (RTBVH_FLAG_GRAPH) holds the device pointers of capture time: every
// reallocation below drops it, so a replay never writes to a freed buffer.
void drop_graph(rtbvh_ctx* c) {
    if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    c->graph_exec = nullptr;
    c->graph = nullptr;
}

rtbvh_status ensure_build_capacity(rtbvh_ctx* c, uint32_t T) {
    if (T <= c->cap_T && c->d_codes) return RTBVH_OK;
    drop_graph(c);
    const size_t n = T, ni = T > 1 ? T - 1 : 1;
    HIPC(c, dalloc(c->d_codes, n));
    HIPC(c, dalloc(c->d_ids, n));
    HIPC(c, dalloc(c->d_ka, n));
    HIPC(c, dalloc(c->d_va, n));
    HIPC(c, dalloc(c->d_kb, n));
    HIPC(c, dalloc(c->d_vb, n));
    HIPC(c, dalloc(c->d_sort_scratch, sort_scratch_words(T)));
    HIPC(c, dalloc(c->d_tclip, TCS * n));
    HIPC(c, dalloc(c->d_leaf, 4 * n));
    HIPC(c, dalloc(c->d_inner, ni));
    HIPC(c, dalloc(c->d_topo, ni));
    HIPC(c, dalloc(c->d_rec, 2 * (size_t)n - 1));
    HIPC(c, dalloc(c->d_nbox, 6 * (size_t)ni));
    HIPC(c, dalloc(c->d_qnode, 2 * (size_t)n - 1));
    HIPC(c, dalloc(c->d_lfp, n));
    HIPC(c, dalloc(c->d_pleaf, n));
    HIPC(c, dalloc(c->d_pint, ni));
    HIPC(c, dalloc(c->d_cnt, ni));
    HIPC(c, dalloc(c->d_xlist, n));
    HIPC(c, dalloc(c->d_qlate, n + 1));
    HIPC(c, dalloc(c->d_xcnt, refit_blocks(T)));
    HIPC(c, dalloc(c->d_zpart, ZPART * (size_t)refit_blocks(T)));
    HIPC(c, dalloc(c->d_bounds, BOUNDS_WORDS));
    HIPC(c, dalloc(c->d_rootbox, ROOTBOX_WORDS));
    c->cap_T = T;
    return RTBVH_OK;
}

rtbvh_status ensure_trace_capacity(rtbvh_ctx* c, size_t P) {
    if (P <= c->cap_P && c->d_color) return RTBVH_OK;
    drop_graph(c);
    HIPC(c, dalloc(c->d_color, P));
    HIPC(c, dalloc(c->d_intensity, P));
    HIPC(c, dalloc(c->d_q[0], P));
    HIPC(c, dalloc(c->d_q[1], P));
    HIPC(c, dalloc(c->d_bkin, P));
    HIPC(c, dalloc(c->d_bvin, P));
    HIPC(c, dalloc(c->d_bka, P));
    HIPC(c, dalloc(c->d_bva, P));
    HIPC(c, dalloc(c->d_bkb, P));
    HIPC(c, dalloc(c->d_bvb, P));
    HIPC(c, dalloc(c->d_bscratch, sort_scratch_words((uint32_t)P)));
    HIPC(c, dalloc(c->d_hit, P));
    if (!c->d_qcount) HIPC(c, dalloc(c->d_qcount, 32 * rtbvh_ctx::MAXSPLIT));
    if (!c->d_next) HIPC(c, dalloc(c->d_next, (size_t)NEXT_WORDS * rtbvh_ctx::MAXSPLIT));
    if (!c->d_counters) HIPC(c, dalloc(c->d_counters, 64 * rtbvh_ctx::MAXSPLIT));
    c->cap_P = P;
    return RTBVH_OK;
}

// chains of a trace (enqueue_trace): RTBVH_FLAG_SPLIT_SHIFT bits, 0 = automatic
uint32_t trace_split(const rtbvh_ctx* c, size_t pixels) {
    const uint32_t v = (c->cfg.flags >> RTBVH_FLAG_SPLIT_SHIFT) & 7u;
    (void)pixels;
    if (v) return v < rtbvh_ctx::MAXSPLIT ? v : rtbvh_ctx::MAXSPLIT;
    return 1;
}

rtbvh_status ensure_split_capacity(rtbvh_ctx* c, uint32_t nsplit, size_t rays) {
    if (nsplit < 2) return RTBVH_OK;
    const bool grow = rays > c->cap_split;
    if (grow) {
        drop_graph(c);   // every chain's queues hold cap_split rays: drop the smaller ones
        for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)   // (after any frame in flight on them)
            if (c->slot_busy[k]) HIPC(c, hipEventSynchronize(c->ev_slot[k]));
        c->cap_split = rays;
        for (uint32_t g = nsplit; g < rtbvh_ctx::MAXSPLIT; g++) {
            dfree(c->d_qs[g][0]); dfree(c->d_qs[g][1]); dfree(c->d_hits[g]);
        }
    }
    for (uint32_t g = 1; g < nsplit; g++) {
        if (!c->sub[g]) HIPC(c, hipStreamCreateWithFlags(&c->sub[g], hipStreamNonBlocking));
        if (!c->ev_join[g]) HIPC(c, hipEventCreateWithFlags(&c->ev_join[g], hipEventDisableTiming));
        if (!c->ev_fork) HIPC(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
        if (c->d_qs[g][0] && !grow) continue;
        HIPC(c, dalloc(c->d_qs[g][0], c->cap_split));
        HIPC(c, dalloc(c->d_qs[g][1], c->cap_split));
        HIPC(c, dalloc(c->d_hits[g], c->cap_split));
    }
    return RTBVH_OK;
}

// Binned primary buffers of buffer set b for T leaves and `tiles` screen tiles.  The bins hold
// BINS_PER_LEAF entries per leaf (C5: 1.37 tiles per leaf); a tile whose bins would pass the end is
// traced by the 4-wide packet walk instead (trace.hip pb_gate), so the capacity is a speed knob only.
constexpr uint32_t BINS_PER_LEAF = 3;
rtbvh_status ensure_pb_capacity(rtbvh_ctx* c, uint32_t b, uint32_t T, uint32_t tiles, size_t pixels) {
    rtbvh_ctx::PbBufs& p = c->pb[b];
    const uint32_t bins = BINS_PER_LEAF * T + 16 * tiles;
    if (T <= p.cap_T && tiles <= p.cap_tiles && bins <= p.cap_bins && pixels <= p.cap_px && p.off) return RTBVH_OK;
    drop_graph(c);
    if (pixels > p.cap_px) {
        HIPC(c, dalloc(p.keys, pixels));
        p.cap_px = pixels;
    }
    const uint32_t nT = std::max(T, p.cap_T), nt = std::max(tiles, p.cap_tiles);
    const uint32_t nb = std::max(BINS_PER_LEAF * nT + 16 * nt, p.cap_bins);
    HIPC(c, dalloc(p.off, (size_t)nt * PB_NZ + 1));
    HIPC(c, dalloc(p.cur, (size_t)nt * PB_NZ));
    HIPC(c, dalloc(p.sums, (size_t)nt * PB_NZ / 1024 + 1));
    HIPC(c, dalloc(p.bins, nb));
    p.cap_T = nT;
    p.cap_tiles = nt;
    p.cap_bins = nb;
    return RTBVH_OK;
}

BuildArgs build_args(rtbvh_ctx* c) {
    BuildArgs a{};
    a.opos = c->d_opos;
    a.idx = c->d_idx;
    a.matidx = c->d_matidx;
    a.V = c->V;
    a.T = c->T;
    a.morton_mode = (int)c->cfg.morton_mode;
    a.delta_mode = (int)c->cfg.delta_mode;
    a.cam = c->d_cam;
    memcpy(a.smin, c->cfg.scene_bb_min, 12);
    memcpy(a.smax, c->cfg.scene_bb_max, 12);
    a.bounds = c->d_bounds;
    a.keys = c->d_codes;
    a.vals = c->d_ids;
    a.tclip = c->d_tclip;
    a.sorted_keys = c->sorted.keys;
    a.sorted_vals = c->sorted.vals;
    a.leaf = c->d_leaf;
    a.inner = c->d_inner;
    a.topo = c->d_topo;
    a.rec = c->d_rec;
    a.pleaf = c->d_pleaf;
    a.pint = c->d_pint;
    a.refit_cnt = c->d_cnt;
    a.xlist = c->d_xlist;
    a.qlate = c->d_qlate;
    a.xcnt = c->d_xcnt;
    a.rootbox = c->d_rootbox;
    a.qnode = c->d_qnode;
    a.lfp = c->d_lfp;
    a.zpart = c->d_zpart;
    // the leaf pseudo-records cost the build 0.64 GB of writes at 10M triangles: written when the
    // context's walks include a packet primary walk (AUTO and the binned pass take none)
    // (choose_walks: a packet primary walk iff PACKET_PRIMARY without BINNED_PRIMARY)
    const uint32_t f = c->cfg.flags;
    a.pseudo = (f & RTBVH_FLAG_PACKET_PRIMARY) &&
               !(f & (RTBVH_FLAG_BINNED_PRIMARY | RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_CERTIFIED));
    // the last build's outputs: node records, or (a certified-only context's) node boxes instead
    a.rec_on = c->build_nbox ? 0u : 1u;
    a.nbox = c->build_nbox ? c->d_nbox : nullptr;
    return a;
}
// the same, with the node-box array for a kernel that reads (or writes) it
BuildArgs build_args_nbox(rtbvh_ctx* c) {
    BuildArgs a = build_args(c);
    a.nbox = c->d_nbox;
    return a;
}

// ---- the band deal ----------------------------------------------
// The frame's 8-row bands b = 0 .. ceil(H / 8) - 1 go to the ranks by smooth weighted round-robin:
// rank 0 has weight `share`, every other rank 16; for each band every rank's credit grows by its
// weight, and the rank with the most credit (the lowest on a tie) takes the band and pays the
// total weight.  share 16 deals b -> b % nranks exactly; below 16, rank 0 -- which also receives
// and assembles the other ranks' bands -- traces share / 16 of another rank's bands, spread evenly
// over the frame (the centre-heavy hit distribution stays balanced).
void deal_owners(uint32_t H, uint32_t nranks, uint32_t share, std::vector<uint32_t>& owner) {
    const uint32_t nb = (H + 7) / 8;
    owner.assign(nb, 0);
    if (nranks <= 1) return;
    std::vector<int64_t> credit(nranks, 0);
    const int64_t total = (int64_t)share + 16 * (int64_t)(nranks - 1);
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t best = 0;
        for (uint32_t r = 0; r < nranks; r++) {
            credit[r] += r == 0 ? share : 16;
            if (credit[r] > credit[best]) best = r;
        }
        credit[best] -= total;
        owner[b] = best;
    }
}
uint32_t band_height(uint32_t H, uint32_t b) { return (H - b * 8) < 8 ? (H - b * 8) : 8; }
uint32_t deal_rows(uint32_t H, uint32_t rank, uint32_t nranks, uint32_t share) {
    if (nranks == 0 || rank >= nranks) return 0;
    if (share == 16 || nranks == 1) {
        uint32_t rows = 0;
        for (uint32_t b = rank; b * 8 < H; b += nranks) rows += band_height(H, b);
        return rows;
    }
    std::vector<uint32_t> owner;
    deal_owners(H, nranks, share, owner);
    uint32_t rows = 0;
    for (uint32_t b = 0; b < owner.size(); b++)
        if (owner[b] == rank) rows += band_height(H, b);
    return rows;
}
uint32_t deal_max_rows(uint32_t H, uint32_t nranks, uint32_t share) {
    uint32_t m = 0;
    for (uint32_t r = 0; r < nranks; r++) m = std::max(m, deal_rows(H, r, nranks, share));
    return m;
}
rtbvh_status sync_all(rtbvh_ctx* c);
// The device table of a weighted deal (null for round-robin: the kernels compute it).  Uploaded on
// first use (a few KB, once per frame size and deal), so not from inside a graph capture (whose frames
// have one rank): an asynchronous copy from pinned staging on the context stream, and an event the
// caller's stream `s` waits for (a trace on a caller stream, an assembly on another).  The MAX_DEALS
// most recently used tables are kept; evicting one first waits for the context's work (traces in
// flight may read it).
void free_deal(rtbvh_ctx::DealTab& t) {
    dfree(t.d);
    if (t.h) (void)hipHostFree(t.h);
    if (t.ready) (void)hipEventDestroy(t.ready);
    t.h = nullptr;
    t.ready = nullptr;
}
rtbvh_status get_deal(rtbvh_ctx* c, uint32_t H, uint32_t nranks, const rtbvh_ctx::DealTab** out, hipStream_t s) {
    *out = nullptr;
    if (c->root_share == 16 || nranks <= 1) return RTBVH_OK;
    for (auto it = c->deals.begin(); it != c->deals.end(); ++it)
        if (it->H == H && it->nranks == nranks && it->share == c->root_share) {
            if (it != c->deals.begin()) {   // most recent first
                rtbvh_ctx::DealTab t = std::move(*it);
                c->deals.erase(it);
                c->deals.push_front(std::move(t));
            }
            *out = &c->deals.front();
            if (s != c->stream && !c->capturing) HIPC(c, hipStreamWaitEvent(s, c->deals.front().ready, 0));
            return RTBVH_OK;
        }
    if (c->capturing) return fail(c, RTBVH_ERR_INVALID_ARG, "a new band deal inside a graph capture");
    if (c->deals.size() >= rtbvh_ctx::MAX_DEALS) {
        rtbvh_status st = sync_all(c);
        if (st) return st;
        free_deal(c->deals.back());
        c->deals.pop_back();
    }
    std::vector<uint32_t> owner;
    deal_owners(H, nranks, c->root_share, owner);
    const uint32_t nb = (uint32_t)owner.size();
    rtbvh_ctx::DealTab t{H, nranks, c->root_share, nullptr, std::vector<uint32_t>(nranks + 1, 0), nullptr, nullptr};
    const size_t words = 2 * (size_t)nb + 1;
    std::vector<uint32_t> cnt(nranks, 0);
    if (hipHostMalloc((void**)&t.h, words * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void**)&t.d, words * sizeof(uint32_t)) != hipSuccess ||
        hipEventCreateWithFlags(&t.ready, hipEventDisableTiming) != hipSuccess) {
        free_deal(t);
        return fail(c, RTBVH_ERR_OOM, "band deal table");
    }
    for (uint32_t b = 0; b < nb; b++) t.off[owner[b] + 1]++;
    for (uint32_t r = 0; r < nranks; r++) t.off[r + 1] += t.off[r];
    t.h[2 * nb] = 0;
    for (uint32_t b = 0; b < nb; b++) {
        const uint32_t r = owner[b], pos = cnt[r]++;
        t.h[t.off[r] + pos] = b;           // rank r's pos-th band
        t.h[nb + b] = r << 24 | pos;       // where band b sits (k_assemble)
    }
    c->deals.push_front(std::move(t));
    rtbvh_ctx::DealTab& f = c->deals.front();
    HIPC(c, hipMemcpyAsync(f.d, f.h, words * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipEventRecord(f.ready, c->stream));
    if (s != c->stream) HIPC(c, hipStreamWaitEvent(s, f.ready, 0));
    *out = &f;
    return RTBVH_OK;
}

TraceArgs trace_args(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t rank, uint32_t nranks, float4* color, float* inten) {
    TraceArgs a{};
    a.inner = c->d_rec;
    a.topo = c->d_topo;
    a.nbox = c->d_nbox;
    a.nb = false;
    a.leaf = c->d_leaf;
    a.qnode = c->d_qnode;
    a.rootbox = c->d_rootbox;
    a.lfp = c->d_lfp;
    a.tclip = c->d_tclip;
    a.verts = c->d_verts;
    a.idx = c->d_idx;
    a.matidx = c->d_matidx;
    a.texels = c->d_texels;
    a.texinfo = c->d_texinfo;
    a.srgb = c->d_srgb;
    a.ntex = c->ntex;
    a.mats = c->d_mats;
    a.T = c->T;
    a.W = W;
    a.H = H;
    a.rank = rank;
    a.nranks = nranks;
    a.band0 = 0;
    a.bstep = 1;
    const uint32_t nb = (H + 7) / 8;
    a.my_bands = rank < nb ? (nb - rank + nranks - 1) / nranks : 0;   // round-robin; enqueue_walks sets a deal's
    a.band_list = nullptr;
    a.cam = c->d_cam;
    a.color = color;
    a.intensity = inten;
    a.counters = c->d_counters;
    a.overflow = c->d_ovf;
    const uint32_t lim = c->cfg.stack_limit;
    a.stack_limit = lim && lim < (uint32_t)STACK_SIZE ? (int)lim : STACK_SIZE;
    a.stack_limit4 = lim && lim < (uint32_t)STACK4 ? (int)lim : STACK4;
    a.stack_limit4b = lim && lim < (uint32_t)STACK4B ? (int)lim : STACK4B;
    a.limited = lim != 0 && lim < (uint32_t)STACK4B;
    a.acyclic = c->built_clz64;
    return a;
}

// The walks of a trace (include/rtbvh.h RTBVH_FLAG_*).  RTBVH_FLAG_AUTO_WALK: the
// reference-order kernels (the exact findCollision DFS) up to AUTO_WALK_MAX_TRIS triangles,
// where they are the fastest (C2/C3: Image_Test.obj, Test.obj); above, the 4-wide
// nearest-first walks (C5: 3.4x the reference order) for a frame key once a frame of that key
// traced both ways compared equal on the device (enqueue_trace), the reference order otherwise.
constexpr uint32_t AUTO_WALK_MAX_TRIS = 1u << 16;
constexpr uint32_t WALK_FLAGS = RTBVH_FLAG_NEAREST_FIRST | RTBVH_FLAG_PACKET_PRIMARY | RTBVH_FLAG_REFILL_BOUNCE |
                                RTBVH_FLAG_WIDE_BVH | RTBVH_FLAG_BINNED_PRIMARY;
bool auto_checked(const rtbvh_ctx* c) {
    return (c->cfg.flags & RTBVH_FLAG_AUTO_WALK) && c->T > AUTO_WALK_MAX_TRIS;
}
// A certified-only context -- RTBVH_FLAG_CERTIFIED, or AUTO_WALK on a scene past AUTO_WALK_MAX_TRIS, on a clz64
// tree with no stack limit (plan_trace) -- traces with walks that read no node record: the binned primary pass
// (leaf footprints and records), the certified 4-wide bounce walk (QNodes; a node without a grid flags the ray),
// and reference-order re-traces of the few flagged rays on the topology and node boxes (trace.hip traverse_nb).
// Its multi-kernel build writes the 24-B node boxes instead of the 64-B node records (C4
// refit stage 0.94 -> 0.81 ms without them); records are derived if another walk needs them (ensure_records).
// RTBVH_KEEP_RECORDS=1 (A/B): write the records anyway.
bool records_skipped(const rtbvh_ctx* c);
rtbvh_status ensure_records(rtbvh_ctx* c, hipStream_t s) {
    if (c->rec_ok || !c->built) return RTBVH_OK;
    launch_records(build_args_nbox(c), c->stream);
    HIPC(c, hipGetLastError());
    c->rec_ok = true;
    if (s != c->stream) {
        if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, c->stream));
        HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
    }
    return RTBVH_OK;
}
bool records_skipped(const rtbvh_ctx* c) {
    const uint32_t f = c->cfg.flags;
    const bool limited = c->cfg.stack_limit != 0 && c->cfg.stack_limit < (uint32_t)STACK_SIZE;
    const bool small = c->T <= small_build_max() && !(f & RTBVH_FLAG_MULTI_KERNEL_BUILD);   // (k_build_small: records)
    return !small && !c->knob_keep_records && ((f & RTBVH_FLAG_CERTIFIED) || auto_checked(c)) &&
           c->cfg.delta_mode == RTBVH_DELTA_CLZ64 && !limited;
}
rtbvh_status ensure_nbox(rtbvh_ctx* c, hipStream_t s) {
    if (c->nbox_ok || !c->built) return RTBVH_OK;
    BuildArgs a = build_args_nbox(c);
    a.rec_on = 1;
    launch_nbox(a, c->stream);
    HIPC(c, hipGetLastError());
    c->nbox_ok = true;
    if (s != c->stream) {
        if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, c->stream));
        HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
    }
    return RTBVH_OK;
}
struct Walks {
    PrimaryKind primary;
    bool refill;        // bounce passes as persistent refill traversal + shading kernel
    BounceWalk bounce;  // refill walk
    bool nearest;       // one-ray-per-lane bounce kernel: nearest-first
    bool sort;          // coherence sort of the bounce queue
};
Walks choose_walks(uint32_t f) {
    Walks w{};
    const bool nearest = (f & RTBVH_FLAG_NEAREST_FIRST) != 0, wide = (f & RTBVH_FLAG_WIDE_BVH) != 0;
    const bool packet = (f & RTBVH_FLAG_PACKET_PRIMARY) != 0;
    w.primary = packet ? (wide ? PrimaryKind::PACKET_WIDE : nearest ? PrimaryKind::PACKET_NEAREST
                                                                    : PrimaryKind::PACKET_REFERENCE)
                       : (nearest ? PrimaryKind::LANE_NEAREST : PrimaryKind::LANE_REFERENCE);
    if (f & RTBVH_FLAG_BINNED_PRIMARY) w.primary = PrimaryKind::BINNED;
    // the ray records are written by k_primary and k_bounce_shade: the split bounce path
    w.refill = (f & (RTBVH_FLAG_REFILL_BOUNCE | RTBVH_FLAG_WIDE_BVH | RTBVH_FLAG_REFRACT_RECORDS)) != 0;
    w.bounce = wide ? BounceWalk::WIDE_QUANTIZED : nearest ? BounceWalk::NEAREST : BounceWalk::REFERENCE;
    w.nearest = nearest;
    w.sort = (f & RTBVH_FLAG_SORT_BOUNCE) != 0;
    return w;
}

// RCCL, resolved at run time: the process's librccl.so.1 if one is already loaded (e.g.
// PyTorch's; dlopen by SONAME returns it), else the system's.  No link-time dependency.
struct Rccl {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
const Rccl& rccl() {
    static const Rccl lib = [] {
        Rccl r;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            r.err = std::string("RCCL not available: ") + (e ? e : "dlopen(librccl.so.1) failed");
            return r;
        }
        bool all = true;
        auto sym = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            if (!f) all = false;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.GetErrorString, "ncclGetErrorString");
        r.ok = all;
        if (!all) r.err = "RCCL: librccl.so.1 lacks a required symbol";
        return r;
    }();
    return lib;
}

rtbvh_status check_launch(rtbvh_ctx* c, const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(c, RTBVH_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return RTBVH_OK;
}

// the context stream and the frames in flight on caller streams, drained
rtbvh_status sync_all(rtbvh_ctx* c) {
    HIPC(c, hipStreamSynchronize(c->stream));
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)
        if (c->slot_busy[k]) HIPC(c, hipEventSynchronize(c->ev_slot[k]));
    return RTBVH_OK;
}

// The camera the kernels read (BuildArgs::cam), uploaded in stream order on the context stream when
// rtbvh_set_camera changed it -- after the frames in flight, which read the old one -- and ordered
// before stream s.  A captured frame (RTBVH_FLAG_GRAPH) reads the buffer, so it survives a camera change
// (Graphics::onUpdate writes the camera every frame and the arrow keys orbit it, Graphics.cpp:40-56,
// 937-960).  The matrices travel as a kernel argument (launch_set_camera): captured at the call, one
// dispatch, no pageable host copy (staged through the driver at the call).  Never inside a capture:
// compute_graph's plain frame before it has cleared cam_dirty, and the captured frame must not bake a
// camera in.
rtbvh_status sync_camera(rtbvh_ctx* c, hipStream_t s) {
    if (!c->cam_dirty) return RTBVH_OK;
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)
        if (c->slot_busy[k]) {
            HIPC(c, hipStreamWaitEvent(c->stream, c->ev_slot[k], 0));
            c->slot_busy[k] = false;
        }
    launch_set_camera(c->wvp, c->wv, c->d_cam, c->stream);
    HIPC(c, hipGetLastError());
    if (s != c->stream) {
        HIPC(c, hipEventRecord(c->ev_built, c->stream));
        HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
    }
    c->cam_dirty = false;
    return RTBVH_OK;
}

// The kernels of one trace with the walks of `flags` (timed: record the stage events when
// RTBVH_FLAG_TIMING asks for them).
// cert: the certified walks (flags = the fast walks: binned primary pass, 4-wide bounce walk):
// every pass checks each ray's certificate and re-traces the rays that fail it in the reference order.
rtbvh_status enqueue_walks(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces, uint32_t rank, uint32_t nranks,
                           float4* color, float* inten, hipStream_t s, uint32_t slot, uint32_t flags, bool timed,
                           bool cert = false) {
    const bool leaf_pending = c->leaf_pending;   // (this trace is the first after the build or none is)
    c->leaf_pending = false;
    // the build's crossing nodes, if left to this trace: run in the binned pass's launches below, or
    // before any walk (and on every early return) by the guard
    struct TailGuard {
        rtbvh_ctx* c;
        bool pending;
        void run() {
            if (pending) launch_refit_tail(build_args(c), c->stream);
            pending = false;
        }
        ~TailGuard() { run(); }
    } tail{c, c->tail_pending};
    c->tail_pending = false;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "trace before build");
    if (W == 0 || H == 0 || nranks == 0 || rank >= nranks || bounces > 14)
        return fail(c, RTBVH_ERR_INVALID_ARG, "bad trace dimensions");
    rtbvh_status st = ensure_trace_capacity(c, (size_t)W * H);
    if (st) return st;
    if (!color) color = c->d_color;
    const bool count = (c->cfg.flags & RTBVH_FLAG_COUNT_VISITS) != 0;
    const bool timing = timed && (c->cfg.flags & RTBVH_FLAG_TIMING) != 0 && s == c->stream && !c->capturing;
    TraceArgs a = trace_args(c, W, H, rank, nranks, color, inten);
    const rtbvh_ctx::DealTab* deal = nullptr;
    rtbvh_status dst = get_deal(c, H, nranks, &deal, s);
    if (dst) return dst;
    if (deal) {
        a.my_bands = deal->off[rank + 1] - deal->off[rank];
        a.band_list = deal->d + deal->off[rank];
        a.band_slots = deal->d + (H + 7) / 8;
    }
    a.counters = c->d_counters + 64 * slot;
    hipEvent_t* ev = c->evt[c->n_traces % rtbvh_ctx::RING];
    const Walks wk = choose_walks(flags);
    const bool sort = wk.sort, refill = wk.refill;
    const bool records = (flags & RTBVH_FLAG_REFRACT_RECORDS) != 0;
    if (records && slot) return fail(c, RTBVH_ERR_INVALID_ARG, "ray records are traced on the context stream only");
    const uint32_t P = W * deal_rows(H, rank, nranks, c->root_share);   // max live rays of this shard
    // persistent grid of the bounce walk: 2048 blocks (8 waves/SIMD), 1024 for a shard of
    // < 4M pixels -- with frames in flight the next frame's primary blocks then share the CUs
    // (C5, rank of N=8, three frames in flight: 0.85 -> 0.78 ms per frame) -- and 512 below 3M pixels once
    // frames are in flight on caller streams (round 5, four in flight, `r05_hh`: the N = 8 rank 0.62 -> 0.60
    // ms per frame, N = 4 1.03 -> 1.00; one frame at a time 512 is slower, 1.13 -> 1.37 ms at N = 8); one frame at
    // a time, 1536 (round 6, with early shading, `r06_bb`: the N = 8 rank 1.198 -> 1.169 ms, N = 4 1.602 -> 1.535;
    // 768 / 2048 / 3072: 1.29 / 1.23 / 1.36 at N = 8)
#ifndef RTBVH_BOUNCE_GRID
#define RTBVH_BOUNCE_GRID (256 * BOUNCE_WAVES)
#endif
    // ("in flight": this trace is on a caller stream's slot, or another slot's frame is still running --
    // not a flag that stays set once any caller stream has traced: ADVICE r5)
    bool inflight = slot != 0;
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT && !inflight && !c->capturing; k++)
        inflight = c->slot_busy[k] && hipEventQuery(c->ev_slot[k]) == hipErrorNotReady;
    uint32_t tblocks = P < (1u << 22) ? (!inflight ? 1536 : P < (3u << 20) ? 512 : 1024) : RTBVH_BOUNCE_GRID;
    if (c->knob_bounce_blocks) tblocks = c->knob_bounce_blocks;   // tuning override (A/B runs)
    if (records) {
        if (c->cap_rec < P) {
            drop_graph(c);
            HIPC(c, dalloc(c->d_refl_rec, 14 * (size_t)P));
            HIPC(c, dalloc(c->d_refr_rec, 14 * (size_t)P));
            c->cap_rec = P;
        }
        a.refl_rec = c->d_refl_rec;
        a.refr_rec = c->d_refr_rec;
    }
    c->rec_P = records ? P : 0;
    // pipelines: the rank's bands dealt round-robin over nsplit primary -> bounce chains
    // (band k of this rank goes to chain k % nsplit), each with its own queues and work
    // counters, chain 0 on the context stream, chain g on sub[g]; joined before the end event
    const uint32_t my_bands = a.my_bands;
    uint32_t nsplit = trace_split(c, (size_t)W * 8 * my_bands);
    // the coherence sort has one set of buffers; frames-in-flight slots use the chains' buffers
    // the binned primary pass covers the rank's whole frame in one chain; the build's leaf footprints
    // are exact for frames of up to 32768 pixels a side (rtbvh_device.h leaf_footprint)
    const uint32_t rows = P / W;
    const bool binned = wk.primary == PrimaryKind::BINNED;
    // (a certified trace past that size: the reference-order lane walk, exact by construction)
    const PrimaryKind pkind = binned && (W > 32768u || H > 32768u)
                                  ? (cert ? PrimaryKind::LANE_REFERENCE : PrimaryKind::PACKET_WIDE)
                                  : wk.primary;
    if (sort || my_bands < nsplit || slot || c->slots_used || binned) nsplit = 1;
    // the walks' node data: a certified trace's re-traces walk the node boxes (a.nb), every other walk the node
    // records; a build writes one of the two, the other is derived here from the complete tree (after the tail)
    const bool need_conv = cert ? !c->nbox_ok : !c->rec_ok;
    const bool fuse_tail = tail.pending && pkind == PrimaryKind::BINNED && s == c->stream && slot == 0 && rows > 0 &&
                           !need_conv;
    if (!fuse_tail && tail.pending) {   // before any walk reads the tree
        tail.run();
        if (s != c->stream) {   // (a caller stream: ordered after it like after the build)
            if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, c->stream));
            HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
        }
    }
    if (need_conv) {
        st = cert ? ensure_nbox(c, s) : ensure_records(c, s);
        if (st) return st;
    }
    a.nb = cert;
    const uint32_t Pg = nsplit == 1 ? P : W * 8 * ((my_bands + nsplit - 1) / nsplit);   // max live rays per chain
    st = ensure_split_capacity(c, slot ? slot + 1 : nsplit, Pg);
    if (st) return st;
    if (!c->qnode_ok && bounces > 0 && wk.refill && wk.bounce == BounceWalk::WIDE_QUANTIZED) {
        // a 4-wide bounce walk over a one-workgroup build that quantized no nodes (the context's
        // walks took none): k_qnodes now, as for the pseudo-records below
        launch_qnodes(build_args(c), c->stream);
        c->qnode_ok = true;
        if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, c->stream));
        if (s != c->stream) HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
    }
    if (!c->pseudo_ok && (pkind == PrimaryKind::PACKET_REFERENCE || pkind == PrimaryKind::PACKET_NEAREST ||
                          pkind == PrimaryKind::PACKET_WIDE)) {
        // a packet walk over a tree built without the leaf pseudo-records (the context's walks took
        // none; set_flags since, or a frame past the binned pass's 32768 pixels a side): written now,
        // on the context stream (no walk of a slot stream reads those slots)
        launch_pseudo(build_args(c), c->stream);
        c->pseudo_ok = true;
        if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, c->stream));
        if (s != c->stream) HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
    }
    // a certified trace's re-trace list (one chain: buffer set `slot`; counts at d_qcount 16 + pass)
    if (cert && bounces > 0 && c->cap_defer[slot] < P) {   // (zeroed once: its readers clear what they take)
        drop_graph(c);
        dfree(c->d_defer[slot]);
        HIPC(c, dalloc(c->d_defer[slot], P));
        HIPC(c, hipMemsetAsync(c->d_defer[slot], 0, sizeof(uint32_t) * P, c->stream));
        if (s != c->stream) {
            if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, c->stream));
            HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
        }
        c->cap_defer[slot] = P;
    }
    if (cert && c->cap_redo[slot] < P) {
        drop_graph(c);
        HIPC(c, dalloc(c->d_redo[slot], P));
        c->cap_redo[slot] = P;
    }
    // the binned pass's buffers (one chain: buffer set `slot`)
    const uint32_t ntx = pb_tiles_x(W), nty = pb_tiles_y(rows);
    if (pkind == PrimaryKind::BINNED) {
        st = ensure_pb_capacity(c, slot, c->T, ntx * nty, (size_t)W * rows);
        if (st) return st;
        if (nranks > 1 && c->pb[slot].cap_list < pb_list_words(c->T)) {
            drop_graph(c);
            HIPC(c, dalloc(c->pb[slot].list, pb_list_words(c->T)));
            c->pb[slot].cap_list = pb_list_words(c->T);
        }
    }
    // the trace's counters, queue counts, bounce work counters and bin counts: one launch
    ZeroList z{};
    z.ptr[0] = reinterpret_cast<uint32_t*>(a.counters);
    z.words[0] = 64 * 2;
    z.ptr[1] = c->d_qcount + 32 * slot;
    z.words[1] = 32 * nsplit;
    if (refill && bounces) {
        z.ptr[2] = c->d_next + (size_t)NEXT_WORDS * slot;
        z.words[2] = (size_t)NEXT_WORDS * nsplit;
    }
    if (pkind == PrimaryKind::BINNED) {
        z.ptr[3] = c->pb[slot].off;
        z.words[3] = (size_t)ntx * nty * PB_NZ + 1;
        if (nranks > 1) {   // the list counters
            z.ptr[4] = c->pb[slot].list;
            z.words[4] = (size_t)PB_LISTS * PB_LIST_STRIDE;
        }

    }
    // rtbvh_compute_bvh: the binned pass (and the zeroing before it) on the side stream, concurrent
    // with the build's crossing nodes (launch_refit_tail)
    const bool overlap = pkind == PrimaryKind::BINNED && leaf_pending && s == c->stream && slot == 0 && nsplit == 1;
    hipStream_t sp = s;
    if (overlap) {
        sp = c->side;
        HIPC(c, hipStreamWaitEvent(sp, c->ev_leaf, 0));
    }
    launch_zero(z, sp);
    if (timing) HIPC(c, hipEventRecord(ev[0], sp));
    if (nsplit > 1) HIPC(c, hipEventRecord(c->ev_fork, s));
    for (uint32_t g = 0; g < nsplit; g++) {
        hipStream_t sg = g ? c->sub[g] : s;
        if (g) HIPC(c, hipStreamWaitEvent(sg, c->ev_fork, 0));
        TraceArgs ag = a;
        ag.band0 = g;
        ag.bstep = nsplit;
        ag.pb_list = pkind == PrimaryKind::BINNED && nranks > 1 ? c->pb[g + slot].list : nullptr;
        const uint32_t b = g + slot;   // buffer set: chain g of the context stream's trace, or the slot
        RayQ* q[2] = {b ? c->d_qs[b][0] : c->d_q[0], b ? c->d_qs[b][1] : c->d_q[1]};
        float2* hit = b ? c->d_hits[b] : c->d_hit;
        uint32_t* qc = c->d_qcount + 32 * b;
        uint32_t* nx = c->d_next + (size_t)NEXT_WORDS * b;
        const bool tg = timing && g == 0;   // stage events: chain 0's kernels
        if (pkind == PrimaryKind::BINNED) {
            const rtbvh_ctx::PbBufs& pbb = c->pb[b];
            const PrimBins pb{pbb.off, pbb.cur, pbb.bins, pbb.keys, pbb.sums, pbb.cap_bins, ntx, nty};
            if (rows) {
                const BuildArgs ba = build_args(c);
                const Redo rd{c->d_redo[b], &qc[16]};
                // a rank's small pass one frame at a time: 512 threads a tile (its ~1,000 tiles all run at once;
                // with frames in flight 256 is faster, round 5 r05_jj). Round 6 (r06_stl): the N = 8 rank's frame
                // 1.13-1.15 -> 1.11 ms; N = 4 (2.1M pixels) the same, N = 2 (4.1M) +0.05 ms: below 1.5M pixels only
                const bool small_tiles = !inflight && !c->knob_no_small_tiles && (size_t)W * rows < (3u << 19);
                launch_pb_pass(ag, pb, rows, q[0], &qc[0], count, bounces > 0, true, overlap ? sp : sg,
                               fuse_tail ? &ba : nullptr, cert ? &rd : nullptr, small_tiles);
                if (fuse_tail) tail.pending = false;
                if (overlap) {
                    HIPC(c, hipEventRecord(c->ev_prim, sp));
                    HIPC(c, hipStreamWaitEvent(sg, c->ev_prim, 0));
                }
                launch_pb_gate(ag, pb, q[0], &qc[0], count, bounces > 0, sg, cert);
            } else if (overlap) {   // (nothing traced: the zeroing still joins)
                HIPC(c, hipEventRecord(c->ev_prim, sp));
                HIPC(c, hipStreamWaitEvent(sg, c->ev_prim, 0));
            }
        } else
            launch_primary(ag, q[0], &qc[0], count, bounces > 0, pkind, sg);
        if (tg) HIPC(c, hipEventRecord(ev[1], sg));
        for (uint32_t b = 0; b < bounces; b++) {
            const uint32_t* perm = nullptr;
            if (sort) {
                launch_bounce_keys(q[b & 1], &qc[b], c->d_rootbox, P, c->d_bkin, c->d_bvin, sg);
                perm = radix_sort_pairs(c->d_bkin, c->d_bvin, c->d_bka, c->d_bva, c->d_bkb, c->d_bvb, P, 30,
                                        c->d_bscratch, sg).vals;
            }
            if (refill) {
                if (tg && b == 0) HIPC(c, hipEventRecord(ev[3], sg));
                uint32_t* nxb = nx + (size_t)NEXT_SEGS * NEXT_STRIDE * b;
                // a frame one at a time shades its rays in the walk's tail (trace.hip RTBVH_EARLY_SHADE: one C5 frame
                // 3.44-3.46 -> 3.37-3.40 ms); with frames in flight other frames' kernels fill that tail, and the
                // shading workgroups cost the in-flight rate 1-3% (r06_x): not then
                const BounceShade es{q[(b + 1) & 1], &qc[b + 1], b + 1 < bounces, c->d_redo[slot], &qc[17 + b], Pg};
                launch_bounce_traverse(ag, q[b & 1], &qc[b], perm, count, wk.bounce, hit, nxb, tblocks, sg, cert,
                                       c->d_defer[slot], cert && !inflight && !c->knob_no_early_shade ? &es : nullptr);
                if (tg && b == 0) HIPC(c, hipEventRecord(ev[4], sg));
                const Redo rd{c->d_redo[slot], &qc[17 + b], c->d_defer[slot], nxb};
                launch_bounce_shade(ag, q[b & 1], &qc[b], hit, q[(b + 1) & 1], &qc[b + 1], count, b + 1 < bounces,
                                    Pg, sg, cert ? &rd : nullptr);
            } else
                launch_bounce(ag, q[b & 1], &qc[b], perm, q[(b + 1) & 1], &qc[b + 1], count, b + 1 < bounces,
                              wk.nearest, sg);
        }
        if (g) {
            HIPC(c, hipEventRecord(c->ev_join[g], sg));
            HIPC(c, hipStreamWaitEvent(s, c->ev_join[g], 0));
        }
    }
    // a snapshot of the overflow word for this stream's slot (rtbvh_synchronize reports a change)
    HIPC(c, hipMemcpyAsync(c->h_ovf + slot, c->d_ovf, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    c->nsplit = nsplit;
    c->last_slot = slot;
    if (timing) {
        HIPC(c, hipEventRecord(ev[2], s));
        c->evt_trav[c->n_traces % rtbvh_ctx::RING] = refill && bounces > 0;
        c->n_traces++;
    }
    c->W = W;
    c->H = H;
    c->bounces = bounces;
    c->rank = rank;
    c->nranks = nranks;
    c->traced = true;
    c->frame_here = color == c->d_color && nranks == 1;
    c->intensity_here = c->frame_here && inten != nullptr;
    c->last_walk = flags & WALK_FLAGS;
    c->last_cert = cert;
    return check_launch(c, "trace kernels");
}

// ---- RTBVH_FLAG_AUTO_WALK: the certified fast walks ---------------------------------
// The fast walks return the lexicographic (t, leaf) minimum over the leaves they reach, findCollision
// (RayTraceTraversal.hlsl:106-193) the first strict minimum over the leaves IT reaches; they agree
// whenever every hit lies inside the boxes on its root path under the same rounding ("containment").
// Where containment fails they can differ (tests/containment.py).  The certified walks make each ray
// carry its own proof: they prune on boxes grown by the rounding margin of the triangle test
// (margin.h), so they see every triangle that could be accepted below their bound -- the minimum they
// return is the minimum over every triangle the reference could test -- and a ray's answer is the
// reference's when its winning leaf's own box passes the reference slab test at that t (the
// certificate).  Rays without one are re-traced in the reference order.  No per-frame check, no frame
// key: a moving camera costs nothing extra, and a captured frame replays as it is.
// The walks of a trace: (flags, certified)
struct TracePlan {
    uint32_t flags;
    bool cert;
    uint32_t state;   // rtbvh_stats.walk_state
};
TracePlan plan_trace(const rtbvh_ctx* c, uint32_t f) {
    if (!(f & (RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_CERTIFIED))) return TracePlan{f, false, 0};
    const uint32_t ref = f & ~WALK_FLAGS;
    // the certificate speaks for the reference order on a clz64 tree with the full stack (a run-time
    // stack limit makes the reference order end rays early, which no fast walk reproduces)
    const bool limited = c->cfg.stack_limit != 0 && c->cfg.stack_limit < (uint32_t)STACK_SIZE;
    const bool want = (f & RTBVH_FLAG_CERTIFIED) || auto_checked(c);
    if (!want || !c->built_clz64 || limited) return TracePlan{ref, false, 0};
    return TracePlan{ref | RTBVH_FLAG_NEAREST_FIRST | RTBVH_FLAG_REFILL_BOUNCE | RTBVH_FLAG_WIDE_BVH |
                         RTBVH_FLAG_BINNED_PRIMARY,
                     true, 2};
}

rtbvh_status enqueue_trace(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces, uint32_t rank, uint32_t nranks,
                           float4* color, float* inten, hipStream_t s, uint32_t slot = 0) {
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "trace before build");
    rtbvh_status st = sync_camera(c, s);
    if (st) return st;
    TracePlan p = plan_trace(c, c->cfg.flags);
    c->last_walk_state = p.state;
    if (p.cert && !c->capturing) c->cert_traces++;
    // AUTO_WALK on a small scene: the reference order, as one-ray-per-lane walks or as wave packets (the
    // same frame: both are the exact findCollision DFS per ray).  Which is faster depends on the scene
    // (C3, Test.obj: packets 0.089 against lanes 0.108 ms; C2, Image_Test.obj: 0.175 against 0.073), so
    // the first full-frame trace of a scene and frame size on the context stream times both primary
    // passes, twice each, and keeps the packets only when they are 5% faster.  Not while capturing: a
    // captured frame keeps the choice made before it (rtbvh_compute_bvh with RTBVH_FLAG_GRAPH traces a
    // frame uncaptured first).  Not with a stack limit (a wave packet shares one stack: its overflows
    // differ from a lane's) nor the CPUTests delta.
    const uint32_t f = c->cfg.flags;
    const bool limited = c->cfg.stack_limit != 0 && c->cfg.stack_limit < (uint32_t)STACK_SIZE;
    if ((f & RTBVH_FLAG_AUTO_WALK) && !p.cert && c->built_clz64 && !limited) {
        const uint64_t key = (uint64_t)W << 48 | (uint64_t)H << 32 | c->T;
        // (the first frame of a key is synchronous: it waits for its own timed passes; the key includes the
        // walk flags, so a set_flags that changes the walks times them again)
        const uint32_t fw = f & (WALK_FLAGS | RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_CERTIFIED | RTBVH_FLAG_SORT_BOUNCE);
        if ((c->small_key != key || c->small_flags != fw) && !c->capturing && s == c->stream && slot == 0 &&
            nranks == 1) {
            hipEvent_t* ev = c->ev_small;
            for (int k = 0; k < 2; k++)
                if (!ev[k]) HIPC(c, hipEventCreate(&ev[k]));
            float best[2] = {INFINITY, INFINITY};
            for (int round = 0; round < 2; round++)
                for (int k = 0; k < 2; k++) {
                    HIPC(c, hipEventRecord(ev[0], s));
                    rtbvh_status cs = enqueue_walks(c, W, H, 0, 0, 1, color, inten, s, 0,
                                                    p.flags | (k ? RTBVH_FLAG_PACKET_PRIMARY : 0u), false);
                    if (cs) return cs;
                    HIPC(c, hipEventRecord(ev[1], s));
                    HIPC(c, hipEventSynchronize(ev[1]));
                    float ms = 0.f;
                    HIPC(c, hipEventElapsedTime(&ms, ev[0], ev[1]));
                    best[k] = std::min(best[k], ms);
                }
            c->small_packet = best[1] < 0.95f * best[0];
            c->small_key = key;
            c->small_flags = fw;
        }
        if (c->small_key == key && c->small_flags == fw && c->small_packet) p.flags |= RTBVH_FLAG_PACKET_PRIMARY;
    }
    return enqueue_walks(c, W, H, bounces, rank, nranks, color, inten, s, slot, p.flags, true, p.cert);
}

}  // namespace

extern "C" {

int rtbvh_abi_version(void) { return RTBVH_ABI_VERSION; }
uint32_t rtbvh_stats_size(void) { return (uint32_t)sizeof(rtbvh_stats); }

void rtbvh_config_default(rtbvh_config* cfg) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->device = 0;
    cfg->morton_mode = RTBVH_MORTON_CPUTESTS;
    cfg->delta_mode = RTBVH_DELTA_CLZ64;
    for (int k = 0; k < 3; k++) {   // Graphics.cpp:528-529
        cfg->scene_bb_min[k] = -700.f;
        cfg->scene_bb_max[k] = 700.f;
    }
}

rtbvh_status rtbvh_create(const rtbvh_config* cfg, rtbvh_ctx** out) {
    if (!out) return fail(nullptr, RTBVH_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    rtbvh_ctx* c = new (std::nothrow) rtbvh_ctx();
    if (!c) return fail(nullptr, RTBVH_ERR_OOM, "host allocation failed");
    if (cfg) c->cfg = *cfg;
    else rtbvh_config_default(&c->cfg);
    if (c->cfg.morton_mode > 1 || c->cfg.delta_mode > 1 || c->cfg.reserved != 0) {
        delete c;
        return fail(nullptr, RTBVH_ERR_INVALID_ARG, "bad morton/delta mode");
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        delete c;
        return fail(nullptr, RTBVH_ERR_NO_DEVICE, "no HIP device");
    }
    if (c->cfg.device < 0 || c->cfg.device >= ndev || hipSetDevice(c->cfg.device) != hipSuccess) {
        delete c;
        return fail(nullptr, RTBVH_ERR_NO_DEVICE, "bad device ordinal");
    }
    if (c->cfg.stream) {
        c->stream = (hipStream_t)c->cfg.stream;
    } else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return fail(nullptr, RTBVH_ERR_HIP, "hipStreamCreate failed");
        }
        c->own_stream = true;
    }
    bool ev_ok = true;
    for (auto& row : c->evb)
        for (auto& e : row) ev_ok = ev_ok && hipEventCreate(&e) == hipSuccess;
    for (auto& row : c->evt)
        for (auto& e : row) ev_ok = ev_ok && hipEventCreate(&e) == hipSuccess;
    if (!ev_ok) {
        rtbvh_destroy(c);
        return fail(nullptr, RTBVH_ERR_HIP, "hipEventCreate failed");
    }
    if (hipEventCreateWithFlags(&c->ev_built, hipEventDisableTiming) != hipSuccess) {
        rtbvh_destroy(c);
        return fail(nullptr, RTBVH_ERR_HIP, "hipEventCreate failed");
    }
    if (hipMalloc((void**)&c->d_ovf, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_ovf, 0, sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc((void**)&c->h_ovf, sizeof(unsigned long long) * rtbvh_ctx::MAXSPLIT, hipHostMallocDefault) !=
            hipSuccess) {
        rtbvh_destroy(c);
        return fail(nullptr, RTBVH_ERR_OOM, "overflow counter allocation failed");
    }
    memset(c->h_ovf, 0, sizeof(unsigned long long) * rtbvh_ctx::MAXSPLIT);
    if (hipMalloc((void**)&c->d_cam, 32 * sizeof(float)) != hipSuccess ||
        hipMemset(c->d_cam, 0, 32 * sizeof(float)) != hipSuccess) {
        rtbvh_destroy(c);
        return fail(nullptr, RTBVH_ERR_OOM, "camera buffer allocation failed");
    }
    // A/B tuning knobs, read once here (not per frame)
    if (const char* e = getenv("RTBVH_BOUNCE_BLOCKS")) c->knob_bounce_blocks = (uint32_t)std::max(0, atoi(e));
    if (const char* e = getenv("RTBVH_OVERLAP")) c->knob_overlap = atoi(e) != 0;
    if (const char* e = getenv("RTBVH_SIDE_PRIORITY")) c->knob_side_priority = atoi(e) != 0;
    if (const char* e = getenv("RTBVH_KEEP_RECORDS")) c->knob_keep_records = atoi(e) != 0;
    if (const char* e = getenv("RTBVH_EARLY_SHADE")) c->knob_no_early_shade = atoi(e) == 0;   // (A/B: 0 = off)
    if (const char* e = getenv("RTBVH_PB_SMALL_TILES")) c->knob_no_small_tiles = atoi(e) == 0;   // (A/B: 0 = off)
    *out = c;
    return RTBVH_OK;
}

void rtbvh_destroy(rtbvh_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)
        if (c->ev_slot[k]) {
            (void)hipEventSynchronize(c->ev_slot[k]);   // frames in flight on caller streams
            (void)hipEventDestroy(c->ev_slot[k]);
        }
    if (c->ev_built) (void)hipEventDestroy(c->ev_built);
    drop_graph(c);
    for (uint32_t g = 1; g < rtbvh_ctx::MAXSPLIT; g++) {
        if (c->sub[g]) {
            (void)hipStreamSynchronize(c->sub[g]);
            (void)hipStreamDestroy(c->sub[g]);
        }
        if (c->ev_join[g]) (void)hipEventDestroy(c->ev_join[g]);
        dfree(c->d_qs[g][0]); dfree(c->d_qs[g][1]); dfree(c->d_hits[g]);
    }
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->side) {
        (void)hipStreamSynchronize(c->side);
        (void)hipStreamDestroy(c->side);
    }
    for (hipEvent_t e : c->ev_small)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_leaf) (void)hipEventDestroy(c->ev_leaf);
    if (c->ev_prim) (void)hipEventDestroy(c->ev_prim);
    for (auto& p : c->pb) { dfree(p.off); dfree(p.cur); dfree(p.bins); dfree(p.sums); dfree(p.keys); }
    dfree(c->d_opos); dfree(c->d_verts); dfree(c->d_idx); dfree(c->d_matidx); dfree(c->d_mats);
    dfree(c->d_codes); dfree(c->d_ids); dfree(c->d_ka); dfree(c->d_va); dfree(c->d_kb); dfree(c->d_vb);
    dfree(c->d_sort_scratch); dfree(c->d_tclip); dfree(c->d_leaf); dfree(c->d_inner); dfree(c->d_topo); dfree(c->d_rec); dfree(c->d_nbox); dfree(c->d_qnode); dfree(c->d_lfp);
    dfree(c->d_band);
    dfree(c->d_pleaf); dfree(c->d_pint); dfree(c->d_cnt); dfree(c->d_xlist); dfree(c->d_qlate); dfree(c->d_xcnt); dfree(c->d_bounds); dfree(c->d_rootbox); dfree(c->d_zpart);
    dfree(c->d_color); dfree(c->d_intensity); dfree(c->d_q[0]); dfree(c->d_q[1]); dfree(c->d_qcount); dfree(c->d_next); dfree(c->d_hit);
    dfree(c->d_bkin); dfree(c->d_bvin); dfree(c->d_bka); dfree(c->d_bva); dfree(c->d_bkb); dfree(c->d_bvb);
    dfree(c->d_bscratch); dfree(c->d_refl_rec); dfree(c->d_refr_rec);
    dfree(c->d_texels); dfree(c->d_texinfo); dfree(c->d_srgb);
    dfree(c->d_counters);
    dfree(c->d_ovf);
    for (auto& r : c->d_redo) dfree(r);
    for (auto& r : c->d_defer) dfree(r);
    for (auto& p : c->pb) dfree(p.list);
    dfree(c->d_cam);
    for (auto& t : c->deals) free_deal(t);
    if (c->h_ovf) (void)hipHostFree(c->h_ovf);
    for (auto& row : c->evb)
        for (auto& e : row)
            if (e) (void)hipEventDestroy(e);
    for (auto& row : c->evt)
        for (auto& e : row)
            if (e) (void)hipEventDestroy(e);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rtbvh_last_error(const rtbvh_ctx* c) { return c ? c->err.c_str() : g_create_error.c_str(); }

rtbvh_status rtbvh_set_scene(rtbvh_ctx* c, const rtbvh_vertex* verts, uint32_t nverts, const uint32_t* indices,
                             uint32_t nidx, const uint32_t* mat_idx, const rtbvh_material* mats, uint32_t nmats,
                             const rtbvh_texture* textures, uint32_t ntex) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    drop_graph(c);   // a captured frame holds the old buffers
    if (ntex && !textures) return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: ntex > 0 without textures");
    for (uint32_t k = 0; k < ntex; k++)
        if (textures[k].width == 0 || textures[k].height == 0 || !textures[k].rgba8)
            return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: empty texture");
    if (!verts || !indices || !mat_idx || !mats || nverts == 0 || nidx == 0 || nidx % 3 != 0 || nmats == 0)
        return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: empty or ragged input");
    const uint32_t T = nidx / 3;
    if (T >= (1u << 30)) return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: too many triangles");
    for (uint32_t i = 0; i < nidx; i++)
        if (indices[i] >= nverts) return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: index out of range");
    for (uint32_t t = 0; t < T; t++)
        if (mat_idx[t] >= nmats) return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: material index out of range");
    HIPC(c, hipSetDevice(c->cfg.device));
    HIPC(c, hipStreamSynchronize(c->stream));
    try {
        std::vector<float4> opos(nverts);
        for (uint32_t i = 0; i < nverts; i++)
            opos[i] = make_float4(verts[i].position[0], verts[i].position[1], verts[i].position[2], 0.f);
        HIPC(c, dalloc(c->d_opos, nverts));
        HIPC(c, dalloc(c->d_verts, (size_t)nverts * 8));
        HIPC(c, dalloc(c->d_idx, nidx));
        HIPC(c, dalloc(c->d_matidx, T));
        HIPC(c, dalloc(c->d_mats, nmats));
        HIPC(c, hipMemcpy(c->d_opos, opos.data(), sizeof(float4) * nverts, hipMemcpyHostToDevice));
        HIPC(c, hipMemcpy(c->d_verts, verts, sizeof(rtbvh_vertex) * nverts, hipMemcpyHostToDevice));
        HIPC(c, hipMemcpy(c->d_idx, indices, sizeof(uint32_t) * nidx, hipMemcpyHostToDevice));
        HIPC(c, hipMemcpy(c->d_matidx, mat_idx, sizeof(uint32_t) * T, hipMemcpyHostToDevice));
        HIPC(c, hipMemcpy(c->d_mats, mats, sizeof(rtbvh_material) * nmats, hipMemcpyHostToDevice));
        // textures: one texel array + a {first texel, width, height} table (t4-t5 of
        // RayTraceGlobal.hlsl:114-115, any count here)
        std::vector<uint4> info(ntex ? ntex : 1);
        size_t total = 0;
        for (uint32_t k = 0; k < ntex; k++) {
            info[k] = make_uint4((uint32_t)total, textures[k].width, textures[k].height, 0u);
            total += (size_t)textures[k].width * textures[k].height;
        }
        if (total >= (1ull << 32)) return fail(c, RTBVH_ERR_INVALID_ARG, "set_scene: textures too large");
        HIPC(c, dalloc(c->d_texels, total ? total : 1));
        HIPC(c, dalloc(c->d_texinfo, info.size()));
        for (uint32_t k = 0; k < ntex; k++)
            HIPC(c, hipMemcpy(c->d_texels + info[k].x, textures[k].rgba8,
                              (size_t)textures[k].width * textures[k].height * 4, hipMemcpyHostToDevice));
        HIPC(c, hipMemcpy(c->d_texinfo, info.data(), sizeof(uint4) * info.size(), hipMemcpyHostToDevice));
        if (!c->d_srgb) {
            float tab[256];
            rtbvh_srgb_table(tab);
            HIPC(c, dalloc(c->d_srgb, 256));
            HIPC(c, hipMemcpy(c->d_srgb, tab, sizeof(tab), hipMemcpyHostToDevice));
        }
        c->ntex = ntex;
    } catch (const std::bad_alloc&) {
        return fail(c, RTBVH_ERR_OOM, "set_scene: host allocation failed");
    }
    static_assert(sizeof(rtbvh_material) == sizeof(Mat), "material layout");
    c->V = nverts;
    c->T = T;
    c->nmat = nmats;
    rtbvh_status st = ensure_build_capacity(c, T);
    if (st) return st;
    if (c->cfg.morton_mode == RTBVH_MORTON_CPUTESTS) {
        // the object-space mesh box the CPUTests Morton codes are normalised by: a property of
        // the scene, computed once after loading as ShaderSim does (ShaderSim/main.cpp:277-285),
        // not per build (it does not depend on the camera)
        BuildArgs a = build_args(c);
        launch_bounds(a, c->stream);
        st = check_launch(c, "mesh bounds");
        if (st) return st;
        HIPC(c, hipStreamSynchronize(c->stream));
    }
    c->have_scene = true;
    c->built = false;
    c->small_key = 0;   // (the primary kind of a small scene is timed again)
    return RTBVH_OK;
}

rtbvh_status rtbvh_set_camera(rtbvh_ctx* c, const float wvp[16], const float wv[16]) {
    if (!c || !wvp || !wv) return RTBVH_ERR_INVALID_ARG;
    // Graphics::onUpdate writes the matrices every frame (Graphics.cpp:44-53); the kernels read them
    // from a device buffer (sync_camera), so a captured frame (RTBVH_FLAG_GRAPH) replays with the new
    // camera as it is
    if (c->have_camera && memcmp(c->wvp, wvp, sizeof(c->wvp)) == 0 && memcmp(c->wv, wv, sizeof(c->wv)) == 0)
        return RTBVH_OK;
    memcpy(c->wvp, wvp, sizeof(c->wvp));
    memcpy(c->wv, wv, sizeof(c->wv));
    c->have_camera = true;
    c->cam_dirty = true;
    return RTBVH_OK;
}

rtbvh_status rtbvh_build_async(rtbvh_ctx* c) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    if (!c->have_scene || !c->have_camera) return fail(c, RTBVH_ERR_NOT_READY, "build before set_scene/set_camera");
    HIPC(c, hipSetDevice(c->cfg.device));
    hipStream_t s = c->stream;
    const bool timing = (c->cfg.flags & RTBVH_FLAG_TIMING) != 0 && !c->capturing;
    BuildArgs a = build_args(c);
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)   // frames in flight read the old BVH
        if (c->slot_busy[k]) {
            HIPC(c, hipStreamWaitEvent(s, c->ev_slot[k], 0));
            c->slot_busy[k] = false;
        }
    rtbvh_status cst = sync_camera(c, s);
    if (cst) return cst;
    hipEvent_t* ev = c->evb[c->n_builds % rtbvh_ctx::RING];
    if (timing) HIPC(c, hipEventRecord(ev[0], s));
    if (c->T <= small_build_max() && !(c->cfg.flags & RTBVH_FLAG_MULTI_KERNEL_BUILD)) {
        // one workgroup (build.hip k_build_small); its time is reported as stage 0
        c->sorted = SortResult{c->d_ka, c->d_va};
        a.sorted_keys = c->d_ka;
        a.sorted_vals = c->d_va;
        a.pseudo = 1;   // (the one-workgroup build writes them anyway)
        a.rec_on = 1;   // (and the node records)
        a.nbox = nullptr;
        c->build_nbox = false;
        c->rec_ok = true;
        c->nbox_ok = false;
        launch_build_small(a, s);
        // the QNodes only for walks that read them (the 4-wide bounce walk; enqueue_walks otherwise)
        c->qnode_ok = (c->cfg.flags & (RTBVH_FLAG_WIDE_BVH | RTBVH_FLAG_CERTIFIED)) != 0 || auto_checked(c);
        if (c->qnode_ok) launch_qnodes(a, s);
        c->leaf_pending = false;
        c->tail_pending = false;
        c->pseudo_ok = true;
        if (timing) for (int k = 1; k <= 5; k++) HIPC(c, hipEventRecord(ev[k], s));
        if (timing) c->n_builds++;
        if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, s));
        c->built = true;
        c->built_clz64 = c->cfg.delta_mode == RTBVH_DELTA_CLZ64;
        return check_launch(c, "build kernel");
    }
    if (timing) HIPC(c, hipEventRecord(ev[1], s));   // (the mesh box is the scene's: rtbvh_set_scene)
    // a certified-only context's build: node boxes instead of node records (records_skipped)
    c->build_nbox = records_skipped(c);
    c->rec_ok = !c->build_nbox;
    c->nbox_ok = c->build_nbox;
    a.rec_on = c->build_nbox ? 0u : 1u;
    a.nbox = c->build_nbox ? c->d_nbox : nullptr;
    if (c->T <= small_sort_max() && !(c->cfg.flags & RTBVH_FLAG_MULTI_KERNEL_BUILD)) {
        // the Morton pass and the sort in one workgroup (build.hip k_morton_sort_small; stage "morton")
        c->sorted = SortResult{c->d_ka, c->d_va};
        a.sorted_keys = c->d_ka;
        a.sorted_vals = c->d_va;
        launch_morton_sort_small(a, s);
        if (timing) HIPC(c, hipEventRecord(ev[2], s));
    } else {
        launch_morton(a, s);
        if (timing) HIPC(c, hipEventRecord(ev[2], s));
        c->sorted = radix_sort_pairs(c->d_codes, c->d_ids, c->d_ka, c->d_va, c->d_kb, c->d_vb, c->T, 30,
                                     c->d_sort_scratch, s);
    }
    if (timing) HIPC(c, hipEventRecord(ev[3], s));
    a.sorted_keys = c->sorted.keys;
    a.sorted_vals = c->sorted.vals;
    launch_karras(a, s);
    if (timing) HIPC(c, hipEventRecord(ev[4], s));
    // leaf records, boxes, node records and QNodes; rtbvh_compute_bvh's primary pass may start
    // after the leaves (ev_leaf)
    launch_refit_leaves(a, s);
    c->pseudo_ok = a.pseudo != 0;
    c->qnode_ok = true;   // (quantized by the refit kernels)
    c->leaf_pending = false;
    if (c->leaf_want) {
        if (!c->side) {   // high priority: its workgroups go first while the crossing nodes' fill the CUs
            int lo = 0, hi = 0;
            HIPC(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
            if (!c->knob_side_priority) hi = lo;   // (A/B runs: RTBVH_SIDE_PRIORITY=0)
            HIPC(c, hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi));
        }
        if (!c->ev_leaf) HIPC(c, hipEventCreateWithFlags(&c->ev_leaf, hipEventDisableTiming));
        if (!c->ev_prim) HIPC(c, hipEventCreateWithFlags(&c->ev_prim, hipEventDisableTiming));
        HIPC(c, hipEventRecord(c->ev_leaf, s));
        c->leaf_pending = true;
    }
    if (c->tail_want && !c->leaf_pending) c->tail_pending = true;   // (the trace runs it: launch_pb_bin_tail)
    else launch_refit_tail(a, s);
    if (timing) HIPC(c, hipEventRecord(ev[5], s));
    if (timing) c->n_builds++;
    if (!c->capturing) HIPC(c, hipEventRecord(c->ev_built, s));
    c->built = true;
    c->built_clz64 = c->cfg.delta_mode == RTBVH_DELTA_CLZ64;
    return check_launch(c, "build kernels");
}

rtbvh_status rtbvh_build(rtbvh_ctx* c) {
    rtbvh_status st = rtbvh_build_async(c);
    if (st) return st;
    return rtbvh_synchronize(c);
}

rtbvh_status rtbvh_trace_async(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    HIPC(c, hipSetDevice(c->cfg.device));
    rtbvh_status st = ensure_trace_capacity(c, (size_t)W * H);
    if (st) return st;
    return enqueue_trace(c, W, H, bounces, 0, 1, c->d_color, c->d_intensity, c->stream);
}

rtbvh_status rtbvh_trace(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces) {
    rtbvh_status st = rtbvh_trace_async(c, W, H, bounces);
    if (st) return st;
    return rtbvh_synchronize(c);
}

// The binned primary pass of rtbvh_compute_bvh on a side stream beside the build's crossing nodes
// (ev_leaf / ev_prim): opt-in (RTBVH_OVERLAP=1).  A/B at C5: the rocprof frame span 5.07 -> ~4.95
// ms in a process with the context's own stream, but bench.py's context (a torch stream, the slot
// streams of frames in flight) ran every build kernel of the frame up to 10x slower while the side
// queue held its wait (6.28 ms per frame against 5.14 without; 5.81 at normal priority), and as a
// hipGraph it was +-0 (4.98 / 4.99 / 5.00 ms).
// the crossing nodes a build left to the trace, when the trace did not run (an error on the way)
static rtbvh_status flush_tail(rtbvh_ctx* c, rtbvh_status st) {
    if (c->tail_pending) {
        launch_refit_tail(build_args(c), c->stream);
        c->tail_pending = false;
    }
    return st;
}

static bool side_overlap(const rtbvh_ctx* c) { return c->knob_overlap; }

// RTBVH_FLAG_GRAPH: Graphics.cpp:56 rebuilds and traces every frame, ~20 launches and memsets
// of little work each on the reference's own meshes; the frame is captured once into a
// hipGraph and replayed.  A plain frame runs first so that every buffer exists before the
// capture; kernel arguments (sizes, buffers) are baked into the graph, hence the key and the
// drop on set_scene and reallocations.  The camera is not: the kernels read it from the
// context's camera buffer, updated before each replay (sync_camera), so a moving camera
// (Graphics::onKeyDown, Graphics.cpp:937-960) replays the same graph; and the certified walks
// (plan_trace) need no per-camera decision.
static rtbvh_status compute_graph(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces) {
    const uint64_t key[5] = {W, H, bounces, (uint64_t)c->cfg.flags | (uint64_t)c->T << 32,
                             (uint64_t)c->slots_used | (uint64_t)c->cfg.stack_limit << 1};
    if (!c->graph_exec || memcmp(key, c->graph_key, sizeof(key)) != 0) {
        drop_graph(c);
        c->leaf_want = side_overlap(c);
        c->tail_want = true;
        rtbvh_status st = rtbvh_build_async(c);
        c->leaf_want = c->tail_want = false;
        if (!st) st = rtbvh_trace_async(c, W, H, bounces);
        st = flush_tail(c, st);
        if (!st) st = rtbvh_synchronize(c);
        if (st && st != RTBVH_ERR_STACK_OVERFLOW) return st;
        HIPC(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        c->capturing = true;
        c->leaf_want = side_overlap(c);
        c->tail_want = true;
        st = rtbvh_build_async(c);
        c->leaf_want = c->tail_want = false;
        if (!st) st = rtbvh_trace_async(c, W, H, bounces);
        st = flush_tail(c, st);
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(c->stream, &g);
        c->capturing = false;
        if (st || e != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            return st ? st : fail(c, RTBVH_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
        }
        c->graph = g;
        HIPC(c, hipGraphInstantiate(&c->graph_exec, g, nullptr, nullptr, 0));
        memcpy(c->graph_key, key, sizeof(key));
        c->graph_state = rtbvh_ctx::TraceState{c->W,     c->H,         c->bounces,        c->nsplit,
                                                c->rec_P, c->last_walk, c->last_walk_state, c->last_cert};
        c->graph_captures++;
    }
    // the replayed build rewrites the BVH (and a split trace the slot queues): after the
    // frames in flight on caller streams, as rtbvh_build_async
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)
        if (c->slot_busy[k]) {
            HIPC(c, hipStreamWaitEvent(c->stream, c->ev_slot[k], 0));
            c->slot_busy[k] = false;
        }
    rtbvh_status cst = sync_camera(c, c->stream);   // this frame's camera, before the replay
    if (cst) return cst;
    HIPC(c, hipGraphLaunch(c->graph_exec, c->stream));
    HIPC(c, hipEventRecord(c->ev_built, c->stream));
    // the host-side state of the captured trace (a trace in between may have changed it)
    const rtbvh_ctx::TraceState& g = c->graph_state;
    c->W = g.W;
    c->H = g.H;
    c->bounces = g.bounces;
    c->nsplit = g.nsplit;
    c->rec_P = g.rec_P;
    c->last_walk = g.walk;
    c->last_walk_state = g.walk_state;
    c->last_cert = g.cert;
    if (g.cert) c->cert_traces++;
    c->rank = 0;
    c->nranks = 1;
    c->last_slot = 0;
    c->traced = c->built = true;
    c->built_clz64 = c->cfg.delta_mode == RTBVH_DELTA_CLZ64;
    c->frame_here = c->intensity_here = true;
    return rtbvh_synchronize(c);
}

rtbvh_status rtbvh_compute_bvh(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    if (c->cfg.flags & RTBVH_FLAG_GRAPH) return compute_graph(c, W, H, bounces);
    c->leaf_want = side_overlap(c);
    c->tail_want = true;
    rtbvh_status st = rtbvh_build_async(c);
    c->leaf_want = c->tail_want = false;
    if (st) return flush_tail(c, st);
    st = flush_tail(c, rtbvh_trace_async(c, W, H, bounces));
    if (st) return st;
    return rtbvh_synchronize(c);
}

// The identity check of a fast walk (DESIGN.md "Traversal orders"): the frame in the
// reference order (the exact findCollision DFS, RayTraceTraversal.hlsl:106-193) into a
// scratch buffer, then the frame with the context's walks into the framebuffer, compared
// on the device.  Leaves the context as rtbvh_trace with its own flags does.
rtbvh_status rtbvh_verify_walk(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces, uint64_t* differing) {
    if (!c || !differing) return RTBVH_ERR_INVALID_ARG;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "verify_walk before build");
    if (W == 0 || H == 0 || bounces > 14) return fail(c, RTBVH_ERR_INVALID_ARG, "bad trace dimensions");
    HIPC(c, hipSetDevice(c->cfg.device));
    rtbvh_status st = ensure_trace_capacity(c, (size_t)W * H);
    if (st) return st;
    const size_t n = (size_t)W * H;
    float4* ref = nullptr;
    unsigned long long* d_diff = nullptr;
    HIPC(c, hipMallocAsync((void**)&ref, n * sizeof(float4) + 256, c->stream));
    d_diff = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ref) + n * sizeof(float4));
    // the reference order, then the walks the context takes (AUTO: the certified fast walks above
    // AUTO_WALK_MAX_TRIS), without the ray records
    const uint32_t f = c->cfg.flags & ~RTBVH_FLAG_REFRACT_RECORDS;
    const uint32_t refw = f & ~(WALK_FLAGS | RTBVH_FLAG_AUTO_WALK);
    const TracePlan mine = plan_trace(c, f);
    st = sync_camera(c, c->stream);
    if (!st) st = enqueue_walks(c, W, H, bounces, 0, 1, ref, nullptr, c->stream, 0, refw, true);
    if (!st) {
        c->last_walk_state = mine.state;
        st = enqueue_walks(c, W, H, bounces, 0, 1, c->d_color, c->d_intensity, c->stream, 0, mine.flags, true,
                           mine.cert);
    }
    unsigned long long diff = 0;
    if (!st) {
        hipError_t e = hipMemsetAsync(d_diff, 0, sizeof(unsigned long long), c->stream);
        if (e == hipSuccess) {
            launch_count_diff(ref, c->d_color, n, d_diff, c->stream);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&diff, d_diff, sizeof(diff), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) st = fail(c, RTBVH_ERR_HIP, std::string("verify_walk: ") + hipGetErrorString(e));
    }
    (void)hipFreeAsync(ref, c->stream);
    if (st) return st;
    *differing = diff;
    return rtbvh_synchronize(c);
}

uint32_t rtbvh_band_rows(uint32_t H, uint32_t rank, uint32_t nranks) { return deal_rows(H, rank, nranks, 16); }

uint32_t rtbvh_deal_rows(uint32_t H, uint32_t rank, uint32_t nranks, uint32_t root_share) {
    return root_share > 16 ? 0 : deal_rows(H, rank, nranks, root_share);
}

uint32_t rtbvh_deal_bands(uint32_t H, uint32_t rank, uint32_t nranks, uint32_t root_share, uint32_t* bands,
                          uint32_t capacity) {
    if (nranks == 0 || rank >= nranks || root_share > 16) return 0;
    std::vector<uint32_t> owner;
    if (root_share == 16 || nranks == 1) {
        owner.resize((H + 7) / 8);
        for (uint32_t b = 0; b < owner.size(); b++) owner[b] = b % nranks;
    } else {
        deal_owners(H, nranks, root_share, owner);
    }
    uint32_t n = 0;
    for (uint32_t b = 0; b < owner.size(); b++)
        if (owner[b] == rank) {
            if (bands && n < capacity) bands[n] = b;
            n++;
        }
    return n;
}

rtbvh_status rtbvh_set_band_deal(rtbvh_ctx* c, uint32_t root_share) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    if (root_share > 16) return fail(c, RTBVH_ERR_INVALID_ARG, "set_band_deal: root_share > 16");
    c->root_share = root_share;
    return RTBVH_OK;
}

rtbvh_status rtbvh_trace_band_async(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces, uint32_t rank,
                                    uint32_t nranks, float* dev_out, void* stream) {
    if (!c || !dev_out) return RTBVH_ERR_INVALID_ARG;
    HIPC(c, hipSetDevice(c->cfg.device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    uint32_t slot = 0;
    if (s != c->stream) {   // a frame in flight: this stream's buffer slot, after the last build
        for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT && !slot; k++)
            if (c->slot_stream[k] == s) slot = k;
        for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT && !slot; k++)
            if (!c->slot_stream[k]) {
                c->slot_stream[k] = s;
                slot = k;
            }
        if (!slot) return fail(c, RTBVH_ERR_INVALID_ARG, "more caller streams trace one context than it has slots");
        if (!c->ev_slot[slot]) HIPC(c, hipEventCreateWithFlags(&c->ev_slot[slot], hipEventDisableTiming));
        c->slots_used = true;
        HIPC(c, hipStreamWaitEvent(s, c->ev_built, 0));
    }
    rtbvh_status st = enqueue_trace(c, W, H, bounces, rank, nranks, (float4*)dev_out, nullptr, s, slot);
    if (st) return st;
    if (slot) {   // the next build (context stream) waits for this trace
        HIPC(c, hipEventRecord(c->ev_slot[slot], s));
        c->slot_busy[slot] = true;
    }
    return RTBVH_OK;
}

rtbvh_status rtbvh_assemble_bands(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t nranks, const float* dev_bands,
                                  uint32_t stride_rows, float* dev_frame, void* stream) {
    if (!c || !dev_bands || !dev_frame || W == 0 || H == 0 || nranks == 0 ||
        stride_rows < deal_max_rows(H, nranks, c->root_share))
        return RTBVH_ERR_INVALID_ARG;
    HIPC(c, hipSetDevice(c->cfg.device));
    const rtbvh_ctx::DealTab* deal = nullptr;
    const hipStream_t as = stream ? (hipStream_t)stream : c->stream;
    rtbvh_status st = get_deal(c, H, nranks, &deal, as);
    if (st) return st;
    launch_assemble((const float4*)dev_bands, deal ? deal->d + (H + 7) / 8 : nullptr, stride_rows, W, H, nranks,
                    (float4*)dev_frame, as);
    return check_launch(c, "assemble bands");
}

rtbvh_status rtbvh_comm_unique_id(uint8_t id[RTBVH_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == RTBVH_COMM_ID_BYTES, "ncclUniqueId is 128 B");
    if (!id) return RTBVH_ERR_INVALID_ARG;
    const Rccl& r = rccl();
    if (!r.ok) return fail(nullptr, RTBVH_ERR_COMM, r.err);
    ncclUniqueId u;
    const ncclResult_t e = r.GetUniqueId(&u);
    if (e != ncclSuccess) return fail(nullptr, RTBVH_ERR_COMM, std::string("ncclGetUniqueId: ") + r.GetErrorString(e));
    memcpy(id, &u, sizeof(u));
    return RTBVH_OK;
}

rtbvh_status rtbvh_comm_init(rtbvh_ctx* c, uint32_t nranks, uint32_t rank, const uint8_t id[RTBVH_COMM_ID_BYTES],
                             void** comm) {
    if (!c || !id || !comm || nranks == 0 || rank >= nranks) return RTBVH_ERR_INVALID_ARG;
    const Rccl& r = rccl();
    if (!r.ok) return fail(c, RTBVH_ERR_COMM, r.err);
    HIPC(c, hipSetDevice(c->cfg.device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t cm = nullptr;
    const ncclResult_t e = r.CommInitRank(&cm, (int)nranks, u, (int)rank);
    if (e != ncclSuccess) return fail(c, RTBVH_ERR_COMM, std::string("ncclCommInitRank: ") + r.GetErrorString(e));
    *comm = cm;
    return RTBVH_OK;
}

rtbvh_status rtbvh_comm_destroy(void* comm) {
    if (!comm) return RTBVH_ERR_INVALID_ARG;
    const Rccl& r = rccl();
    if (!r.ok) return fail(nullptr, RTBVH_ERR_COMM, r.err);
    const ncclResult_t e = r.CommDestroy((ncclComm_t)comm);
    if (e != ncclSuccess) return fail(nullptr, RTBVH_ERR_COMM, std::string("ncclCommDestroy: ") + r.GetErrorString(e));
    return RTBVH_OK;
}

// bands of 8 rows dealt by the context's deal (rtbvh_set_band_deal); one RCCL
// group of point-to-point transfers into rank 0 (xGMI is point to point: each rank's shard
// travels its own link), then the row scatter on rank 0.  Rank 0's buffer holds every rank's
// bands, rank r at r * rows0 rows (rows0 = the most band rows any rank has).
rtbvh_status rtbvh_trace_tiles(rtbvh_ctx* c, uint32_t W, uint32_t H, uint32_t bounces, uint32_t rank,
                               uint32_t nranks, void* comm) {
    if (!c || !comm || W == 0 || H == 0 || nranks == 0 || rank >= nranks) return RTBVH_ERR_INVALID_ARG;
    const Rccl& r = rccl();
    if (!r.ok) return fail(c, RTBVH_ERR_COMM, r.err);
    HIPC(c, hipSetDevice(c->cfg.device));
    const uint32_t rows0 = deal_max_rows(H, nranks, c->root_share);
    const size_t need = (size_t)(rank == 0 ? nranks : 1) * rows0 * W;
    if (c->cap_band < need) {
        HIPC(c, dalloc(c->d_band, need));
        c->cap_band = need;
    }
    rtbvh_status st = enqueue_trace(c, W, H, bounces, rank, nranks, c->d_band, nullptr, c->stream);
    if (st) return st;
    const ncclComm_t cm = (ncclComm_t)comm;
    ncclResult_t e = r.GroupStart();
    if (rank != 0) {
        if (e == ncclSuccess)
            e = r.Send(c->d_band, (size_t)deal_rows(H, rank, nranks, c->root_share) * W * 4, ncclFloat32, 0, cm,
                       c->stream);
    } else {
        for (uint32_t q = 1; q < nranks && e == ncclSuccess; q++)
            e = r.Recv(c->d_band + (size_t)q * rows0 * W, (size_t)deal_rows(H, q, nranks, c->root_share) * W * 4,
                       ncclFloat32,
                       (int)q, cm, c->stream);
    }
    const ncclResult_t e2 = r.GroupEnd();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(c, RTBVH_ERR_COMM, std::string("band gather: ") + r.GetErrorString(e));
    if (rank == 0) {
        const rtbvh_ctx::DealTab* deal = nullptr;
        st = get_deal(c, H, nranks, &deal, c->stream);
        if (st) return st;
        launch_assemble(c->d_band, deal ? deal->d + (H + 7) / 8 : nullptr, rows0, W, H, nranks, c->d_color,
                        c->stream);
        st = check_launch(c, "assemble bands");
        if (st) return st;
    }
    c->frame_here = rank == 0;
    return rtbvh_synchronize(c);
}

rtbvh_status rtbvh_synchronize(rtbvh_ctx* c) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    HIPC(c, hipStreamSynchronize(c->stream));
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)   // and the frames in flight on caller streams
        if (c->slot_busy[k]) HIPC(c, hipEventSynchronize(c->ev_slot[k]));
    // each trace ends by copying the never-reset overflow word into its slot's pinned word
    unsigned long long ovf = c->ovf_seen;
    for (uint32_t k = 0; k < rtbvh_ctx::MAXSPLIT; k++)
        if (c->h_ovf[k] > ovf) ovf = c->h_ovf[k];
    if (ovf > c->ovf_seen) {
        const unsigned long long n = ovf - c->ovf_seen;
        c->ovf_seen = ovf;
        return fail(c, RTBVH_ERR_STACK_OVERFLOW,
                    "traversal stack overflow: " + std::to_string(n) +
                        " event(s) -- a per-lane walk's ray ended early, or a packet walk skipped a subtree "
                        "for the rays that hit it; each keeps the best hit found so far (stack limit " +
                        std::to_string(c->cfg.stack_limit ? c->cfg.stack_limit : (uint32_t)STACK_SIZE) +
                        " entries; the reference's 32-entry stack is unchecked, RayTraceTraversal.hlsl:9,115)");
    }
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_framebuffer(rtbvh_ctx* c, float* rgba) {
    if (!c || !rgba) return RTBVH_ERR_INVALID_ARG;
    if (!c->traced) return fail(c, RTBVH_ERR_NOT_READY, "no trace yet");
    if (!c->frame_here) return fail(c, RTBVH_ERR_NOT_READY, "the last trace was a band trace: the frame is elsewhere");
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(rgba, c->d_color, sizeof(float4) * (size_t)c->W * c->H, hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_intensity(rtbvh_ctx* c, float* inten) {
    if (!c || !inten) return RTBVH_ERR_INVALID_ARG;
    if (!c->traced || !c->intensity_here) return fail(c, RTBVH_ERR_NOT_READY, "no full-frame trace yet");
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(inten, c->d_intensity, sizeof(float) * (size_t)c->W * c->H, hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

const float* rtbvh_framebuffer_device(rtbvh_ctx* c) { return c ? (const float*)c->d_color : nullptr; }

rtbvh_status rtbvh_read_bvh(rtbvh_ctx* c, rtbvh_node* out, uint32_t capacity) {
    if (!c || !out) return RTBVH_ERR_INVALID_ARG;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "no build yet");
    const size_t total = 2 * (size_t)c->T - 1;
    if (capacity < total) return fail(c, RTBVH_ERR_INVALID_ARG, "read_bvh: capacity < 2n-1");
    HIPC(c, hipSetDevice(c->cfg.device));
    void* tmp = nullptr;
    HIPC(c, hipMalloc(&tmp, total * sizeof(rtbvh_node)));
    BuildArgs a = build_args(c);
    launch_export(a, tmp, c->stream);
    hipError_t e1 = hipGetLastError();
    hipError_t e2 = hipStreamSynchronize(c->stream);
    hipError_t e3 = hipMemcpy(out, tmp, total * sizeof(rtbvh_node), hipMemcpyDeviceToHost);
    (void)hipFree(tmp);
    HIPC(c, e1);
    HIPC(c, e2);
    HIPC(c, e3);
    return RTBVH_OK;
}

rtbvh_status rtbvh_present(rtbvh_ctx* c, uint8_t* rgba8) {
    if (!c || !rgba8) return RTBVH_ERR_INVALID_ARG;
    if (!c->traced || !c->frame_here) return fail(c, RTBVH_ERR_NOT_READY, "present: no full frame on this context");
    HIPC(c, hipSetDevice(c->cfg.device));
    const size_t n = (size_t)c->W * c->H;
    uint32_t* d = nullptr;
    HIPC(c, hipMallocAsync((void**)&d, n * 4, c->stream));
    launch_present(c->d_color, c->W, c->H, d, c->stream);
    hipError_t e1 = hipGetLastError();
    hipError_t e2 = hipMemcpyAsync(rgba8, d, n * 4, hipMemcpyDeviceToHost, c->stream);
    hipError_t e3 = hipFreeAsync(d, c->stream);
    hipError_t e4 = hipStreamSynchronize(c->stream);
    HIPC(c, e1);
    HIPC(c, e2);
    HIPC(c, e3);
    HIPC(c, e4);
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_wide(rtbvh_ctx* c, uint32_t* out, uint64_t capacity) {
    if (!c || !out) return RTBVH_ERR_INVALID_ARG;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "no build yet");
    const size_t total = c->T > 1 ? 2 * (size_t)(c->T - 1) : 0;
    if (capacity < total) return fail(c, RTBVH_ERR_INVALID_ARG, "read_wide: capacity < 2(n-1)");
    HIPC(c, hipSetDevice(c->cfg.device));
    rtbvh_status rs = ensure_records(c, c->stream);   // (a certified-only build wrote node boxes instead)
    if (rs) return rs;
    if (!c->pseudo_ok) {   // a build that wrote no leaf pseudo-records (binned / AUTO walks): now
        launch_pseudo(build_args(c), c->stream);
        c->pseudo_ok = true;
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    if (total) HIPC(c, hipMemcpy(out, c->d_rec, total * sizeof(Inner), hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_qnodes(rtbvh_ctx* c, uint32_t* out, uint64_t capacity) {
    if (!c || !out) return RTBVH_ERR_INVALID_ARG;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "no build yet");
    const size_t total = c->T > 1 ? 2 * (size_t)c->T - 1 : 0;
    if (capacity < total) return fail(c, RTBVH_ERR_INVALID_ARG, "read_qnodes: capacity < 2n-1");
    HIPC(c, hipSetDevice(c->cfg.device));
    if (!c->qnode_ok) {
        launch_qnodes(build_args(c), c->stream);
        c->qnode_ok = true;
    }
    HIPC(c, hipStreamSynchronize(c->stream));
    if (total) HIPC(c, hipMemcpy(out, c->d_qnode, total * sizeof(QNode), hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_morton(rtbvh_ctx* c, uint32_t* codes) {
    if (!c || !codes) return RTBVH_ERR_INVALID_ARG;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "no build yet");
    HIPC(c, hipStreamSynchronize(c->stream));
    HIPC(c, hipMemcpy(codes, c->d_codes, sizeof(uint32_t) * c->T, hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_sorted(rtbvh_ctx* c, uint32_t* keys, uint32_t* ids) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    if (!c->built) return fail(c, RTBVH_ERR_NOT_READY, "no build yet");
    HIPC(c, hipStreamSynchronize(c->stream));
    if (keys) HIPC(c, hipMemcpy(keys, c->sorted.keys, sizeof(uint32_t) * c->T, hipMemcpyDeviceToHost));
    if (ids) HIPC(c, hipMemcpy(ids, c->sorted.vals, sizeof(uint32_t) * c->T, hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

rtbvh_status rtbvh_read_rays(rtbvh_ctx* c, rtbvh_ray_present* reflect_out, rtbvh_ray_present* refract_out) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    if (!c->traced || c->rec_P == 0)
        return fail(c, RTBVH_ERR_NOT_READY, "read_rays: the last trace ran without RTBVH_FLAG_REFRACT_RECORDS");
    HIPC(c, hipSetDevice(c->cfg.device));
    HIPC(c, hipStreamSynchronize(c->stream));
    const size_t bytes = c->rec_P * sizeof(rtbvh_ray_present);
    if (reflect_out) HIPC(c, hipMemcpy(reflect_out, c->d_refl_rec, bytes, hipMemcpyDeviceToHost));
    if (refract_out) HIPC(c, hipMemcpy(refract_out, c->d_refr_rec, bytes, hipMemcpyDeviceToHost));
    return RTBVH_OK;
}

rtbvh_status rtbvh_get_stats(rtbvh_ctx* c, rtbvh_stats* out) {
    if (!c || !out) return RTBVH_ERR_INVALID_ARG;
    memset(out, 0, sizeof(*out));
    HIPC(c, hipStreamSynchronize(c->stream));
    for (uint32_t k = 1; k < rtbvh_ctx::MAXSPLIT; k++)
        if (c->slot_busy[k]) HIPC(c, hipEventSynchronize(c->ev_slot[k]));
    out->num_tris = c->T;
    out->num_nodes = c->T ? 2 * c->T - 1 : 0;
    out->width = c->W;
    out->height = c->H;
    const uint32_t nb = c->n_builds < (uint32_t)rtbvh_ctx::RING ? c->n_builds : rtbvh_ctx::RING;
    for (uint32_t k = 0; k < nb; k++) {
        float ms;
        HIPC(c, hipEventElapsedTime(&ms, c->evb[k][0], c->evb[k][5]));
        out->ms_build += ms / nb;
        for (int st = 0; st < 5; st++) {
            HIPC(c, hipEventElapsedTime(&ms, c->evb[k][st], c->evb[k][st + 1]));
            out->ms_stage[st] += ms / nb;
        }
    }
    out->timed_builds = nb;
    const uint32_t nt = c->n_traces < (uint32_t)rtbvh_ctx::RING ? c->n_traces : rtbvh_ctx::RING;
    for (uint32_t k = 0; k < nt; k++) {
        float ms;
        HIPC(c, hipEventElapsedTime(&ms, c->evt[k][0], c->evt[k][2]));
        out->ms_trace += ms / nt;
        HIPC(c, hipEventElapsedTime(&ms, c->evt[k][0], c->evt[k][1]));
        out->ms_stage[5] += ms / nt;
        HIPC(c, hipEventElapsedTime(&ms, c->evt[k][1], c->evt[k][2]));
        out->ms_stage[6] += ms / nt;
        if (c->evt_trav[k]) {
            HIPC(c, hipEventElapsedTime(&ms, c->evt[k][3], c->evt[k][4]));
            out->ms_stage[7] += ms / nt;
        }
    }
    out->timed_traces = nt;
    if (c->traced && c->d_counters) {
        unsigned long long cnt[64];
        uint32_t q[32 * rtbvh_ctx::MAXSPLIT];
        HIPC(c, hipMemcpy(cnt, c->d_counters + 64 * c->last_slot, sizeof(cnt), hipMemcpyDeviceToHost));
        HIPC(c, hipMemcpy(q, c->d_qcount + 32 * c->last_slot, sizeof(uint32_t) * 32 * c->nsplit,
                          hipMemcpyDeviceToHost));
        out->primary_rays = (uint64_t)c->W * deal_rows(c->H, c->rank, c->nranks, c->root_share);
        uint64_t b = 0;
        for (uint32_t g = 0; g < c->nsplit; g++)
            for (uint32_t k = 0; k < c->bounces; k++) b += q[32 * g + k];
        out->bounce_rays = b;
        for (int p = 0; p < 2; p++) {
            out->internal_visits[p] = cnt[2 + 3 * p];
            out->leaf_visits[p] = cnt[3 + 3 * p];
            out->hits[p] = cnt[4 + 3 * p];
        }
        out->stack_overflows = cnt[8];
        out->textured_hits = cnt[9];
        out->trav_wave_steps = cnt[10];
        out->trav_max_steps = cnt[13];
        out->trav_longest = cnt[20];
        for (int k = 0; k < 32; k++) out->trav_steps_log2[k] = cnt[32 + k];
        out->trav_mixed_steps = cnt[11];
        out->trav_active_lanes = cnt[12];
    }
    out->graph_captures = c->graph_captures;
    if (c->traced && c->d_counters) {
        unsigned long long w[4];
        HIPC(c, hipMemcpy(w, c->d_counters + 64 * c->last_slot + 14, sizeof(w), hipMemcpyDeviceToHost));
        out->packet_steps[0] = w[0];
        out->packet_steps[1] = w[1];
        out->bin_entries[0] = w[2];
        out->bin_entries[1] = w[3];
    }
    out->walk_flags = c->last_walk;
    out->walk_state = c->last_walk_state;
    out->cert_traces = c->cert_traces;
    if (c->traced && c->last_cert && c->d_qcount) {   // the last trace's re-trace counts (d_qcount 16..)
        uint32_t q[32];
        HIPC(c, hipMemcpy(q, c->d_qcount + 32 * c->last_slot, sizeof(q), hipMemcpyDeviceToHost));
        out->redo_rays[0] = q[16];
        for (uint32_t k = 0; k < c->bounces && k < 15; k++) out->redo_rays[1] += q[17 + k];
        // ... and the bounce walks' deferred rays (walked in the reference order by the walk or k_bounce_redo)
        for (uint32_t k = 0; k < c->bounces && k < 15; k++) {
            uint32_t nd = 0;
            HIPC(c, hipMemcpy(&nd, c->d_next + (size_t)NEXT_WORDS * c->last_slot + (size_t)NEXT_SEGS * NEXT_STRIDE * k +
                                       DEFER_COUNT, sizeof(nd), hipMemcpyDeviceToHost));
            out->redo_rays[1] += nd;
            out->redo_deferred += nd;
        }
    }
    out->redo_total = out->redo_rays[0] + out->redo_rays[1];
    return RTBVH_OK;
}

rtbvh_status rtbvh_set_flags(rtbvh_ctx* c, uint32_t flags) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    c->cfg.flags = flags;
    return RTBVH_OK;
}

rtbvh_status rtbvh_reset_stats(rtbvh_ctx* c) {
    if (!c) return RTBVH_ERR_INVALID_ARG;
    HIPC(c, hipStreamSynchronize(c->stream));
    c->n_builds = 0;
    c->n_traces = 0;
    return RTBVH_OK;
}

rtbvh_status rtbvh_sort_pairs_async(rtbvh_ctx* c, uint32_t* kin, uint32_t* vin, uint32_t* kout, uint32_t* vout,
                                    uint32_t n, uint32_t key_bits) {
    if (!c || (n && (!kin || !vin || !kout || !vout)) || key_bits == 0 || key_bits > 32)
        return RTBVH_ERR_INVALID_ARG;
    if (n == 0) return RTBVH_OK;
    HIPC(c, hipSetDevice(c->cfg.device));
    const uint32_t passes = (key_bits + RADIX_BITS - 1) / RADIX_BITS;
    uint32_t *tk = nullptr, *tv = nullptr, *scratch = nullptr;
    HIPC(c, hipMallocAsync((void**)&scratch, sort_scratch_words(n) * 4, c->stream));
    if (passes > 1) {
        HIPC(c, hipMallocAsync((void**)&tk, (size_t)n * 4, c->stream));
        HIPC(c, hipMallocAsync((void**)&tv, (size_t)n * 4, c->stream));
    }
    // odd pass count ends in A, even in B: arrange for the result to land in (kout, vout)
    if (passes & 1) radix_sort_pairs(kin, vin, kout, vout, tk, tv, n, key_bits, scratch, c->stream);
    else radix_sort_pairs(kin, vin, tk, tv, kout, vout, n, key_bits, scratch, c->stream);
    rtbvh_status st = check_launch(c, "sort kernels");
    (void)hipFreeAsync(scratch, c->stream);
    if (tk) (void)hipFreeAsync(tk, c->stream);
    if (tv) (void)hipFreeAsync(tv, c->stream);
    return st;
}

rtbvh_status rtbvh_sort_pairs_host(rtbvh_ctx* c, const uint32_t* keys, const uint32_t* vals, uint32_t* kout,
                                   uint32_t* vout, uint32_t n, uint32_t key_bits) {
    if (!c || (n && (!keys || !vals || !kout || !vout))) return RTBVH_ERR_INVALID_ARG;
    if (n == 0) return RTBVH_OK;
    HIPC(c, hipSetDevice(c->cfg.device));
    uint32_t* d = nullptr;
    HIPC(c, hipMalloc((void**)&d, (size_t)n * 16));
    uint32_t *dk = d, *dv = d + n, *ok = d + 2 * (size_t)n, *ov = d + 3 * (size_t)n;
    rtbvh_status st = RTBVH_OK;
    if (hipMemcpy(dk, keys, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dv, vals, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess)
        st = fail(c, RTBVH_ERR_HIP, "sort_pairs_host: upload failed");
    if (!st) st = rtbvh_sort_pairs_async(c, dk, dv, ok, ov, n, key_bits);
    if (!st && hipStreamSynchronize(c->stream) != hipSuccess) st = fail(c, RTBVH_ERR_HIP, "sort_pairs_host: sync");
    if (!st && (hipMemcpy(kout, ok, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(vout, ov, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess))
        st = fail(c, RTBVH_ERR_HIP, "sort_pairs_host: download failed");
    (void)hipFree(d);
    return st;
}

rtbvh_status rtbvh_build_from_codes(rtbvh_ctx* c, const uint32_t* sorted_codes, const float* leaf_boxes, uint32_t n,
                                    rtbvh_node* out) {
    if (!c || !sorted_codes || !leaf_boxes || !out || n == 0 || n >= (1u << 30)) return RTBVH_ERR_INVALID_ARG;
    HIPC(c, hipSetDevice(c->cfg.device));
    rtbvh_status st = ensure_build_capacity(c, n);
    if (st) return st;
    float* d_boxes = nullptr;
    void* d_out = nullptr;
    HIPC(c, hipMalloc((void**)&d_boxes, (size_t)n * 24));
    HIPC(c, hipMalloc(&d_out, (2 * (size_t)n - 1) * sizeof(rtbvh_node)));
    HIPC(c, hipMemcpy(c->d_ka, sorted_codes, (size_t)n * 4, hipMemcpyHostToDevice));
    HIPC(c, hipMemcpy(d_boxes, leaf_boxes, (size_t)n * 24, hipMemcpyHostToDevice));
    BuildArgs a = build_args(c);
    a.T = n;
    a.sorted_keys = c->d_ka;
    a.sorted_vals = nullptr;
    a.leaf = nullptr;
    a.rec_on = 1;   // (its QNodes and export read the records)
    a.nbox = nullptr;
    launch_from_codes(a, d_boxes, c->stream);
    launch_export(a, d_out, c->stream);
    st = check_launch(c, "build_from_codes kernels");
    hipError_t e = hipStreamSynchronize(c->stream);
    if (!st && e == hipSuccess) e = hipMemcpy(out, d_out, (2 * (size_t)n - 1) * sizeof(rtbvh_node), hipMemcpyDeviceToHost);
    (void)hipFree(d_boxes);
    (void)hipFree(d_out);
    if (st) return st;
    HIPC(c, e);
    c->built = false;   // the scene's BVH buffers were reused
    c->build_nbox = false;
    c->rec_ok = c->nbox_ok = false;
    return RTBVH_OK;
}

}  // extern "C"
