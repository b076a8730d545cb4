/*
 * rtbvh.h -- C ABI of librtbvh.so, the MI355X (gfx950) LBVH build + ray traversal path.
 *
 * Drop-in boundary for the reference's GPU hot path (Fierykev/RayTraceBVH).  The
 * reference has no plugin API: the whole path is the private member
 * Graphics::computeBVH() (Graphics.cpp:667-831), fed through a D3D12 binding
 * contract (RayTraceGlobal.hlsl:87-120, Graphics.h:50-83, Graphics.cpp:293-303)
 * by Graphics::onUpdate() (Graphics.cpp:40-61) with inputs produced by
 * ObjLoader (ObjectFileLoader.h:120-240).  Each entry point below names the
 * reference interface it replaces.  See INTEGRATION.md for the binding a
 * maintainer adds on the reference side.
 *
 * Conventions: plain pointers and sizes only, no C++ or torch types.  A context
 * is single-thread affine and owns one HIP stream (or uses the caller's) and
 * every device buffer it allocates.  Input arrays are owned by the caller and
 * copied on the call.  Calls never throw; they return rtbvh_status and leave a
 * message for rtbvh_last_error().  All calls are synchronous unless the name
 * says `_async` (those only enqueue on the context stream).
 */
#ifndef RTBVH_H
#define RTBVH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTBVH_ABI_VERSION 8

typedef enum {
    RTBVH_OK = 0,
    RTBVH_ERR_INVALID_ARG = 1,
    RTBVH_ERR_HIP = 2,            /* a HIP runtime call failed (message has the HIP error) */
    RTBVH_ERR_OOM = 3,
    RTBVH_ERR_NOT_READY = 4,      /* e.g. trace before build, build before set_scene */
    RTBVH_ERR_STACK_OVERFLOW = 5, /* rays of a trace hit rtbvh_config.stack_limit (or a cyclic CPUTests-delta
                                     tree tripped the walk-length guard): the frame is complete; a per-lane
                                     walk's ray ended early, a packet walk skipped the subtree for the rays
                                     that hit it, each with the best hit found so far (stats.stack_overflows
                                     counts those rays per event); returned by the synchronising call
                                     after the trace (rtbvh_trace, rtbvh_compute_bvh, rtbvh_trace_tiles,
                                     rtbvh_synchronize), once per new overflow.  The reference's 32-entry
                                     stack is unchecked (RayTraceTraversal.hlsl:9,115,187). */
    RTBVH_ERR_IO = 6,             /* scene file could not be read / parsed */
    RTBVH_ERR_NO_DEVICE = 7,
    RTBVH_ERR_COMM = 8            /* RCCL missing or an RCCL call failed (message has the RCCL error) */
} rtbvh_status;

/* ---- data layouts (byte-identical to the reference's HLSL structs) -------- */

/* Vertex, RayTraceGlobal.hlsl:53-58 / ObjectFileLoader.h:98-103 (32 B) */
typedef struct {
    float position[3];
    float normal[3];
    float texcoord[2];
} rtbvh_vertex;

/* Material as uploaded, RayTraceGlobal.hlsl:60-72 / MaterialUpload ObjectFileLoader.h:79-96 (68 B) */
typedef struct {
    float ambient[4];
    float diffuse[4];
    float specular[4];
    float shininess;
    float optical_density;
    float alpha;
    uint32_t specularb; /* HLSL bool = 4 bytes */
    int32_t tex_num;    /* -1 = untextured */
} rtbvh_material;

/* Node, RayTraceGlobal.hlsl:39-51 / Graphics.h:157-169 (44 B).  Export layout
 * of rtbvh_read_bvh: leaves [0,n), internal node k at n+k, root at n.
 * parent of the root and child_l/child_r of leaves = 0xFFFFFFFF; internal
 * nodes have code = 0 and index = 0 (the reference leaves sort scratch there). */
typedef struct {
    uint32_t parent, child_l, child_r, code;
    float bb_min[3], bb_max[3];
    uint32_t index; /* 3 * triangle id, for leaves */
} rtbvh_node;

/* RayPresent, RayTraceGlobal.hlsl:30-35 (56 B) */
typedef struct {
    float intensity;
    float origin[3], direction[3], inv_direction[3];
    float color[4];
} rtbvh_ray_present;

/* An RGBA8 texture (sRGB encoded, as the reference's R8G8B8A8_UNORM_SRGB, Image.cpp:9).
 * Row 0 is the first row ilCopyPixels returns (Image.cpp:48-49; DevIL without IL_ORIGIN_SET
 * keeps the file's own row order: the bottom row first for BMP, the top row for JPEG) and
 * is texture row v = 0.  Sampling (RayTraceRender.hlsl:22-26, sampler Image.cpp:154-169:
 * MIN_MAG_MIP_LINEAR, WRAP, SampleLevel 0), as restated here (parity unpinned: DevIL and
 * the D3D filter precision are not available): texels decoded sRGB -> linear through the
 * table of rtbvh_srgb_table (alpha / 255), x = u*W - 0.5, y = v*H - 0.5, wrap, and
 * bilinear in fp32 as lerp(lerp(t00, t10, fx), lerp(t01, t11, fx), fy). */
typedef struct {
    uint32_t width, height;
    const uint8_t* rgba8; /* width*height*4 bytes */
} rtbvh_texture;

enum {
    RTBVH_MORTON_CPUTESTS = 0, /* ShaderSim/main.cpp:292-301: object-space centroid, mesh AABB, x<<2|y<<1|z (default) */
    RTBVH_MORTON_HLSL = 1      /* MortonCodes.hlsl:70-106: clip-space, avg=bbMin/3, config scene box, x|y<<1|z<<2 */
};
enum {
    RTBVH_DELTA_CLZ64 = 0,   /* BVHConstructP1.hlsl:61-72: clz, ties 32 + clz(i^j) (default, always valid) */
    RTBVH_DELTA_CPUTESTS = 1 /* RadixBVHCombo/main.cpp:136-151: ties clz(i^j), De Bruijn quirks */
};
enum {
    RTBVH_FLAG_TIMING = 1u << 0,         /* record per-stage hipEvent times (rtbvh_get_stats) */
    RTBVH_FLAG_COUNT_VISITS = 1u << 1,   /* count traversal visits (slower; for the byte model) */
    RTBVH_FLAG_REFRACT_RECORDS = 1u << 2, /* keep the reflectRay and refractRay RayPresent records
                                             (RayTraceLaunch.hlsl:48-80, RayTraceReflection.hlsl:24-55)
                                             for rtbvh_read_rays */
    RTBVH_FLAG_SORT_BOUNCE = 1u << 3,     /* sort live bounce rays by (octant, origin Morton) before
                                             tracing them: same results, better coherence for the
                                             reference-order traversal */
    RTBVH_FLAG_NEAREST_FIRST = 1u << 4,   /* visit the nearer child first and keep the lexicographic
                                             (t, leaf) minimum: the reference DFS's answer unless
                                             rounding breaks box/triangle containment */
    RTBVH_FLAG_PACKET_PRIMARY = 1u << 5,  /* primary rays: one wave walks its 8x8 tile's rays as a
                                             masked packet with scalar node fetches (same per-ray
                                             visit sequence, same results) */
    RTBVH_FLAG_REFILL_BOUNCE = 1u << 6,   /* bounce rays: persistent traversal whose lanes take a new
                                             ray as soon as theirs is done, then a shading pass */
    RTBVH_FLAG_WIDE_BVH = 1u << 7,        /* trace: walk the node records 4-wide (a node's four grandchild
                                             boxes share one 128-B line), keeping the lexicographic
                                             (t, leaf) minimum as NEAREST_FIRST does */
    RTBVH_FLAG_AUTO_WALK = 1u << 8,       /* choose the walks, ignoring the walk flags (the four above and
                                             BINNED_PRIMARY), and return the reference-order frame always: up
                                             to 65536 triangles the reference-order kernels (exact by
                                             construction; the fastest on the reference's own meshes), the
                                             primary rays per lane or per wave packet, whichever the first
                                             frame of a (W, H, scene) timed faster (stats walk_flags); above
                                             that, the CERTIFIED fast walks: BINNED_PRIMARY and
                                             the 4-wide bounce walk, pruning on boxes grown by the triangle
                                             test's rounding margin so that they see every triangle that could
                                             be accepted below their bound, then a per-ray certificate (the
                                             winning leaf's own box passes the reference slab test at its t);
                                             the rays without one are re-traced in the reference order
                                             (stats walk_state 2, redo_rays).  No per-frame or per-camera check.
                                             The reference order throughout with a stack_limit below the
                                             capacity or the CPUTests delta */
    RTBVH_FLAG_BINNED_PRIMARY = 1u << 9,  /* primary rays: every leaf listed in the 32 x 32 screen tiles its box
                                             covers (the set of orthographic primary rays a box passes is a
                                             pixel rectangle, recorded by the build), then per tile each listed
                                             leaf tested against the pixels of its rectangle whose bound its
                                             min.z does not exceed, nearest depth bucket first, the (t, leaf)
                                             keys in LDS: the lexicographic minimum of the 4-wide walks, with no
                                             dependent record fetches.  Frames up to 32768 pixels
                                             a side (larger ones take the 4-wide packet walk); a tile whose bins
                                             overflow takes the per-lane nearest-first walk */
    RTBVH_FLAG_CERTIFIED = 1u << 10,      /* the certified fast walks of RTBVH_FLAG_AUTO_WALK whatever the scene's
                                             size (the reference-order frame, per-ray certificates) */
    RTBVH_FLAG_MULTI_KERNEL_BUILD = 1u << 16, /* scenes of <= 2048 triangles: use the multi-kernel
                                              build instead of the one-workgroup build (same output) */
    /* bits 17..19: trace chains (0 = automatic, n = 1..4): a trace deals its bands over n
       independent primary -> bounce kernel chains on n streams (same results) */
    RTBVH_FLAG_SPLIT_SHIFT = 17,
    RTBVH_FLAG_GRAPH = 1u << 20   /* rtbvh_compute_bvh replays one hipGraph of the whole frame (build +
                                     trace: ~20 launches and memsets), captured on the first call and
                                     re-captured when W, H, bounces, the flags or the scene change (not
                                     the camera: the kernels read it from a device buffer updated before
                                     each replay); no per-stage times (rtbvh_get_stats) */
};

typedef struct {
    int32_t device;          /* HIP device ordinal */
    uint32_t morton_mode;    /* RTBVH_MORTON_* */
    uint32_t delta_mode;     /* RTBVH_DELTA_* */
    uint32_t flags;          /* RTBVH_FLAG_* */
    float scene_bb_min[3];   /* MORTON_HLSL only: cbuffer sceneBBMin (Graphics.cpp:529 uses -700) */
    float scene_bb_max[3];   /* MORTON_HLSL only: cbuffer sceneBBMax (Graphics.cpp:528 uses +700) */
    void* stream;            /* hipStream_t to use, or NULL: the context creates its own */
    uint32_t stack_limit;    /* traversal stack entries a ray may use, 0 = the compiled capacity (66 binary,
                                100 for the 4-wide primary packets, 192 for the 4-wide bounce walk; a clz64
                                tree never needs more); 32 = the reference's stack
                                (RayTraceTraversal.hlsl:9): rays that would overflow it end early and the
                                trace reports RTBVH_ERR_STACK_OVERFLOW */
    uint32_t reserved;       /* must be 0 */
} rtbvh_config;

typedef struct {
    uint32_t num_tris, num_nodes, width, height;
    uint64_t primary_rays, bounce_rays;        /* rays traced by the last trace */
    /* RTBVH_FLAG_COUNT_VISITS only, last trace; [0] = primary pass, [1] = bounce passes */
    uint64_t internal_visits[2], leaf_visits[2], hits[2];
    uint64_t textured_hits, stack_overflows;
    /* RTBVH_FLAG_TIMING only: hipEvent averages over the builds / traces enqueued on
     * the context stream since rtbvh_reset_stats (the most recent 32 of each) */
    uint32_t timed_builds, timed_traces;
    float ms_build, ms_trace;
    float ms_stage[8];   /* 0 (the mesh box is computed by set_scene), morton, sort, karras, refit (+ leaf and node
                            records, QNodes), primary, bounce (all passes),
                            first bounce pass's traversal kernel (RTBVH_FLAG_REFILL_BOUNCE) */
    /* RTBVH_FLAG_COUNT_VISITS with RTBVH_FLAG_REFILL_BOUNCE: wave iterations of the bounce
     * traversal, those with both a leaf lane and an internal-node lane, and active lanes
     * summed over iterations (lane utilisation = active_lanes / (64 * wave_steps)) */
    uint64_t trav_wave_steps, trav_mixed_steps, trav_active_lanes;
    /* ... and the walk length of the bounce rays (loop iterations per ray): the longest,
     * and a histogram, [k] = rays of floor(log2(iterations)) == k */
    uint64_t trav_max_steps, trav_steps_log2[32];
    uint64_t graph_captures;   /* RTBVH_FLAG_GRAPH: frames captured so far (a replay captures nothing) */
    uint32_t walk_flags;       /* the walk flags the last trace's frame was traced with (RTBVH_FLAG_AUTO_WALK:
                                  the reference order, or the four walk flags once verified) */
    uint32_t walk_state;       /* RTBVH_FLAG_AUTO_WALK, last trace: 0 the reference order (<= 65536 triangles,
                                  a stack limit, the CPUTests delta) or no AUTO; 2 the certified fast walks */
    /* RTBVH_FLAG_COUNT_VISITS, wave-packet primary walks: wave steps (one record fetch for the
     * wave each) at internal nodes [0] and at leaves [1] */
    uint64_t packet_steps[2];
    /* RTBVH_FLAG_AUTO_WALK: traces run with the certified walks since rtbvh_create, and the rays the last
     * one re-traced in the reference order (no certificate: redo_rays[0] + redo_rays[1]).  ABI 7 renamed
     * them (ABI <= 5: walk_checks counted device frame checks and walk_fallbacks frame keys that fell back
     * to the reference order; a re-traced ray is normal, not a wrong fast walk) */
    uint64_t cert_traces, redo_total;
    /* RTBVH_FLAG_COUNT_VISITS, RTBVH_FLAG_BINNED_PRIMARY: (leaf, screen tile) bin entries of the primary
     * pass [0] and those that passed the tile's 8 x 8-block bound test [1] (one leaf-record fetch each) */
    uint64_t bin_entries[2];
    /* RTBVH_FLAG_AUTO_WALK, last trace: the rays re-traced in the reference order because their certificate
     * failed, of the primary pass [0] and of the bounce passes [1] (deferred rays included) */
    uint64_t redo_rays[2];
    /* RTBVH_FLAG_COUNT_VISITS with RTBVH_FLAG_REFILL_BOUNCE, last trace: the longest bounce walk, as its
     * loop iterations << 32 | the pixel (framebuffer index) of its ray */
    uint64_t trav_longest;
    /* RTBVH_FLAG_AUTO_WALK, last trace (ABI 8): of redo_rays[1], the bounce rays the certified walk's margin does
     * not cover (a direction component under 2^-20, |d| off unit, |o| > 2^90), deferred at their first step and
     * walked in the reference order by the walk's drained waves or the re-trace kernel */
    uint64_t redo_deferred;
} rtbvh_stats;
typedef struct rtbvh_ctx rtbvh_ctx;

/* ---- lifecycle ------------------------------------------------------------ */
/* Fills cfg with defaults (device 0, CPUTests Morton, clz64 delta, +-700 box). */
void rtbvh_config_default(rtbvh_config* cfg);
/* Replaces Graphics::onInit/loadPipeline device + queue creation (Graphics.cpp:34-38,110-235). */
rtbvh_status rtbvh_create(const rtbvh_config* cfg, rtbvh_ctx** out);
/* Replaces Graphics::onDestroy (Graphics.cpp:94-103). NULL is a no-op. */
void rtbvh_destroy(rtbvh_ctx* ctx);
/* Last error message of this context (or of the last failed rtbvh_create when ctx == NULL). */
const char* rtbvh_last_error(const rtbvh_ctx* ctx);
int rtbvh_abi_version(void);
/* sizeof(rtbvh_stats) as this library was built: a binding checks its mirror of the struct against it */
uint32_t rtbvh_stats_size(void);

/* ---- inputs (the binding contract, RayTraceGlobal.hlsl:87-120) ------------ */
/* SRV t0 verts, t1 indices, t2 matIndices, t3 materials, t4.. textures:
 * replaces ObjLoader::UploadData (ObjectFileLoader.cpp:549-624).  nidx must be
 * a positive multiple of 3; mat_idx has nidx/3 entries; textures may be NULL. */
rtbvh_status rtbvh_set_scene(rtbvh_ctx* ctx, const rtbvh_vertex* verts, uint32_t nverts,
                             const uint32_t* indices, uint32_t nidx, const uint32_t* mat_idx,
                             const rtbvh_material* mats, uint32_t nmats,
                             const rtbvh_texture* textures, uint32_t ntex);
/* cbuffer WORLD_POS (b0) {WVP, WV}: replaces the CB write in Graphics::onUpdate
 * (Graphics.cpp:50-53).  Row-major 4x4, row-vector convention (p' = [p 1] * M),
 * i.e. the DirectXMath matrices BEFORE the transpose for HLSL packing. */
rtbvh_status rtbvh_set_camera(rtbvh_ctx* ctx, const float wvp[16], const float wv[16]);

/* ---- the hot path (Graphics::computeBVH, Graphics.cpp:667-831) ------------ */
/* MortonCodes -> radix sort -> BVHConstructP1 -> BVHConstructP2 (Graphics.cpp:705-782). */
rtbvh_status rtbvh_build(rtbvh_ctx* ctx);
rtbvh_status rtbvh_build_async(rtbvh_ctx* ctx);
/* RayTraceLaunch + `bounces` x RayTraceReflection (Graphics.cpp:785-810) at W x H. */
rtbvh_status rtbvh_trace(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t bounces);
rtbvh_status rtbvh_trace_async(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t bounces);
/* The whole computeBVH: build + trace (Graphics.cpp:667-831). */
rtbvh_status rtbvh_compute_bvh(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t bounces);
/* Image-tile shard for multi-GPU (no reference equivalent): trace
 * only this rank's 8-row bands of a W x H frame under the context's deal (rtbvh_set_band_deal;
 * by default b % nranks == rank) and write them compacted (band order) as RGBA f32 into
 * dev_out (device memory, at least rtbvh_deal_rows(H, rank, nranks, share) * W * 4 floats,
 * = rtbvh_band_rows(H, rank, nranks) for the default deal), enqueued on `stream`
 * (hipStream_t, NULL = the context stream).  The caller gathers the shards.
 * Frames in flight: each caller stream other than the context's (up to 3) gets trace
 * buffers of its own over the one BVH, so traces on different streams run concurrently
 * (each into its own dev_out); they wait for the last build, and the next build waits for
 * them; rtbvh_synchronize waits for them too, and rtbvh_get_stats reports the last
 * trace.  Ray records (RTBVH_FLAG_REFRACT_RECORDS) are traced on the context stream only. */
rtbvh_status rtbvh_trace_band_async(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t bounces,
                                    uint32_t rank, uint32_t nranks, float* dev_out, void* stream);
uint32_t rtbvh_band_rows(uint32_t height, uint32_t rank, uint32_t nranks);
/* The band deal.  Bands b = 0 .. ceil(H/8)-1 go to the ranks by smooth weighted round-robin:
 * rank 0 weighs root_share (0..16), every other rank 16; per band each rank's credit grows by its
 * weight and the rank with the most credit (lowest rank on a tie) takes the band and pays the total
 * weight.  root_share 16 (the default) is b % nranks; below 16, rank 0 -- which also receives and
 * assembles every other rank's bands -- traces root_share/16 of another rank's share, spread evenly
 * over the frame.  rtbvh_deal_bands writes rank's band indices in order (up to capacity) and
 * returns their count; rtbvh_deal_rows returns its rows.  rtbvh_set_band_deal sets the context's
 * deal for rtbvh_trace_band_async, rtbvh_assemble_bands and rtbvh_trace_tiles (every rank must use
 * the same root_share). */
uint32_t rtbvh_deal_bands(uint32_t height, uint32_t rank, uint32_t nranks, uint32_t root_share, uint32_t* bands,
                          uint32_t capacity);
uint32_t rtbvh_deal_rows(uint32_t height, uint32_t rank, uint32_t nranks, uint32_t root_share);
rtbvh_status rtbvh_set_band_deal(rtbvh_ctx* ctx, uint32_t root_share);
/* The per-scene identity check of a fast walk: traces the W x H frame in the reference order
 * (the exact findCollision DFS) and with the context's walk flags, compares the two on the device
 * and stores the number of pixels whose RGBA bits differ (0: the fast walk renders this frame
 * exactly as the reference order).  Synchronous; afterwards the context holds the frame of its
 * own walks, as after rtbvh_trace. */
rtbvh_status rtbvh_verify_walk(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t bounces,
                               uint64_t* differing_pixels);
/* The frame from the ranks' compact band buffers, all on this device: buffer r (rank r's
 * rtbvh_trace_band_async output) starts stride_rows * W * 4 floats after buffer r-1
 * (stride_rows >= the most rows any rank has under the context's deal: rtbvh_deal_rows);
 * writes W*H*4 floats to dev_frame.
 * Enqueued on `stream` (NULL = the context stream).  rtbvh_trace_tiles uses it on rank 0. */
rtbvh_status rtbvh_assemble_bands(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t nranks,
                                  const float* dev_bands, uint32_t stride_rows, float* dev_frame, void* stream);

/* ---- multi-GPU inside the library: one context per rank/GPU ----------
 * For a C/C++ host with no framework of its own.  RCCL is resolved at run time: the
 * process's librccl.so.1 if one is loaded (e.g. PyTorch's), else the system's; librtbvh.so
 * has no link-time RCCL dependency (RTBVH_ERR_COMM if none can be loaded).
 * rtbvh_comm_unique_id on rank 0, share the bytes with every rank (any channel), then
 * rtbvh_comm_init on every rank.  `comm` is an ncclComm_t; a host's own communicator
 * (one rank per GPU, same rank numbering) may be passed to rtbvh_trace_tiles instead. */
#define RTBVH_COMM_ID_BYTES 128
rtbvh_status rtbvh_comm_unique_id(uint8_t id[RTBVH_COMM_ID_BYTES]);
rtbvh_status rtbvh_comm_init(rtbvh_ctx* ctx, uint32_t nranks, uint32_t rank, const uint8_t id[RTBVH_COMM_ID_BYTES],
                             void** comm);
rtbvh_status rtbvh_comm_destroy(void* comm);
/* computeBVH's trace on nranks GPUs: this rank traces its 8-row bands (as
 * rtbvh_trace_band_async), every rank sends its bands to rank 0 (ncclSend / ncclRecv on the
 * context stream, one group) and rank 0 assembles the frame.  Collective: every rank calls
 * it with the same W, H, bounces.  Returns when this rank's part is done; afterwards
 * rtbvh_read_framebuffer / rtbvh_present on rank 0 give the whole frame (other ranks:
 * RTBVH_ERR_NOT_READY). */
rtbvh_status rtbvh_trace_tiles(rtbvh_ctx* ctx, uint32_t width, uint32_t height, uint32_t bounces, uint32_t rank,
                               uint32_t nranks, void* comm);
rtbvh_status rtbvh_synchronize(rtbvh_ctx* ctx);

/* ---- outputs --------------------------------------------------------------- */
/* reflectRay[].color, the framebuffer of record (RayTraceBVHPS.hlsl:13-16): W*H*4 floats, row y at y*W. */
rtbvh_status rtbvh_read_framebuffer(rtbvh_ctx* ctx, float* rgba);
/* Final reflectRay[].intensity per pixel (W*H floats). */
rtbvh_status rtbvh_read_intensity(rtbvh_ctx* ctx, float* intensity);
/* What the presentation pass shows (RayTraceBVHPS.hlsl:13-16 into the R8G8B8A8_UNORM swap
 * chain, Graphics.cpp:163): screen row y (top = 0) is framebuffer row H-1-y (the shader's
 * index at pixel centres), each channel floor(saturate(c) * 255 + 0.5).  W*H*4 bytes, of
 * the last full-frame trace (not of a band trace). */
rtbvh_status rtbvh_present(rtbvh_ctx* ctx, uint8_t* rgba8);
/* SaveBMP (SaveBMP.cpp:3-62): 24-bit BI_RGB file, 0x0ec4 pixels per metre, rows bottom-up;
 * `rgba8` is a presented image (top row first).  Rows are padded to 4 bytes as BMP
 * requires (the reference writes them unpadded; identical when 3*W is a multiple of 4). */
rtbvh_status rtbvh_save_bmp(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height);
/* Device pointer of the W*H*4-float framebuffer (valid until the next trace/destroy). */
const float* rtbvh_framebuffer_device(rtbvh_ctx* ctx);
/* BVHTree UAV u0 in the reference layout (2n-1 nodes, see rtbvh_node). */
rtbvh_status rtbvh_read_bvh(rtbvh_ctx* ctx, rtbvh_node* out, uint32_t capacity);
/* Node records in slots (the layout every traversal walk reads): 2(n-1) records of 16 u32;
 * record 2p+side belongs to c = child `side` of internal node p and holds the boxes of
 * c's children L and R as words {L.min.x, L.min.y, L.max.x, L.max.y, R.min.x, R.min.y,
 * R.max.x, R.max.y, L.min.z, L.max.z, R.min.z, R.max.z, id_L, id_R, c, 0}; ids: internal k,
 * or 0x80000000|j for sorted leaf j.  A leaf child c holds {its box as L and as R,
 * 0x80000000|c, ~0u, 0x80000000|c, 0}.  (The root's record follows at slot 2(n-1).)  Only the
 * packet primary walks read the leaf children's records: a build for other walks (binned, AUTO)
 * leaves them out, and the first packet walk or this call writes them. */
rtbvh_status rtbvh_read_wide(rtbvh_ctx* ctx, uint32_t* records, uint64_t capacity);
/* Quantized 4-wide nodes of the bounce walk, one 64-B record (16 words) per slot (2n-1):
 * internal node k's at the slot of its record (2 * parent + side; the root's at 2n-2;
 * slots of leaves unused): words 0-2 grid origin xyz, 3-5 grid step xyz (f32; step x ==
 * 0: not quantized), 6-8 lo bytes x/y/z, 9-11 hi bytes x/y/z (byte c = grandchild c),
 * 12-15 grandchildren (slot, 0x80000000 | leaf, or 0xFFFFFFFF); decoded corner = origin +
 * q * step.  The low 16 bits of words 4 and 5 carry the certified walk's margin codes (the
 * largest edge bound of the node's leaves and its margin range, as the high half of an f32):
 * mask them off (& 0xFF800000) to read the steps.  Only the QNodes the walk reads are
 * written -- the root's and, recursively, those of the internal grandchildren listed in words
 * 12-15 (a build of more than 2048 triangles leaves the others untouched); capacity in records
 * (>= 2n-1). */
rtbvh_status rtbvh_read_qnodes(rtbvh_ctx* ctx, uint32_t* nodes, uint64_t capacity);
/* Per-triangle Morton codes in triangle order (MortonCodes.hlsl:104-112). */
rtbvh_status rtbvh_read_morton(rtbvh_ctx* ctx, uint32_t* codes);
/* Stable radix order: sorted codes and the triangle id of each sorted position. */
rtbvh_status rtbvh_read_sorted(rtbvh_ctx* ctx, uint32_t* sorted_codes, uint32_t* tri_ids);
/* reflectRay (after the last pass) and refractRay records of the last trace, one per traced
 * pixel in framebuffer order; needs RTBVH_FLAG_REFRACT_RECORDS at trace time.  Ray fields
 * HLSL leaves unset (a hit whose intensity is 0) are 0.  Either pointer may be NULL. */
rtbvh_status rtbvh_read_rays(rtbvh_ctx* ctx, rtbvh_ray_present* reflect_out, rtbvh_ray_present* refract_out);
rtbvh_status rtbvh_get_stats(rtbvh_ctx* ctx, rtbvh_stats* out);
/* Restart the timing averages of rtbvh_get_stats. */
rtbvh_status rtbvh_reset_stats(rtbvh_ctx* ctx);
/* Replace the RTBVH_FLAG_* bits of the context (takes effect for the next build/trace). */
rtbvh_status rtbvh_set_flags(rtbvh_ctx* ctx, uint32_t flags);

/* ---- primitives (exposed for tests and callers with their own buffers) ---- */
/* Stable LSD radix sort of (key, value) pairs, 8-bit digits over bits [0, key_bits).
 * Device pointers; keys/vals_in may be overwritten (ping-pong); the sorted
 * result lands in keys_out/vals_out.  Enqueued on the context stream. */
rtbvh_status rtbvh_sort_pairs_async(rtbvh_ctx* ctx, uint32_t* keys_in, uint32_t* vals_in,
                                    uint32_t* keys_out, uint32_t* vals_out, uint32_t n,
                                    uint32_t key_bits);
/* Host-memory convenience wrapper of the above (synchronous). */
rtbvh_status rtbvh_sort_pairs_host(rtbvh_ctx* ctx, const uint32_t* keys, const uint32_t* vals,
                                   uint32_t* keys_out, uint32_t* vals_out, uint32_t n, uint32_t key_bits);
/* Karras + refit on caller-given sorted codes and leaf boxes (host arrays; leaf
 * boxes n x 6 floats {min xyz, max xyz}); writes 2n-1 nodes (reference layout).
 * Lets the build kernels be checked on the reference's own RadixBVHCombo data. */
rtbvh_status rtbvh_build_from_codes(rtbvh_ctx* ctx, const uint32_t* sorted_codes,
                                    const float* leaf_boxes, uint32_t n, rtbvh_node* out);

/* ---- host-side scene helpers (ObjLoader replacement, camera) ---------------- */
/* Decode an uncompressed BMP (BI_RGB 1/4/8-bit paletted or 24/32-bit, BI_BITFIELDS 32-bit) into RGBA8 rows in
 * file order (bottom row first for the usual positive height), as DevIL hands them to
 * Image.cpp:48-49.  Free with rtbvh_texture_free. */
rtbvh_status rtbvh_texture_load_bmp(const char* path, rtbvh_texture* out);
/* Decode a baseline (sequential DCT, Huffman, 8-bit, 1 or 3 components, sampling up to 2x2)
 * JPEG file / memory buffer into RGBA8 rows, top row first, as DevIL hands them to
 * Image.cpp:48-49 (Test.mtl:12 binds Balls.jpg).  The arithmetic of libjpeg's default
 * decompression (islow IDCT, fancy upsampling, fixed-point YCbCr -> RGB), restated: bit-exact
 * against libjpeg-turbo on the reference's files.  RTBVH_ERR_IO for other or malformed files.
 * Free with rtbvh_texture_free. */
rtbvh_status rtbvh_texture_load_jpeg(const char* path, rtbvh_texture* out);
rtbvh_status rtbvh_texture_decode_jpeg(const uint8_t* data, size_t size, rtbvh_texture* out);
/* BMP or JPEG by the file's magic bytes (ObjLoader's map_Kd files, Image::loadImage). */
rtbvh_status rtbvh_texture_load(const char* path, rtbvh_texture* out);
void rtbvh_texture_free(rtbvh_texture* tex);
/* The 256-entry sRGB -> linear table the texture sampling uses (IEC 61966-2-1, in double). */
void rtbvh_srgb_table(float out[256]);
typedef struct rtbvh_scene rtbvh_scene;
/* ObjLoader::Load (ObjectFileLoader.cpp:212-547) incl. its de-duplication rules. */
rtbvh_status rtbvh_scene_load_obj(const char* path, rtbvh_scene** out);
/* Synthetic random triangles: splitmix64(seed), centroids uniform
 * in [-half,+half], vertex offsets (u-0.5)*1.0, face normals, one material. */
rtbvh_status rtbvh_scene_synthetic(uint64_t seed, uint32_t ntris, const float half_extent[3],
                                   rtbvh_scene** out);
void rtbvh_scene_free(rtbvh_scene* s);
uint32_t rtbvh_scene_num_vertices(const rtbvh_scene* s);
uint32_t rtbvh_scene_num_indices(const rtbvh_scene* s);
uint32_t rtbvh_scene_num_materials(const rtbvh_scene* s);
uint32_t rtbvh_scene_num_textures(const rtbvh_scene* s);
const rtbvh_vertex* rtbvh_scene_vertices(const rtbvh_scene* s);
const uint32_t* rtbvh_scene_indices(const rtbvh_scene* s);
const uint32_t* rtbvh_scene_mat_indices(const rtbvh_scene* s);
const rtbvh_material* rtbvh_scene_materials(const rtbvh_scene* s);
/* texture path of texture k (as named by map_Kd), or NULL */
const char* rtbvh_scene_texture_path(const rtbvh_scene* s, uint32_t k);
/* Upload a loaded scene (set_scene with the scene's arrays; textures as given). */
rtbvh_status rtbvh_set_scene_obj(rtbvh_ctx* ctx, const rtbvh_scene* s, const rtbvh_texture* textures,
                                 uint32_t ntex);
/* Graphics::onUpdate's camera (Graphics.cpp:44-53, Graphics.h:200-204):
 * LookAtLH(eye (0,5,-100), at 0, up +y) * PerspectiveFovLH(pi/4, H/W, 0.1, 1000). */
void rtbvh_camera_reference(uint32_t width, uint32_t height, float wvp[16], float wv[16]);
/* The same camera from any eye (at 0, up +y): Graphics::onUpdate after the eye has moved. */
void rtbvh_camera_look(const float eye[3], uint32_t width, uint32_t height, float wvp[16], float wv[16]);
/* Graphics::onKeyDown (Graphics.cpp:937-960): the eye rotated about `at` = 0 by CAM_DELTA = 0.1 rad
 * (Graphics.h:14): key 0 VK_LEFT (RotationY(-0.1)), 1 VK_RIGHT (RotationY(0.1)), 2 VK_UP (RotationX(0.1)),
 * 3 VK_DOWN (RotationX(-0.1)); the vector times the rotation matrix, row-vector convention (XMVector4Transform).
 * Other keys leave the eye unchanged.  (DirectXMath's own sin/cos approximation is not restated: libm's.) */
void rtbvh_camera_orbit(float eye[3], uint32_t key);

#ifdef __cplusplus
}
#endif
#endif /* RTBVH_H */
