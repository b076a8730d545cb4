/*
 * rtbvh_oracle.h -- CPU ORACLE for the LBVH build + ray traversal path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (raytracebvh_amd/, include/)
 * links, loads or calls this library; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg do, and only as the checker / the timed CPU
 * baseline.  It is a plain C++17 restatement of the reference algorithm, each
 * function citing the reference file:line it follows (paths relative to the
 * Fierykev/RayTraceBVH root).
 *
 * Parity pinning: the Morton / split-sort / Karras / refit pieces are checked
 * against fixtures produced by the reference's own CPUTests programs compiled
 * from /root/reference (oracle/Makefile target `ref`, outputs in oracle/_ref/,
 * fixtures committed in tests/golden/ by tests/golden/make_golden.py), and
 * against the ShaderSim known-answer values recorded in SURVEY.md §8(c).
 * The traversal / shading half restates the HLSL (which cannot run here: no
 * D3D12, no dxc) and is therefore pinned only by its own properties; see
 * DESIGN.md "Oracle".
 *
 * Floating point: built with -ffp-contract=off and no fast-math, so every
 * a*b+c is two IEEE roundings, in the written left-to-right order; min/max
 * are fminf/fmaxf (NaN-dropping, = HLSL min/max).
 */
#ifndef RTBVH_ORACLE_H
#define RTBVH_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same byte layouts as include/rtbvh.h (and as the reference's HLSL structs). */
typedef struct { float position[3]; float normal[3]; float texcoord[2]; } orc_vertex;      /* RayTraceGlobal.hlsl:53-58 */
typedef struct {
    float ambient[4], diffuse[4], specular[4];
    float shininess, optical_density, alpha;
    uint32_t specularb;
    int32_t tex_num;
} orc_material;                                                                           /* RayTraceGlobal.hlsl:60-72, ObjectFileLoader.h:79-96 */
typedef struct {
    uint32_t parent, child_l, child_r, code;
    float bb_min[3], bb_max[3];
    uint32_t index;
} orc_node;                                                                               /* RayTraceGlobal.hlsl:39-51 */
typedef struct { uint32_t width, height; const uint8_t* rgba8; } orc_texture;

typedef struct {
    const orc_vertex* verts; uint32_t num_verts;
    const uint32_t* indices; uint32_t num_indices;
    const uint32_t* mat_indices;                  /* one per triangle */
    const orc_material* materials; uint32_t num_materials;
    const orc_texture* textures; uint32_t num_textures;
} orc_scene;

enum { ORC_MORTON_CPUTESTS = 0, ORC_MORTON_HLSL = 1 };
enum { ORC_DELTA_CLZ64 = 0, ORC_DELTA_CPUTESTS = 1 };

/* ---- Morton -------------------------------------------------------------- */
uint32_t orc_expand_bits(uint32_t v);                               /* MortonCodes.hlsl:13-31 */
uint32_t orc_morton_point_cputests(float x, float y, float z);     /* Morton Code/main.cpp:75-98 */
uint32_t orc_morton_point_hlsl(float x, float y, float z);         /* MortonCodes.hlsl:33-52 */
/* per-triangle codes, triangle order.  CPUTests: ShaderSim/main.cpp:269-301 */
void orc_morton_tris_cputests(const orc_scene* s, uint32_t* codes);
/* HLSL: MortonCodes.hlsl:70-106 (clip-space, avg = bbMin/3 bug, fixed scene box) */
void orc_morton_tris_hlsl(const orc_scene* s, const float wvp[16], const float scene_min[3],
                          const float scene_max[3], uint32_t* codes);

/* ---- sort ------------------------------------------------------------------ */
/* Reference-faithful 32 x 1-bit split sort with 256-wide Blelloch group scans
 * (RadixBVHCombo/main.cpp:249-284,369-480 == RadixSortP1.hlsl + RadixSortP2.hlsl).
 * perm[i] = original position of the i-th element of the stable order. */
void orc_split_sort(const uint32_t* keys, uint32_t n, uint32_t* perm);
/* Same permutation by an 8-bit LSD counting sort (fast; for large inputs). */
void orc_lsd_sort(const uint32_t* keys, uint32_t n, uint32_t* perm);
/* One Blelloch up/down sweep over 256 entries (RadixBVHCombo/main.cpp:249-284). */
void orc_blelloch_scan256(uint32_t* data);

/* ---- Karras + refit -------------------------------------------------------- */
int32_t orc_delta(int mode, const uint32_t* codes, uint32_t n, uint32_t i, int64_t j);
/* node arrays have 2n-1 entries: leaves [0,n), internal node k at n+k, root n.
 * parent[root] = 0xFFFFFFFF, child_* of leaves = 0xFFFFFFFF. */
void orc_karras(int mode, const uint32_t* sorted_codes, uint32_t n,
                uint32_t* parent, uint32_t* child_l, uint32_t* child_r);   /* BVHConstructP1.hlsl:99-188 */
/* bb arrays: 2n-1 x 3 floats; leaves filled by caller.  Returns the longest climb
 * (loop trips of the arriving thread, RadixBVHCombo/main.cpp:535-576). */
uint32_t orc_refit(uint32_t n, const uint32_t* parent, const uint32_t* child_l,
                   const uint32_t* child_r, float* bb_min, float* bb_max);  /* BVHConstructP2.hlsl:8-37 */

/* ---- full build ------------------------------------------------------------ */
/* MortonCodes -> sort -> Karras -> refit (Graphics.cpp:705-782), no padding:
 * n = number of triangles.  out has 2n-1 nodes in the reference layout.
 * sort_mode 0 = faithful split sort, 1 = LSD (same permutation). */
int orc_build(const orc_scene* s, const float wvp[16], int morton_mode, int delta_mode,
              const float scene_min[3], const float scene_max[3], int sort_mode,
              orc_node* out);

/* ---- trace ----------------------------------------------------------------- */
/* Primary (RayTraceLaunch.hlsl) + `bounces` x RayTraceReflection.hlsl over the
 * rows [row_begin, row_end) of a W x H frame (row_step 1 = every row).
 * rgba: (rows) x W x 4 floats in row order of the traced rows; intensity may be NULL.
 * counters (may be NULL), 8 x u64: primary rays, bounce rays traced, internal
 * visits, leaf visits, hits, textured hits, stack-overflows, max stack depth. */
int orc_trace(const orc_scene* s, const orc_node* nodes, uint32_t n,
              const float wvp[16], const float wv[16], uint32_t W, uint32_t H,
              uint32_t bounces, uint32_t row_begin, uint32_t row_end, uint32_t row_step,
              float* rgba, float* intensity, uint64_t* counters);
/* orc_trace plus the per-pixel RayPresent records (RayTraceGlobal.hlsl:30-35; 14 floats:
 * intensity, origin, direction, invDirection, color): reflectRay after the last pass
 * (RayTraceLaunch.hlsl:48-67, RayTraceReflection.hlsl:24-55) and refractRay
 * (RayTraceLaunch.hlsl:70-80).  Ray fields HLSL leaves unset (zero intensity at the
 * hit) are written as 0.  Either record pointer may be NULL. */
int orc_trace_ex(const orc_scene* s, const orc_node* nodes, uint32_t n,
                 const float wvp[16], const float wv[16], uint32_t W, uint32_t H,
                 uint32_t bounces, uint32_t row_begin, uint32_t row_end, uint32_t row_step,
                 float* rgba, float* intensity, uint64_t* counters, float* refl_rec, float* refr_rec);

/* diffuseTex.SampleLevel(linear, wrap, uv, 0) on an sRGB RGBA8 texture, as restated for
 * RayTraceRender.hlsl:22-26 (include/rtbvh.h rtbvh_texture). */
void orc_sample_texture(const orc_texture* t, float u, float v, float out[4]);

/* ---- misc ------------------------------------------------------------------ */
/* XMMatrixLookAtLH * XMMatrixPerspectiveFovLH as Graphics.cpp:44-53 (row-vector
 * convention, float32, libm sinf/cosf).  wvp and wv row-major 4x4. */
void orc_camera_reference(uint32_t W, uint32_t H, float wvp[16], float wv[16]);
uint64_t orc_fnv1a64(const void* data, uint64_t nbytes);
int orc_num_threads(void);
/* threads orc_trace / orc_trace_ex use over rows (default 1; results are identical) */
void orc_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
