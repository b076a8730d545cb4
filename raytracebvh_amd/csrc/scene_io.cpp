// scene_io.cpp -- host-side scene inputs of the path: the OBJ/MTL loader that
// replaces ObjLoader (ObjectFileLoader.cpp:77-468), the synthetic scene
// generator of SURVEY §8(d), and the camera of Graphics::onUpdate
// (Graphics.cpp:44-53).  Plain C++17; exported through include/rtbvh.h.
#include "../../include/rtbvh.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

struct rtbvh_scene {
    std::vector<rtbvh_vertex> verts;
    std::vector<uint32_t> indices;
    std::vector<uint32_t> mat_indices;
    std::vector<rtbvh_material> materials;
    std::vector<std::string> texture_paths;
};

namespace {

struct Pos {
    float x, y, z;
    bool operator==(const Pos& o) const { return x == o.x && y == o.y && z == o.z; }
};
struct PosHash {
    // std::hash<float> maps -0 and +0 to the same value; so does this
    size_t operator()(const Pos& p) const {
        auto h = [](float f) -> size_t {
            if (f == 0.0f) return 0;
            uint32_t u;
            memcpy(&u, &f, 4);
            return (size_t)u * 0x9E3779B97F4A7C15ull;
        };
        return h(p.x) ^ (h(p.y) << 1) ^ (h(p.z) << 2);
    }
};
struct VData { float n[3]; float t[2]; uint32_t index; };

// sscanf(s, "%f %f ...", ...): stops at the first failed conversion
int scan_floats(const char* s, float* out, int count) {
    int got = 0;
    for (; got < count; got++) {
        char* end = nullptr;
        float v = strtof(s, &end);
        if (end == s) break;
        out[got] = v;
        s = end;
    }
    return got;
}

// sscanf(s, "%i/%i/%i %i/%i/%i %i/%i/%i ", ...)
void scan_face(const char* s, int v[3], int t[3], int n[3]) {
    int vals[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 9; k++) {
        if (k % 3 != 0) {
            if (*s == '/') s++;
            else break;
        }
        char* end = nullptr;
        long x = strtol(s, &end, 0);
        if (end == s) break;
        vals[k] = (int)x;
        s = end;
    }
    for (int c = 0; c < 3; c++) { v[c] = vals[3 * c]; t[c] = vals[3 * c + 1]; n[c] = vals[3 * c + 2]; }
}

bool read_lines(const std::string& path, std::vector<std::string>& lines) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return false;
    std::string line;
    while (std::getline(f, line)) lines.push_back(line);
    return true;
}

void base_material(rtbvh_material& m) {   // Base_Mat, ObjectFileLoader.cpp:64-74
    const float a[4] = {0.2f, 0.2f, 0.2f, 1.f}, d[4] = {0.8f, 0.8f, 0.8f, 1.f}, s[4] = {1.f, 1.f, 1.f, 1.f};
    memcpy(m.ambient, a, 16);
    memcpy(m.diffuse, d, 16);
    memcpy(m.specular, s, 16);
    m.shininess = 0;
    m.optical_density = 0;
    m.alpha = 1.0f;
    m.specularb = 0;
    m.tex_num = -1;
}

// Material_File, ObjectFileLoader.cpp:77-210
void material_file(const std::string& obj_path, const std::string& matfile, std::vector<rtbvh_material>& mats,
                   std::vector<std::string>& names, std::vector<std::string>& tex_paths) {
    std::string directory = obj_path.substr(0, obj_path.find_last_of('/') + 1);
    std::vector<std::string> lines;
    if (!read_lines(directory + matfile, lines)) return;   // reference prints and continues
    for (const std::string& line : lines) {
        const char* p = line.c_str();
        if (p[0] == '\t') p++;
        size_t len = strlen(p);
        if (len >= 6 && !strncmp(p, "newmtl", 6)) {
            rtbvh_material m;
            base_material(m);
            mats.push_back(m);
            names.push_back(len > 7 ? std::string(p + 7) : std::string());
            tex_paths.push_back(std::string());
        } else if (mats.empty()) {
            continue;
        } else if (p[0] == 'K' && p[1] == 'a') {
            scan_floats(p + 2, mats.back().ambient, 3);
            mats.back().ambient[3] = 1.f;
        } else if (p[0] == 'K' && p[1] == 'd') {
            scan_floats(p + 2, mats.back().diffuse, 3);
            mats.back().diffuse[3] = 1.f;
        } else if (p[0] == 'K' && p[1] == 's') {
            scan_floats(p + 2, mats.back().specular, 3);
            mats.back().specular[3] = 1.f;
        } else if (p[0] == 'N' && p[1] == 's') {
            scan_floats(p + 2, &mats.back().shininess, 1);
        } else if (p[0] == 'N' && p[1] == 'i') {
            scan_floats(p + 2, &mats.back().optical_density, 1);
        } else if (p[0] == 'd') {
            scan_floats(p + 1, &mats.back().alpha, 1);
        } else if (len >= 6 && !strncmp(p, "map_Kd", 6)) {
            tex_paths.back() = directory + (len > 7 ? std::string(p + 7) : std::string());
        }
        // `Tr` is never parsed by the reference (:177 tests ptr[0] == 'T' && ptr[0] == 'r')
    }
}

}  // namespace

extern "C" {

// ObjLoader::Load_Geometry, ObjectFileLoader.cpp:212-468
rtbvh_status rtbvh_scene_load_obj(const char* path, rtbvh_scene** out) {
    if (!path || !out) return RTBVH_ERR_INVALID_ARG;
    *out = nullptr;
    try {
        std::vector<std::string> lines;
        if (!read_lines(path, lines)) return RTBVH_ERR_IO;
        std::unique_ptr<rtbvh_scene> s(new rtbvh_scene());
        std::vector<float> vx, vn, vt;
        std::vector<std::string> names;
        std::unordered_map<Pos, std::vector<VData>, PosHash> vmap;
        std::vector<Pos> first_pos;   // position key of each output vertex
        uint32_t material_num = 0;
        for (const std::string& line : lines) {
            const char* p = line.c_str();
            if (!strncmp(p, "mtllib ", 7)) material_file(path, std::string(p + 7), s->materials, names, s->texture_paths);
            if (p[0] == 'v' && p[1] == ' ') {
                float t[3] = {0, 0, 0};
                scan_floats(p + 2, t, 3);
                vx.insert(vx.end(), t, t + 3);
            } else if (p[0] == 'v' && p[1] == 'n') {
                float t[3] = {0, 0, 0};
                scan_floats(p + 2, t, 3);
                vn.insert(vn.end(), t, t + 3);
            } else if (p[0] == 'v' && p[1] == 't') {
                float t[2] = {0, 0};
                scan_floats(p + 2, t, 2);
                vt.insert(vt.end(), t, t + 2);
            } else if (!strncmp(p, "usemtl", 6)) {
                std::string name = line.size() > 7 ? line.substr(7) : std::string();
                for (size_t k = 0; k < names.size(); k++)
                    if (name == names[k]) material_num = (uint32_t)k;
            } else if (p[0] == 'f') {
                int vi[3], ti[3], ni[3];
                scan_face(p + 1, vi, ti, ni);
                for (int c = 0; c < 3; c++) {
                    // the reference indexes vx/vn/vt unchecked (UB when out of range): reject instead
                    if (vi[c] < 1 || (size_t)vi[c] * 3 > vx.size() || ni[c] < 1 || (size_t)ni[c] * 3 > vn.size() ||
                        ti[c] < 1 || (size_t)ti[c] * 2 > vt.size())
                        return RTBVH_ERR_IO;
                    Pos pos{vx[3 * (vi[c] - 1)], vx[3 * (vi[c] - 1) + 1], vx[3 * (vi[c] - 1) + 2]};
                    VData vd;
                    memcpy(vd.n, &vn[3 * (ni[c] - 1)], 12);
                    memcpy(vd.t, &vt[2 * (ti[c] - 1)], 8);
                    uint32_t index = 0;
                    bool found = false;
                    auto it = vmap.find(pos);
                    if (it != vmap.end()) {
                        for (const VData& d : it->second) {
                            // Helper.h:11-14: XMFLOAT3 == compares a.z with itself -> z ignored
                            if (vd.n[0] == d.n[0] && vd.n[1] == d.n[1] && vd.t[0] == d.t[0] && vd.t[1] == d.t[1]) {
                                index = d.index;
                                found = true;
                                break;
                            }
                        }
                    }
                    if (!found) {
                        index = (uint32_t)s->verts.size();
                        vd.index = index;
                        Pos key = it != vmap.end() ? first_pos[it->second.front().index] : pos;
                        vmap[pos].push_back(vd);
                        rtbvh_vertex v;
                        v.position[0] = key.x; v.position[1] = key.y; v.position[2] = key.z;
                        memcpy(v.normal, vd.n, 12);
                        memcpy(v.texcoord, vd.t, 8);
                        s->verts.push_back(v);
                        first_pos.push_back(key);
                    }
                    s->indices.push_back(index);
                }
                s->mat_indices.push_back(material_num);
            }
        }
        // texNum per material: ObjectFileLoader.cpp:440-459
        int32_t ntex = 0;
        std::vector<std::string> tex;
        for (size_t k = 0; k < s->materials.size(); k++) {
            if (!s->texture_paths[k].empty()) {
                s->materials[k].tex_num = ntex++;
                tex.push_back(s->texture_paths[k]);
            } else {
                s->materials[k].tex_num = -1;
            }
        }
        s->texture_paths.swap(tex);
        if (s->materials.empty()) {   // no mtllib: the reference would index material 0 of an empty table
            rtbvh_material m;
            base_material(m);
            s->materials.push_back(m);
        }
        *out = s.release();
        return RTBVH_OK;
    } catch (const std::bad_alloc&) {
        return RTBVH_ERR_OOM;
    } catch (...) {
        return RTBVH_ERR_IO;
    }
}

static inline uint64_t splitmix64_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline float u01(uint64_t x) { return (float)(x >> 40) * (1.0f / 16777216.0f); }

// per triangle 12 draws (cx, cy, cz, then v0..v2 x,y,z offsets)
rtbvh_status rtbvh_scene_synthetic(uint64_t seed, uint32_t ntris, const float half[3], rtbvh_scene** out) {
    if (!out || !half || ntris == 0 || ntris > (1u << 30) / 3) return RTBVH_ERR_INVALID_ARG;
    *out = nullptr;
    try {
        std::unique_ptr<rtbvh_scene> s(new rtbvh_scene());
        s->verts.resize((size_t)ntris * 3);
        s->indices.resize((size_t)ntris * 3);
        s->mat_indices.assign(ntris, 0);
#pragma omp parallel for schedule(static)
        for (int64_t t = 0; t < (int64_t)ntris; t++) {
            uint64_t k = (uint64_t)t * 12;
            float c[3];
            for (int a = 0; a < 3; a++) c[a] = (u01(splitmix64_at(seed, k++)) * 2.0f - 1.0f) * half[a];
            float v[3][3];
            for (int i = 0; i < 3; i++)
                for (int a = 0; a < 3; a++) v[i][a] = c[a] + (u01(splitmix64_at(seed, k++)) - 0.5f) * 1.0f;
            float e1[3] = {v[1][0] - v[0][0], v[1][1] - v[0][1], v[1][2] - v[0][2]};
            float e2[3] = {v[2][0] - v[0][0], v[2][1] - v[0][1], v[2][2] - v[0][2]};
            float n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            float l2 = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
            if (l2 == 0.0f) { n[0] = 0; n[1] = 0; n[2] = 1; }
            else { float inv = 1.0f / sqrtf(l2); n[0] *= inv; n[1] *= inv; n[2] *= inv; }
            for (int i = 0; i < 3; i++) {
                rtbvh_vertex& vx = s->verts[3 * (size_t)t + i];
                memcpy(vx.position, v[i], 12);
                memcpy(vx.normal, n, 12);
                vx.texcoord[0] = 0;
                vx.texcoord[1] = 0;
                s->indices[3 * (size_t)t + i] = (uint32_t)(3 * (size_t)t + i);
            }
        }
        rtbvh_material m;
        const float ka[4] = {0, 0, 0, 1}, kd[4] = {0.64f, 0.64f, 0.64f, 1}, ks[4] = {0.5f, 0.5f, 0.5f, 1};
        memcpy(m.ambient, ka, 16);
        memcpy(m.diffuse, kd, 16);
        memcpy(m.specular, ks, 16);
        m.shininess = 300.0f;
        m.optical_density = 1.0f;
        m.alpha = 1.0f;
        m.specularb = 0;
        m.tex_num = -1;
        s->materials.push_back(m);
        *out = s.release();
        return RTBVH_OK;
    } catch (const std::bad_alloc&) {
        return RTBVH_ERR_OOM;
    }
}

void rtbvh_scene_free(rtbvh_scene* s) { delete s; }
uint32_t rtbvh_scene_num_vertices(const rtbvh_scene* s) { return s ? (uint32_t)s->verts.size() : 0; }
uint32_t rtbvh_scene_num_indices(const rtbvh_scene* s) { return s ? (uint32_t)s->indices.size() : 0; }
uint32_t rtbvh_scene_num_materials(const rtbvh_scene* s) { return s ? (uint32_t)s->materials.size() : 0; }
uint32_t rtbvh_scene_num_textures(const rtbvh_scene* s) { return s ? (uint32_t)s->texture_paths.size() : 0; }
const rtbvh_vertex* rtbvh_scene_vertices(const rtbvh_scene* s) { return s ? s->verts.data() : nullptr; }
const uint32_t* rtbvh_scene_indices(const rtbvh_scene* s) { return s ? s->indices.data() : nullptr; }
const uint32_t* rtbvh_scene_mat_indices(const rtbvh_scene* s) { return s ? s->mat_indices.data() : nullptr; }
const rtbvh_material* rtbvh_scene_materials(const rtbvh_scene* s) { return s ? s->materials.data() : nullptr; }
const char* rtbvh_scene_texture_path(const rtbvh_scene* s, uint32_t k) {
    return (s && k < s->texture_paths.size()) ? s->texture_paths[k].c_str() : nullptr;
}

rtbvh_status rtbvh_set_scene_obj(rtbvh_ctx* ctx, const rtbvh_scene* s, const rtbvh_texture* textures, uint32_t ntex) {
    if (!s) return RTBVH_ERR_INVALID_ARG;
    return rtbvh_set_scene(ctx, s->verts.data(), (uint32_t)s->verts.size(), s->indices.data(),
                           (uint32_t)s->indices.size(), s->mat_indices.data(), s->materials.data(),
                           (uint32_t)s->materials.size(), textures, ntex);
}

// Graphics.cpp:44-53: XMMatrixLookAtLH(eye, at, up) * XMMatrixPerspectiveFovLH(pi/4, H/W, .1, 1000)
void rtbvh_camera_reference(uint32_t W, uint32_t H, float wvp[16], float wv[16]) {
    const float eye[3] = {0.0f, 5.0f, -100.0f};   // Graphics.h:200-205
    rtbvh_camera_look(eye, W, H, wvp, wv);
}

// Graphics::onKeyDown (Graphics.cpp:937-960): eye = at + XMVector4Transform(eye - at, R), at = 0, with
// R = XMMatrixRotationY(-+CAM_DELTA) (left / right) or XMMatrixRotationX(+-CAM_DELTA) (up / down), CAM_DELTA
// = .1f (Graphics.h:14).  DirectXMath's rotations (row vectors, v' = v R): RotationY(a) = {c 0 -s; 0 1 0;
// s 0 c}, RotationX(a) = {1 0 0; 0 c s; 0 -s c}.
void rtbvh_camera_orbit(float eye[3], uint32_t key) {
    if (key > 3) return;
    const float a = key == 0 || key == 3 ? -0.1f : 0.1f;
    const float s = sinf(a), c = cosf(a);
    const float x = eye[0], y = eye[1], z = eye[2];
    if (key < 2) {   // about y
        eye[0] = x * c + z * s;
        eye[2] = x * -s + z * c;
    } else {         // about x
        eye[1] = y * c + z * -s;
        eye[2] = y * s + z * c;
    }
}

void rtbvh_camera_look(const float eye_in[3], uint32_t W, uint32_t H, float wvp[16], float wv[16]) {
    const float eye[3] = {eye_in[0], eye_in[1], eye_in[2]}, at[3] = {0, 0, 0}, up[3] = {0, 1.f, 0};
    auto dot3 = [](const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    auto cross3 = [](const float* a, const float* b, float* r) {
        r[0] = a[1] * b[2] - a[2] * b[1];
        r[1] = a[2] * b[0] - a[0] * b[2];
        r[2] = a[0] * b[1] - a[1] * b[0];
    };
    float dir[3] = {at[0] - eye[0], at[1] - eye[1], at[2] - eye[2]};
    float r2[3], r0[3], r1[3], cx[3];
    float inv = 1.0f / sqrtf(dot3(dir, dir));
    for (int a = 0; a < 3; a++) r2[a] = dir[a] * inv;
    cross3(up, r2, cx);
    inv = 1.0f / sqrtf(dot3(cx, cx));
    for (int a = 0; a < 3; a++) r0[a] = cx[a] * inv;
    cross3(r2, r0, r1);
    float ne[3] = {-eye[0], -eye[1], -eye[2]};
    float view[16] = {r0[0], r1[0], r2[0], 0, r0[1], r1[1], r2[1], 0, r0[2], r1[2], r2[2], 0,
                      dot3(r0, ne), dot3(r1, ne), dot3(r2, ne), 1};
    float fov = 3.14159265358979323846f / 4, aspect = (float)H / (float)W, zn = 0.1f, zf = 1000.0f;
    float sn = sinf(0.5f * fov), cs = cosf(0.5f * fov);
    float hgt = cs / sn, wdt = hgt / aspect, range = zf / (zf - zn);
    float proj[16] = {wdt, 0, 0, 0, 0, hgt, 0, 0, 0, 0, range, 1, 0, 0, -range * zn, 0};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            wvp[4 * i + j] = ((view[4 * i] * proj[j] + view[4 * i + 1] * proj[4 + j]) + view[4 * i + 2] * proj[8 + j]) +
                             view[4 * i + 3] * proj[12 + j];
    memcpy(wv, view, sizeof(view));
}

}  // extern "C"

// ---- textures ------------------------------------------------------------------
extern "C" {

void rtbvh_srgb_table(float out[256]) {
    for (int i = 0; i < 256; i++) {
        const double c = i / 255.0;
        out[i] = (float)(c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4));
    }
}

static uint32_t rd_u32(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }
static uint16_t rd_u16(const uint8_t* p) { return (uint16_t)(p[0] | p[1] << 8); }

rtbvh_status rtbvh_texture_load_bmp(const char* path, rtbvh_texture* out) {
    if (!path || !out) return RTBVH_ERR_INVALID_ARG;
    out->width = out->height = 0;
    out->rgba8 = nullptr;
    std::ifstream f(path, std::ios::binary);
    if (!f) return RTBVH_ERR_IO;
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() < 54 || b[0] != 'B' || b[1] != 'M') return RTBVH_ERR_IO;
    const uint32_t off = rd_u32(&b[10]), hsize = rd_u32(&b[14]);
    const int32_t w = (int32_t)rd_u32(&b[18]), h = (int32_t)rd_u32(&b[22]);
    const uint16_t bpp = rd_u16(&b[28]);
    const uint32_t comp = hsize >= 40 ? rd_u32(&b[30]) : 0;
    const bool paletted = bpp == 1 || bpp == 4 || bpp == 8;
    if (w <= 0 || h == 0 || !(paletted || bpp == 24 || bpp == 32) || !(comp == 0 || (comp == 3 && bpp == 32)))
        return RTBVH_ERR_IO;
    // palette (BGRA quads after the info header), 2^bpp or biClrUsed entries
    uint32_t npal = 0;
    const uint8_t* pal = nullptr;
    if (paletted) {
        const uint32_t used = hsize >= 36 ? rd_u32(&b[46]) : 0;
        npal = used ? used : (1u << bpp);
        if (npal > 256 || 14 + (size_t)hsize + 4 * npal > b.size()) return RTBVH_ERR_IO;
        pal = &b[14 + hsize];
    }
    const uint32_t W = (uint32_t)w, H = (uint32_t)(h < 0 ? -h : h);
    uint32_t mr = 0x00FF0000u, mg = 0x0000FF00u, mb = 0x000000FFu, ma = bpp == 32 ? 0xFF000000u : 0u;
    if (comp == 3 && b.size() >= 14 + 52) {
        mr = rd_u32(&b[54]); mg = rd_u32(&b[58]); mb = rd_u32(&b[62]);
        ma = hsize >= 56 ? rd_u32(&b[66]) : 0u;
    }
    const size_t stride = ((size_t)W * bpp / 8 + 3) & ~(size_t)3;
    if ((size_t)off + stride * H > b.size()) return RTBVH_ERR_IO;
    auto chan = [](uint32_t px, uint32_t m) -> uint8_t {
        if (!m) return 255;
        int sh = 0;
        while (!((m >> sh) & 1u)) sh++;
        const uint32_t v = (px & m) >> sh, mx = m >> sh;
        return (uint8_t)(mx == 255 ? v : (v * 255 + mx / 2) / mx);
    };
    uint8_t* px = (uint8_t*)std::malloc((size_t)W * H * 4);
    if (!px) return RTBVH_ERR_OOM;
    for (uint32_t r = 0; r < H; r++) {   // file order: row r of the pixel array
        const uint8_t* src = &b[off + stride * r];
        uint8_t* dst = px + (size_t)r * W * 4;
        for (uint32_t x = 0; x < W; x++) {
            if (paletted) {
                const uint32_t bit = x * bpp;
                uint32_t k = (src[bit >> 3] >> (8 - bpp - (bit & 7))) & ((1u << bpp) - 1u);
                if (k >= npal) k = 0;
                dst[4 * x + 0] = pal[4 * k + 2];
                dst[4 * x + 1] = pal[4 * k + 1];
                dst[4 * x + 2] = pal[4 * k + 0];
                dst[4 * x + 3] = 255;
            } else if (bpp == 24) {
                dst[4 * x + 0] = src[3 * x + 2];
                dst[4 * x + 1] = src[3 * x + 1];
                dst[4 * x + 2] = src[3 * x + 0];
                dst[4 * x + 3] = 255;
            } else {
                const uint32_t v = rd_u32(src + 4 * x);
                dst[4 * x + 0] = chan(v, mr);
                dst[4 * x + 1] = chan(v, mg);
                dst[4 * x + 2] = chan(v, mb);
                dst[4 * x + 3] = chan(v, ma);
            }
        }
    }
    out->width = W;
    out->height = H;
    out->rgba8 = px;
    return RTBVH_OK;
}

rtbvh_status rtbvh_save_bmp(const char* path, const uint8_t* rgba8, uint32_t W, uint32_t H) {
    if (!path || !rgba8 || W == 0 || H == 0 || W > 65535 || H > 65535) return RTBVH_ERR_INVALID_ARG;
    const uint32_t stride = (3 * W + 3) & ~3u, size = stride * H;
    uint8_t hdr[54] = {0};
    auto put32 = [&](int o, uint32_t v) { hdr[o] = v; hdr[o + 1] = v >> 8; hdr[o + 2] = v >> 16; hdr[o + 3] = v >> 24; };
    hdr[0] = 'B'; hdr[1] = 'M';                       // bfType 0x4d42
    put32(2, 54 + size);                              // bfSize
    put32(10, 0x36);                                  // bfOffBits
    put32(14, 40);                                    // biSize
    put32(18, W); put32(22, H);                       // positive height: bottom-up rows
    hdr[26] = 1; hdr[28] = 24;                        // planes, 24 bpp, BI_RGB
    put32(34, 0);                                     // biSizeImage 0
    put32(38, 0x0ec4); put32(42, 0x0ec4);             // pixels per metre (SaveBMP.cpp:26-27)
    std::ofstream f(path, std::ios::binary);
    if (!f) return RTBVH_ERR_IO;
    f.write((const char*)hdr, 54);
    std::vector<uint8_t> row(stride, 0);
    for (uint32_t r = 0; r < H; r++) {                // file row r = image row H-1-r
        const uint8_t* src = rgba8 + (size_t)(H - 1 - r) * W * 4;
        for (uint32_t x = 0; x < W; x++) {
            row[3 * x + 0] = src[4 * x + 2];
            row[3 * x + 1] = src[4 * x + 1];
            row[3 * x + 2] = src[4 * x + 0];
        }
        f.write((const char*)row.data(), stride);
    }
    return f ? RTBVH_OK : RTBVH_ERR_IO;
}

void rtbvh_texture_free(rtbvh_texture* tex) {
    if (!tex) return;
    std::free((void*)tex->rgba8);
    tex->rgba8 = nullptr;
    tex->width = tex->height = 0;
}

}  // extern "C"
