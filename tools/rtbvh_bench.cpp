// rtbvh_bench -- the C++ host over the C ABI (include/rtbvh.h) alone: what
// Graphics::onInit / onUpdate / computeBVH (Graphics.cpp:20-60, 667-831) become when the
// reference's host links librtbvh.so.  No Python, no torch.  SURVEY §8(b) "callers".
//
//   rtbvh_bench [--obj PATH | --synthetic NTRIS [--seed S] [--half X,Y,Z]]
//               [--width W] [--height H] [--bounces B] [--iters K] [--warmup W]
//               [--flags F] [--bmp OUT.bmp] [--comm-file PATH]
//
// One JSON line on stdout.  Multi-GPU: one process per GPU with RANK / WORLD_SIZE /
// LOCAL_RANK in the environment and --comm-file naming a path every rank can read; rank 0
// writes the RCCL id there, the frame is traced with rtbvh_trace_tiles and lands on rank 0.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "rtbvh.h"

namespace {

[[noreturn]] void die(const std::string& what, rtbvh_ctx* ctx = nullptr) {
    const char* e = rtbvh_last_error(ctx);
    std::fprintf(stderr, "rtbvh_bench: %s%s%s\n", what.c_str(), e && *e ? ": " : "", e ? e : "");
    std::exit(1);
}
void check(rtbvh_status st, const std::string& what, rtbvh_ctx* ctx = nullptr) {
    if (st != RTBVH_OK) die(what + " (status " + std::to_string(st) + ")", ctx);
}
uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = std::getenv(name);
    return v && *v ? (uint32_t)std::strtoul(v, nullptr, 10) : dflt;
}
double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

// rank 0 writes the 128-B RCCL id to path (via a rename, so readers never see half a file)
void share_comm_id(const std::string& path, uint32_t rank, uint8_t id[RTBVH_COMM_ID_BYTES]) {
    if (rank == 0) {
        check(rtbvh_comm_unique_id(id), "rtbvh_comm_unique_id");
        const std::string tmp = path + ".tmp";
        std::ofstream(tmp, std::ios::binary).write((const char*)id, RTBVH_COMM_ID_BYTES);
        if (std::rename(tmp.c_str(), path.c_str()) != 0) die("cannot write " + path);
        return;
    }
    for (int tries = 0; tries < 1200; tries++) {   // up to 60 s
        std::ifstream f(path, std::ios::binary);
        if (f && f.read((char*)id, RTBVH_COMM_ID_BYTES) && f.gcount() == RTBVH_COMM_ID_BYTES) return;
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    die("no RCCL id in " + path + " after 60 s");
}

}  // namespace

int main(int argc, char** argv) {
    std::string obj, bmp, comm_file;
    uint32_t ntris = 0, W = 1920, H = 1080, bounces = 1, iters = 10, warmup = 2, flags = 0;
    uint64_t seed = 0x5EED0004ull;
    float half[3] = {50.f, 50.f, 50.f};
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) die("missing value for " + a);
            return argv[++i];
        };
        if (a == "--obj") obj = next();
        else if (a == "--synthetic") ntris = (uint32_t)std::stoul(next());
        else if (a == "--seed") seed = std::stoull(next(), nullptr, 0);
        else if (a == "--half") {
            const std::string v = next();
            if (std::sscanf(v.c_str(), "%f,%f,%f", &half[0], &half[1], &half[2]) != 3) die("--half X,Y,Z");
        } else if (a == "--width") W = (uint32_t)std::stoul(next());
        else if (a == "--height") H = (uint32_t)std::stoul(next());
        else if (a == "--bounces") bounces = (uint32_t)std::stoul(next());
        else if (a == "--iters") iters = (uint32_t)std::stoul(next());
        else if (a == "--warmup") warmup = (uint32_t)std::stoul(next());
        else if (a == "--flags") flags = (uint32_t)std::stoul(next(), nullptr, 0);
        else if (a == "--bmp") bmp = next();
        else if (a == "--comm-file") comm_file = next();
        else die("unknown argument " + a + " (see the header of tools/rtbvh_bench.cpp)");
    }
    if (obj.empty() == (ntris == 0)) die("give exactly one of --obj PATH or --synthetic NTRIS");
    if (iters == 0) die("--iters must be positive");
    const uint32_t rank = env_u32("RANK", 0), nranks = env_u32("WORLD_SIZE", 1);
    if (nranks > 1 && comm_file.empty()) die("WORLD_SIZE > 1 needs --comm-file");

    // ObjLoader::Load (Graphics::onInit) or the SURVEY §8(d) generator
    rtbvh_scene* scene = nullptr;
    if (!obj.empty()) check(rtbvh_scene_load_obj(obj.c_str(), &scene), "load " + obj);
    else check(rtbvh_scene_synthetic(seed, ntris, half, &scene), "synthetic scene");
    // textures t4-t5 (Image::loadImage, Image.cpp:35-61): BMP and baseline JPEG decoded natively;
    // a file that cannot be decoded falls back to one white texel (as in the Python loader)
    std::vector<rtbvh_texture> tex(rtbvh_scene_num_textures(scene));
    std::vector<bool> owned(tex.size(), false);
    static const uint8_t white[4] = {255, 255, 255, 255};
    for (uint32_t k = 0; k < tex.size(); k++) {
        const char* name = rtbvh_scene_texture_path(scene, k);
        std::string path = name ? name : "";
        if (!path.empty() && path[0] != '/') {   // map_Kd names are relative to the .obj
            const size_t slash = obj.find_last_of('/');
            if (slash != std::string::npos) path = obj.substr(0, slash + 1) + path;
        }
        const char* p = name ? path.c_str() : nullptr;
        if (p && rtbvh_texture_load(p, &tex[k]) == RTBVH_OK) {
            owned[k] = true;
            continue;
        }
        std::fprintf(stderr, "rtbvh_bench: texture %u (%s) not decoded here: white\n", k, p ? p : "?");
        tex[k] = rtbvh_texture{1, 1, white};
    }

    rtbvh_config cfg;
    rtbvh_config_default(&cfg);
    cfg.device = (int32_t)env_u32("LOCAL_RANK", 0);
    cfg.flags = flags | RTBVH_FLAG_TIMING;
    rtbvh_ctx* ctx = nullptr;
    check(rtbvh_create(&cfg, &ctx), "rtbvh_create");
    check(rtbvh_set_scene_obj(ctx, scene, tex.data(), (uint32_t)tex.size()), "rtbvh_set_scene_obj", ctx);
    float wvp[16], wv[16];
    rtbvh_camera_reference(W, H, wvp, wv);   // Graphics::onUpdate's camera
    check(rtbvh_set_camera(ctx, wvp, wv), "rtbvh_set_camera", ctx);

    void* comm = nullptr;
    if (nranks > 1) {
        uint8_t id[RTBVH_COMM_ID_BYTES];
        share_comm_id(comm_file, rank, id);
        check(rtbvh_comm_init(ctx, nranks, rank, id, &comm), "rtbvh_comm_init", ctx);
    }

    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); };
    std::vector<double> build_ms, trace_ms;
    for (uint32_t it = 0; it < warmup + iters; it++) {
        auto t0 = clk::now();
        check(rtbvh_build(ctx), "rtbvh_build", ctx);
        const double b = ms_since(t0);
        t0 = clk::now();
        if (comm) check(rtbvh_trace_tiles(ctx, W, H, bounces, rank, nranks, comm), "rtbvh_trace_tiles", ctx);
        else check(rtbvh_trace(ctx, W, H, bounces), "rtbvh_trace", ctx);
        const double t = ms_since(t0);
        if (it >= warmup) {
            build_ms.push_back(b);
            trace_ms.push_back(t);
        }
    }
    rtbvh_stats st;
    check(rtbvh_get_stats(ctx, &st), "rtbvh_get_stats", ctx);
    if (!bmp.empty() && rank == 0) {   // Graphics::onRender's presentation + SaveBMP
        std::vector<uint8_t> img((size_t)W * H * 4);
        check(rtbvh_present(ctx, img.data()), "rtbvh_present", ctx);
        check(rtbvh_save_bmp(bmp.c_str(), img.data(), W, H), "rtbvh_save_bmp", ctx);
    }
    const double rays = (double)st.primary_rays + (double)st.bounce_rays;   // this rank's rays
    const double tmed = median(trace_ms);
    std::printf("{\"tool\": \"rtbvh_bench\", \"scene\": \"%s\", \"tris\": %u, \"width\": %u, \"height\": %u, "
                "\"bounces\": %u, \"rank\": %u, \"nranks\": %u, \"iters\": %u, \"build_ms_median\": %.4f, "
                "\"trace_ms_median\": %.4f, \"rays_this_rank\": %.0f, \"mrays_s_this_rank\": %.2f, "
                "\"gpu_ms_build\": %.4f, \"gpu_ms_trace\": %.4f}\n",
                obj.empty() ? "synthetic" : obj.c_str(), st.num_tris, W, H, bounces, rank, nranks, iters,
                median(build_ms), tmed, rays, tmed > 0 ? rays / (tmed * 1e3) : 0.0, st.ms_build, st.ms_trace);
    if (comm) check(rtbvh_comm_destroy(comm), "rtbvh_comm_destroy");
    rtbvh_destroy(ctx);
    for (uint32_t k = 0; k < tex.size(); k++)
        if (owned[k]) rtbvh_texture_free(&tex[k]);
    rtbvh_scene_free(scene);
    return 0;
}
