// tools/sanitize_host.cpp -- the host-side code of librtbvh (the OBJ/MTL loader, the BMP and
// JPEG decoders, the synthetic generator, the camera) and the CPU oracle, built with
// -fsanitize=address,undefined (tools/Makefile `sanitize`; SURVEY §5 asks for ASan/UBSan on
// the CPU side).  scene_io.cpp parses untrusted files in the product path, so besides the
// given files the driver feeds it truncated and bit-flipped copies of each (a deterministic
// mutation fuzzer), then runs the oracle's build and trace on the parsed scenes.
//   sanitize_host [--mutations N] FILE...   (.obj, .bmp, .jpg / .jpeg)
// Exit status 0 when every run finished; a sanitizer report aborts with a non-zero status.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include <unistd.h>

#include "../include/rtbvh.h"
#include "../oracle/rtbvh_oracle.h"

// scene_io.cpp's rtbvh_set_scene_obj forwards to the device API (api.hip), which is not part
// of this host-only build
extern "C" rtbvh_status rtbvh_set_scene(rtbvh_ctx*, const rtbvh_vertex*, uint32_t, const uint32_t*, uint32_t,
                                        const uint32_t*, const rtbvh_material*, uint32_t, const rtbvh_texture*,
                                        uint32_t) {
    return RTBVH_ERR_NO_DEVICE;
}

namespace {

uint64_t g_rng = 0x5A17123456789ULL;
uint64_t next_rand() {   // splitmix64
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

bool ends_with(const std::string& s, const char* suf) {
    const size_t n = strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

std::vector<uint8_t> read_all(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

void write_all(const std::string& path, const std::vector<uint8_t>& b) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(b.data()), (std::streamsize)b.size());
}

// oracle build + a small trace of a parsed scene (bounded so a fuzzed scene stays cheap)
void oracle_run(const rtbvh_scene* s) {
    const uint32_t nidx = rtbvh_scene_num_indices(s), nv = rtbvh_scene_num_vertices(s);
    const uint32_t nm = rtbvh_scene_num_materials(s);
    if (nidx < 3 || nidx > 3 * 200000 || nv == 0 || nm == 0) return;
    const uint32_t* idx = rtbvh_scene_indices(s);
    for (uint32_t i = 0; i < nidx; i++)
        if (idx[i] >= nv) return;
    const uint32_t* mi = rtbvh_scene_mat_indices(s);
    for (uint32_t t = 0; t < nidx / 3; t++)
        if (mi[t] >= nm) return;
    orc_scene os{};
    os.verts = reinterpret_cast<const orc_vertex*>(rtbvh_scene_vertices(s));
    os.num_verts = nv;
    os.indices = idx;
    os.num_indices = nidx;
    os.mat_indices = mi;
    os.materials = reinterpret_cast<const orc_material*>(rtbvh_scene_materials(s));
    os.num_materials = nm;
    const uint32_t n = nidx / 3, W = 64, H = 48;
    float wvp[16], wv[16];
    orc_camera_reference(W, H, wvp, wv);
    const float smin[3] = {-700, -700, -700}, smax[3] = {700, 700, 700};
    std::vector<orc_node> nodes(2 * (size_t)n - 1);
    if (orc_build(&os, wvp, 0, 0, smin, smax, 1, nodes.data()) != 0) return;
    std::vector<float> rgba((size_t)W * H * 4);
    uint64_t counters[8];
    (void)orc_trace(&os, nodes.data(), n, wvp, wv, W, H, 2, 0, H, 1, rgba.data(), nullptr, counters);
}

int run_file(const std::string& path) {
    if (ends_with(path, ".obj")) {
        rtbvh_scene* s = nullptr;
        if (rtbvh_scene_load_obj(path.c_str(), &s) == RTBVH_OK) {
            oracle_run(s);
            rtbvh_scene_free(s);
            return 1;
        }
        return 0;
    }
    rtbvh_texture t{};
    const rtbvh_status st = rtbvh_texture_load(path.c_str(), &t);
    if (st == RTBVH_OK) {
        volatile uint32_t sum = 0;
        for (size_t i = 0; i < (size_t)t.width * t.height * 4; i++) sum += t.rgba8[i];
        rtbvh_texture_free(&t);
        return 1;
    }
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    int mutations = 200;
    std::vector<std::string> files;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--mutations") && i + 1 < argc) mutations = atoi(argv[++i]);
        else files.push_back(argv[i]);
    }
    // the synthetic generator and the camera
    rtbvh_scene* syn = nullptr;
    const float half[3] = {30, 30, 20};
    if (rtbvh_scene_synthetic(7, 5000, half, &syn) != RTBVH_OK) return 2;
    oracle_run(syn);
    rtbvh_scene_free(syn);
    int ok = 0, total = 0;
    const std::string tmp = std::string(getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp") + "/rtbvh_sanitize_" +
                            std::to_string((long)getpid());
    for (const std::string& f : files) {
        total++;
        ok += run_file(f);
        const std::vector<uint8_t> orig = read_all(f);
        if (orig.empty()) continue;
        const std::string ext = f.substr(f.find_last_of('.'));
        const std::string mpath = tmp + ext;
        for (int m = 0; m < mutations; m++) {
            std::vector<uint8_t> b = orig;
            const uint64_t r = next_rand();
            switch (r % 4) {
                case 0: b.resize((size_t)(next_rand() % b.size())); break;   // truncation
                case 1:                                                      // bit flips
                    for (int k = 0; k < 1 + (int)(r >> 8) % 8; k++) b[next_rand() % b.size()] ^= (uint8_t)(1u << (next_rand() % 8));
                    break;
                case 2:                                                      // byte overwrite
                    for (int k = 0; k < 1 + (int)(r >> 8) % 4; k++) b[next_rand() % b.size()] = (uint8_t)next_rand();
                    break;
                default: {                                                   // header corruption
                    const size_t lim = b.size() < 64 ? b.size() : 64;
                    for (int k = 0; k < 4; k++) b[next_rand() % lim] = (uint8_t)next_rand();
                }
            }
            write_all(mpath, b);
            total++;
            ok += run_file(mpath);
        }
        std::remove(mpath.c_str());
    }
    std::printf("{\"runs\": %d, \"parsed\": %d}\n", total, ok);
    return 0;
}
