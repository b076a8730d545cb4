// Test-infrastructure driver for the reference's CPUTests/"Morton Code" program
// (compiled unmodified, -Dmain=morton_ref_main).  Evaluates the reference's two
// encoders (Karras expandBits/morton3D, main.cpp:33-54, and the repo's
// expand/calcMorton, main.cpp:56-98) on a fixed set of points and dumps
//   morton_points.f32  (M x 3)   morton_calc.u32 (M)   morton_karras.u32 (M)
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

unsigned int morton3D(float x, float y, float z);
unsigned int calcMorton(float x, float y, float z);
unsigned int expand(unsigned int var);
int morton_ref_main();

static void dump(const char* dir, const char* name, const void* p, size_t bytes) {
    char path[4096];
    snprintf(path, sizeof(path), "%s/%s", dir, name);
    FILE* f = fopen(path, "wb");
    if (!f) { perror(path); exit(1); }
    fwrite(p, 1, bytes, f);
    fclose(f);
}

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : ".";
    morton_ref_main();   // prints the KAT bit strings
    std::vector<float> pts;
    // the KAT point, corners, clamp edges
    const float special[][3] = {{.625f, .4375f, .75f}, {0, 0, 0}, {1, 1, 1}, {-0.5f, 2.f, 0.5f},
                                {0.99951171875f, 0.9990234375f, 1.0f / 1024}, {-0.0f, 1e-9f, 1023.5f / 1024}};
    for (auto& p : special) pts.insert(pts.end(), {p[0], p[1], p[2]});
    uint64_t s = 99;
    for (int i = 0; i < 20000; i++)
        for (int k = 0; k < 3; k++) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            float u = (float)((s >> 40) * (1.0 / 16777216.0));
            pts.push_back(u * 1.2f - 0.1f);
        }
    size_t M = pts.size() / 3;
    std::vector<unsigned> calc(M), karras(M), ex(1024);
    for (size_t i = 0; i < M; i++) {
        calc[i] = calcMorton(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
        karras[i] = morton3D(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    }
    for (unsigned v = 0; v < 1024; v++) ex[v] = expand(v);
    dump(dir, "morton_points.f32", pts.data(), pts.size() * 4);
    dump(dir, "morton_calc.u32", calc.data(), M * 4);
    dump(dir, "morton_karras.u32", karras.data(), M * 4);
    dump(dir, "morton_expand.u32", ex.data(), ex.size() * 4);
    return 0;
}
