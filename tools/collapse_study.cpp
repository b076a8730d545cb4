// collapse_study.cpp -- a CPU study, not part of the library: how many QNode visits and triangle tests a
// nearest-first 4-wide walk makes over two collapses of the same binary tree (the reference's Karras
// tree): the build's greedy rule (build.hip greedy_qnode_words: expand the largest-area internal entry,
// twice) and an SAH-optimal cut per node (dynamic programming over the binary subtree: D(x, 1) = the cost
// of x as an entry, D(x, j >= 2) = the cheapest cover of x's subtree by j entries; a node's QNode is its
// cheapest cover by 2..4 entries).  Exact float boxes, no quantization and no margins: the walk is the
// unchecked nearest-first one, counts only.
//
// Inputs (tests/collapse_study_inputs.py writes them, from the oracle build and trace): nodes.bin (the reference layout, 44-B records, leaves
// [0, T), internal k at T + k, root T), tris.bin (9 floats per sorted leaf: clip-space v0, v1, v2),
// rays.bin (6 floats per ray: origin, direction).  Usage: collapse_study DIR [C_tri] [max leaves per cluster]
// [width]; DUMP=path writes the greedy collapse's QNode visits per ray (uint32)
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Node {
    uint32_t parent, child_l, child_r, code;
    float bmin[3], bmax[3];
    uint32_t index;
};
static_assert(sizeof(Node) == 44, "44-B node");

static std::vector<char> slurp(const char* path) {
    std::vector<char> d;
    FILE* f = fopen(path, "rb");
    if (!f) return d;
    fseek(f, 0, SEEK_END);
    d.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(d.data(), 1, d.size(), f) != d.size()) d.clear();
    fclose(f);
    return d;
}

static double half_area(const Node& n) {
    const double dx = (double)n.bmax[0] - n.bmin[0], dy = (double)n.bmax[1] - n.bmin[1],
                 dz = (double)n.bmax[2] - n.bmin[2];
    return std::max(dx * dy + dy * dz + dz * dx, 0.0);
}

constexpr int WMAX = 8;
struct QNodeE {
    uint32_t e[WMAX];
    int n;
    float qb[WMAX][6];   // QUANT=1: the entries' boxes decoded from the node's 8-bit grid (build.hip quantize_axis)
};
// build.hip quantize_axis over n boxes: the decoded corners (origin + q * step, one rounding) that contain them
static float pow2f_(int e) { uint32_t u = (uint32_t)(e + 127) << 23; float f; memcpy(&f, &u, 4); return f; }
static void quantize(QNodeE& q, const Node* N) {
    for (int a = 0; a < 3; a++) {
        float o = INFINITY, m = -INFINITY;
        for (int k = 0; k < q.n; k++) { o = std::min(o, N[q.e[k]].bmin[a]); m = std::max(m, N[q.e[k]].bmax[a]); }
        const float ext = m - o;
        int e = -120;
        if (ext > 0.f) {
            uint32_t u; memcpy(&u, &ext, 4);
            e = std::max((int)((u >> 23) & 255u) - 127 - 8, -120);
        }
        while (std::fma(255.f, pow2f_(e), o) < m) ++e;
        const float sc = pow2f_(e), rs = pow2f_(-e);
        for (int k = 0; k < q.n; k++) {
            const float lo = N[q.e[k]].bmin[a], hi = N[q.e[k]].bmax[a];
            uint32_t l = (uint32_t)std::min(std::max(std::floor((lo - o) * rs), 0.f), 255.f);
            uint32_t h = (uint32_t)std::min(std::max(std::ceil((hi - o) * rs), 0.f), 255.f);
            if (l > 0 && std::fma((float)l, sc, o) > lo) --l;
            if (h < 255 && std::fma((float)h, sc, o) < hi) ++h;
            q.qb[k][a] = std::fma((float)l, sc, o);
            q.qb[k][3 + a] = std::fma((float)h, sc, o);
        }
    }
}

// the ray / box slab test (entry distance, hit)
static bool slab(const float o[3], const float inv[3], const Node& b, float best, float& tn) {
    float t0 = 0.f, t1 = best;
    for (int a = 0; a < 3; a++) {
        float lo = (b.bmin[a] - o[a]) * inv[a], hi = (b.bmax[a] - o[a]) * inv[a];
        if (lo > hi) std::swap(lo, hi);
        t0 = std::max(t0, lo);
        t1 = std::min(t1, hi);
    }
    tn = t0;
    return t0 <= t1;
}
static bool slab6(const float o[3], const float inv[3], const float* b, float best, float& tn) {
    Node n;
    for (int a = 0; a < 3; a++) { n.bmin[a] = b[a]; n.bmax[a] = b[3 + a]; }
    return slab(o, inv, n, best, tn);
}
// Moller-Trumbore as the kernels (EPSILON 0.01 on the determinant)
static float tri_hit(const float o[3], const float d[3], const float* v) {
    const float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
    const float h[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    const float a = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
    if (std::fabs(a) < 0.01f) return -1.f;
    const float f = 1.f / a;
    const float s[3] = {o[0] - v[0], o[1] - v[1], o[2] - v[2]};
    const float u = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
    if (u < 0.f || u > 1.f) return -1.f;
    const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float vv = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
    if (vv < 0.f || u + vv > 1.f) return -1.f;
    const float t = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
    return t > 0.01f ? t : -1.f;
}

// REBUILD=sah: a binned-SAH top-down binary tree over the same leaves (their boxes; 16 centroid bins on each
// axis, the cheapest plane), in place of the reference's Karras tree -- what a higher-quality tree would save
// the walk (max leaves 1 only: the leaf ranges of the Karras tree no longer hold)
struct SahBuilder {
    std::vector<Node>& N;
    uint32_t T;
    std::vector<uint32_t> idx;
    uint32_t next;   // internal ids from T + 1 (the root is T)
    static void grow(float (&b)[6], const Node& n) {
        for (int a = 0; a < 3; a++) { b[a] = std::min(b[a], n.bmin[a]); b[3 + a] = std::max(b[3 + a], n.bmax[a]); }
    }
    static double area(const float (&b)[6]) {
        const double dx = (double)b[3] - b[0], dy = (double)b[4] - b[1], dz = (double)b[5] - b[2];
        return dx < 0 ? 0.0 : dx * dy + dy * dz + dz * dx;
    }
    uint32_t alloc() {
        uint32_t v;
#pragma omp atomic capture
        v = next++;
        return v;
    }
    uint32_t build(size_t lo, size_t hi, uint32_t id) {
        if (hi - lo == 1) return idx[lo];
        constexpr int NB = 16;
        float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        float box[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
        for (size_t i = lo; i < hi; i++) {
            const Node& n = N[idx[i]];
            grow(box, n);
            for (int a = 0; a < 3; a++) {
                const float c = 0.5f * (n.bmin[a] + n.bmax[a]);
                cl[a] = std::min(cl[a], c); ch[a] = std::max(ch[a], c);
            }
        }
        int ba = -1, bb = 0;
        double bc = INFINITY;
        for (int a = 0; a < 3; a++) {
            if (!(ch[a] > cl[a])) continue;
            const float sc = NB / (ch[a] - cl[a]);
            float bx[NB][6];
            size_t cnt[NB] = {};
            for (auto& b : bx) { b[0] = b[1] = b[2] = INFINITY; b[3] = b[4] = b[5] = -INFINITY; }
            for (size_t i = lo; i < hi; i++) {
                const Node& n = N[idx[i]];
                const int k = std::min(NB - 1, (int)((0.5f * (n.bmin[a] + n.bmax[a]) - cl[a]) * sc));
                cnt[k]++;
                grow(bx[k], n);
            }
            double ra[NB];
            float acc[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
            size_t rc = 0, rcnt[NB];
            for (int k = NB - 1; k > 0; k--) {
                for (int q = 0; q < 3; q++) { acc[q] = std::min(acc[q], bx[k][q]); acc[3 + q] = std::max(acc[3 + q], bx[k][3 + q]); }
                rc += cnt[k];
                ra[k] = area(acc);
                rcnt[k] = rc;
            }
            float lacc[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
            size_t lc = 0;
            for (int k = 0; k < NB - 1; k++) {
                for (int q = 0; q < 3; q++) { lacc[q] = std::min(lacc[q], bx[k][q]); lacc[3 + q] = std::max(lacc[3 + q], bx[k][3 + q]); }
                lc += cnt[k];
                if (lc == 0 || rcnt[k + 1] == 0) continue;
                const double c = area(lacc) * lc + ra[k + 1] * rcnt[k + 1];
                if (c < bc) { bc = c; ba = a; bb = k; }
            }
        }
        size_t mid;
        if (ba < 0) {
            mid = (lo + hi) / 2;   // every centroid equal: halves
        } else {
            const float sc = NB / (ch[ba] - cl[ba]);
            auto it = std::partition(idx.begin() + lo, idx.begin() + hi, [&](uint32_t j) {
                const Node& n = N[j];
                return std::min(NB - 1, (int)((0.5f * (n.bmin[ba] + n.bmax[ba]) - cl[ba]) * sc)) <= bb;
            });
            mid = (size_t)(it - idx.begin());
            if (mid == lo || mid == hi) mid = (lo + hi) / 2;
        }
        const uint32_t il = hi - lo > 2 && mid - lo > 1 ? alloc() : 0, ir = hi - mid > 1 ? alloc() : 0;
        uint32_t l, r;
        if (hi - lo > 200000) {
#pragma omp task shared(l)
            l = build(lo, mid, il);
#pragma omp task shared(r)
            r = build(mid, hi, ir);
#pragma omp taskwait
        } else {
            l = build(lo, mid, il);
            r = build(mid, hi, ir);
        }
        Node& n = N[id];
        n.child_l = l;
        n.child_r = r;
        N[l].parent = id;
        N[r].parent = id;
        for (int a = 0; a < 3; a++) { n.bmin[a] = box[a]; n.bmax[a] = box[3 + a]; }
        return id;
    }
};

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: collapse_study DIR [C_tri]\n");
        return 2;
    }
    const double CT = argc > 2 ? atof(argv[2]) : 0.5, CI = 1.0;
    const uint32_t ML = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;   // leaf clusters: subtrees of <= ML leaves
    const int W = argc > 4 ? std::min(std::max(atoi(argv[4]), 2), WMAX) : 4;   // the greedy collapse's width
    char path[1024];
    snprintf(path, sizeof path, "%s/nodes.bin", argv[1]);
    std::vector<char> nb = slurp(path);
    snprintf(path, sizeof path, "%s/tris.bin", argv[1]);
    std::vector<char> tb = slurp(path);
    snprintf(path, sizeof path, "%s/rays.bin", argv[1]);
    std::vector<char> rb = slurp(path);
    const Node* N = reinterpret_cast<const Node*>(nb.data());
    const size_t NN = nb.size() / sizeof(Node);
    const uint32_t T = (uint32_t)((NN + 1) / 2);
    std::vector<Node> rebuilt;
    const char* rebuild = getenv("REBUILD");
    if (rebuild && !strcmp(rebuild, "sah") && T >= 2) {
        rebuilt.assign(N, N + NN);
        SahBuilder B{rebuilt, T, std::vector<uint32_t>(T), T + 1};
        for (uint32_t j = 0; j < T; j++) B.idx[j] = j;
#pragma omp parallel
#pragma omp single
        B.build(0, T, T);
        rebuilt[T].parent = ~0u;
        N = rebuilt.data();
        fprintf(stderr, "rebuilt: %u internal nodes\n", B.next - T);
    }
    const float* tri = reinterpret_cast<const float*>(tb.data());
    const float* rays = reinterpret_cast<const float*>(rb.data());
    const size_t R = rb.size() / (6 * sizeof(float));
    if (T < 2 || tb.size() != (size_t)T * 9 * sizeof(float) || R == 0) {
        fprintf(stderr, "bad inputs (T %u, rays %zu)\n", T, R);
        return 2;
    }
    const uint32_t root = T;
    // leaves below each node (a cluster: <= ML of them, tested as one entry -- all its triangles)
    std::vector<uint32_t> nleaf(NN, 1), first(NN);
    for (uint32_t j = 0; j < T; j++) first[j] = j;
    {
        std::vector<std::pair<uint32_t, bool>> st{{T, false}};
        while (!st.empty()) {
            auto [x, done] = st.back();
            st.pop_back();
            if (x < T) continue;
            if (done) {
                nleaf[x] = nleaf[N[x].child_l] + nleaf[N[x].child_r];
                first[x] = std::min(first[N[x].child_l], first[N[x].child_r]);
                continue;
            }
            st.push_back({x, true});
            st.push_back({N[x].child_l, false});
            st.push_back({N[x].child_r, false});
        }
    }
    auto leaf = [&](uint32_t x) { return x < T || nleaf[x] <= ML; };
    // post-order of the internal nodes
    std::vector<uint32_t> order;
    order.reserve(T);
    {
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            auto [x, done] = st.back();
            st.pop_back();
            if (leaf(x)) continue;
            if (done) { order.push_back(x); continue; }
            st.push_back({x, true});
            st.push_back({N[x].child_l, false});
            st.push_back({N[x].child_r, false});
        }
    }
    // greedy collapse (build.hip greedy_qnode_words)
    std::vector<QNodeE> greedy(NN), sah(NN);
    // LEAFRUN=1: the leaf entries of a node must be one run of consecutive sorted leaves (a 64-B 6-wide node
    // addresses them by the run's first leaf and a mask): an expansion that would break the run is skipped
    const bool leafrun = getenv("LEAFRUN") != nullptr;
    const bool quant = getenv("QUANT") != nullptr;
    auto run_ok = [&](const uint32_t* E, int n) {
        uint32_t lo = ~0u, hi = 0, c = 0;
        for (int k = 0; k < n; k++)
            if (E[k] < T) { lo = std::min(lo, E[k]); hi = std::max(hi, E[k]); ++c; }
        return c == 0 || hi - lo + 1 == c;
    };
    for (uint32_t x : order) {
        uint32_t E[WMAX] = {N[x].child_l, N[x].child_r};
        int n = 2;
        for (int step = 0; step < W - 2; step++) {   // (W = 4: build.hip's rule, which looks at the first 3)
            int pick = -1;
            double best = -1;
            for (int k = 0; k < n && k < W - 1; k++)
                if (!leaf(E[k])) {
                    const double ar = half_area(N[E[k]]);
                    if (ar > best) {
                        if (leafrun) {   // the expansion keeps the leaf run
                            uint32_t F[WMAX];
                            memcpy(F, E, sizeof F);
                            F[k] = N[E[k]].child_l;
                            F[n] = N[E[k]].child_r;
                            if (!run_ok(F, n + 1)) continue;
                        }
                        best = ar;
                        pick = k;
                    }
                }
            if (pick < 0) break;
            const uint32_t sel = E[pick];
            E[pick] = N[sel].child_l;
            E[n] = N[sel].child_r;
            ++n;
        }
        QNodeE& q = greedy[x];
        q.n = n;
        for (int k = 0; k < WMAX; k++) q.e[k] = k < n ? E[k] : 0;
        if (quant) quantize(q, N);
    }
    // SAH-optimal cuts: D[x][j], j = 1..4
    const double INF = 1e300;
    std::vector<std::array<double, 5>> D(NN);
    std::vector<double> C(NN, 0.0);
    for (uint32_t j = 0; j < T; j++) {
        D[j].fill(INF);
        D[j][1] = half_area(N[j]) * CT;
    }
    for (uint32_t x : order) {
        if (leaf(x)) {
            D[x].fill(INF);
            D[x][1] = half_area(N[x]) * CT * nleaf[x];
            continue;
        }
        const uint32_t l = N[x].child_l, r = N[x].child_r;
        std::array<double, 5> e;
        e.fill(INF);
        for (int j = 2; j <= 4; j++)
            for (int a = 1; a < j; a++) e[j] = std::min(e[j], D[l][a] + D[r][j - a]);
        C[x] = std::min(e[2], std::min(e[3], e[4]));
        D[x] = e;
        D[x][1] = half_area(N[x]) * CI + C[x];
    }
    auto cut = [&](auto&& self, uint32_t x, int j, std::vector<uint32_t>& out) -> void {
        if (j == 1) { out.push_back(x); return; }
        const uint32_t l = N[x].child_l, r = N[x].child_r;
        int ba = 1;
        double bv = INF;
        for (int a = 1; a < j; a++)
            if (D[l][a] + D[r][j - a] < bv) { bv = D[l][a] + D[r][j - a]; ba = a; }
        self(self, l, ba, out);
        self(self, r, j - ba, out);
    };
    for (uint32_t x : order) {
        int bj = 2;
        double bv = INF;
        for (int j = 2; j <= 4; j++) {
            double v = INF;
            for (int a = 1; a < j; a++) v = std::min(v, D[N[x].child_l][a] + D[N[x].child_r][j - a]);
            if (v < bv) { bv = v; bj = j; }
        }
        std::vector<uint32_t> out;
        cut(cut, x, bj, out);
        QNodeE& q = sah[x];
        q.n = (int)out.size();
        for (int k = 0; k < WMAX; k++) q.e[k] = k < q.n ? out[k] : 0;
    }
    // the SAH cost of both (from the root, per unit root area)
    auto sah_cost = [&](const std::vector<QNodeE>& Q) {
        double c = 0;
        std::vector<uint32_t> st{root};
        while (!st.empty()) {
            const uint32_t x = st.back();
            st.pop_back();
            if (leaf(x)) { c += half_area(N[x]) * CT * nleaf[x]; continue; }
            c += half_area(N[x]) * CI;
            for (int k = 0; k < Q[x].n; k++) st.push_back(Q[x].e[k]);
        }
        return c / half_area(N[root]);
    };
    // the nearest-first walk, counts
    auto walk = [&](const std::vector<QNodeE>& Q, uint64_t& qv, uint64_t& lt, uint64_t& reached, uint64_t& lsteps) {
        qv = lt = reached = lsteps = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : qv, lt, reached, lsteps)
        for (size_t i = 0; i < R; i++) {
            const float* o = rays + 6 * i;
            const float* d = o + 3;
            const float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
            float best = INFINITY;
            std::vector<std::pair<uint32_t, float>> st;
            st.reserve(256);
            st.push_back({root, 0.f});
            while (!st.empty()) {
                auto [x, t] = st.back();
                st.pop_back();
                if (t > best) continue;
                if (leaf(x)) {
                    ++lsteps;
                    for (uint32_t j = first[x]; j < first[x] + nleaf[x]; j++) {
                        ++lt;
                        const float h = tri_hit(o, d, tri + 9 * (size_t)j);
                        if (h > 0.f && h < best) best = h;
                    }
                    continue;
                }
                ++qv;
                std::pair<uint32_t, float> hit[WMAX];
                int nh = 0;
                for (int k = 0; k < Q[x].n; k++) {
                    float tn;
                    if (slab(o, inv, N[Q[x].e[k]], best, tn)) hit[nh++] = {Q[x].e[k], tn};
                }
                std::sort(hit, hit + nh, [](auto& a, auto& b) { return a.second > b.second; });   // farthest first
                for (int k = 0; k < nh; k++) st.push_back(hit[k]);
            }
            reached += best < INFINITY;
        }
    };
    // STEPS=1: the bounce kernel's loop (trace.hip k_bounce_trav, WIDE): a step tests one QNode and then one
    // leaf -- the nearest child when it is a leaf (the next child goes on without a push), or the leaf the
    // step began at -- and pops until an entry's key is within the bound.  ORDER 0: the children by entry
    // distance (the kernel's sort); 1: the nearest first, the others pushed in slot order (no sort)
    uint64_t deep[4] = {0, 0, 0, 0};   // steps that end with > 13 / > 20 / > 32 stack entries, pushes
    auto steps_walk = [&](const std::vector<QNodeE>& Q, int order, double& steps, double& qv, double& lt) {
        uint64_t S = 0, V = 0, L = 0, D0 = 0, D1 = 0, D2 = 0, PU = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : S, V, L, D0, D1, D2, PU)
        for (size_t i = 0; i < R; i++) {
            const float* o = rays + 6 * i;
            const float* d = o + 3;
            const float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
            float best = INFINITY;
            std::vector<std::pair<uint32_t, float>> st;
            st.reserve(256);
            constexpr uint32_t NONE = ~0u;
            uint32_t node = root;
            while (true) {
                ++S;
                uint32_t lf = NONE;
                if (leaf(node)) {
                    lf = node;
                    node = NONE;
                } else {
                    ++V;
                    std::pair<uint32_t, float> hit[WMAX];
                    int nh = 0;
                    for (int k = 0; k < Q[node].n; k++) {
                        float tn;
                        const bool h = quant ? slab6(o, inv, Q[node].qb[k], best, tn)
                                             : slab(o, inv, N[Q[node].e[k]], best, tn);
                        if (h) hit[nh++] = {Q[node].e[k], tn};
                    }
                    if (order == 0) {
                        std::stable_sort(hit, hit + nh, [](auto& a, auto& b) { return a.second < b.second; });
                    } else if (nh > 1) {   // the nearest to the front, the others in slot order
                        int m = 0;
                        for (int k = 1; k < nh; k++) if (hit[k].second < hit[m].second) m = k;
                        std::rotate(hit, hit + m, hit + m + 1);
                    }
                    int k0 = 0;
                    node = NONE;
                    if (nh > 0 && leaf(hit[0].first)) { lf = hit[0].first; k0 = 1; }
                    if (k0 < nh) node = hit[k0].first;
                    for (int k = nh - 1; k > k0; k--) st.push_back(hit[k]);
                    PU += nh > k0 ? nh - k0 - 1 : 0;
                }
                D0 += st.size() > 13;
                D1 += st.size() > 20;
                D2 += st.size() > 32;
                if (lf != NONE) {
                    for (uint32_t j = first[lf]; j < first[lf] + nleaf[lf]; j++) {
                        ++L;
                        const float h = tri_hit(o, d, tri + 9 * (size_t)j);
                        if (h > 0.f && h < best) best = h;
                    }
                }
                while (node == NONE && !st.empty()) {
                    auto [x, t] = st.back();
                    st.pop_back();
                    if (t <= best) node = x;
                }
                if (node == NONE) break;
            }
        }
        steps = (double)S / R;
        deep[0] = D0; deep[1] = D1; deep[2] = D2; deep[3] = PU;
        qv = (double)V / R;
        lt = (double)L / R;
    };
    if (getenv("STEPS")) {
        for (int order = 0; order < 2; order++) {
            double sS, sV, sL;
            steps_walk(greedy, order, sS, sV, sL);
            printf("{\"T\": %u, \"rays\": %zu, \"width\": %d, \"leafrun\": %d, \"quant\": %d, \"order\": \"%s\", "
                   "\"steps\": %.4f, \"qnode_visits\": %.4f, \"leaf_tests\": %.4f, \"fetches\": %.4f, "
                   "\"steps_past_13_20_32_entries\": [%.4f, %.4f, %.4f], \"pushes\": %.4f}\n", T, R, W, (int)leafrun,
                   (int)quant, order ? "nearest, slot order" : "sorted", sS, sV, sL, sV + sL, (double)deep[0] / R,
                   (double)deep[1] / R, (double)deep[2] / R, (double)deep[3] / R);
        }
        return 0;
    }
    if (const char* dump = getenv("DUMP")) {   // per-ray QNode visits of the greedy collapse (uint32)
        std::vector<uint32_t> vis(R);
#pragma omp parallel for schedule(dynamic, 256)
        for (size_t i = 0; i < R; i++) {
            const float* o = rays + 6 * i;
            const float* d = o + 3;
            const float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
            float best = INFINITY;
            uint32_t v = 0;
            std::vector<std::pair<uint32_t, float>> st{{root, 0.f}};
            while (!st.empty()) {
                auto [x, t] = st.back();
                st.pop_back();
                if (t > best) continue;
                if (leaf(x)) {
                    for (uint32_t j = first[x]; j < first[x] + nleaf[x]; j++) {
                        const float h = tri_hit(o, d, tri + 9 * (size_t)j);
                        if (h > 0.f && h < best) best = h;
                    }
                    continue;
                }
                ++v;
                std::pair<uint32_t, float> hit[WMAX];
                int nh = 0;
                for (int k = 0; k < greedy[x].n; k++) {
                    float tn;
                    if (slab(o, inv, N[greedy[x].e[k]], best, tn)) hit[nh++] = {greedy[x].e[k], tn};
                }
                std::sort(hit, hit + nh, [](auto& a, auto& b) { return a.second > b.second; });
                for (int k = 0; k < nh; k++) st.push_back(hit[k]);
            }
            vis[i] = v;
        }
        FILE* f = fopen(dump, "wb");
        if (f) { fwrite(vis.data(), 4, R, f); fclose(f); }
    }
    uint64_t gq, gl, gr, sq, sl, sr, gs, ss;
    walk(greedy, gq, gl, gr, gs);
    walk(sah, sq, sl, sr, ss);
    size_t gn = 0, sn = 0, g4 = 0, s4 = 0;
    for (uint32_t x : order) { gn += greedy[x].n; sn += sah[x].n; g4 += greedy[x].n == W; s4 += sah[x].n == 4; }
    printf("{\"T\": %u, \"rays\": %zu, \"C_tri\": %.3f, \"max_leaves\": %u, \"width\": %d, \"greedy\": {\"sah\": %.4f, \"qnode_visits\": %.4f, \"leaf_tests\": %.4f, \"leaf_steps\": %.4f, "
           "\"hits\": %llu, \"four_wide_frac\": %.4f}, \"sah_opt\": {\"sah\": %.4f, \"qnode_visits\": %.4f, \"leaf_tests\": %.4f, \"leaf_steps\": %.4f, "
           "\"hits\": %llu, \"four_wide_frac\": %.4f}}\n",
           T, R, CT, ML, W, sah_cost(greedy), (double)gq / R, (double)gl / R, (double)gs / R, (unsigned long long)gr,
           (double)g4 / order.size(), sah_cost(sah), (double)sq / R, (double)sl / R, (double)ss / R,
           (unsigned long long)sr, (double)s4 / order.size());
    (void)gn;
    (void)sn;
    return 0;
}
