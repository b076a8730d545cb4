// gather_policy.hip -- the refit's sorted-order gather (build.hip leaf_record_words: 48 B of a 64-B
// clip record per sorted leaf, records in random order, each read once) under the load cache
// policies of gfx950 (buffer loads, aux = sc0 1 | nt 2 | sc1 16).  Does any policy make the L2
// fetch 64 B instead of its 128-B line (TCC_EA0_RDREQ_64B vs _128B under rocprofv3 --pmc), and
// what does each cost in time?  Each variant is its own kernel instance (k_gather_pol<AUX>).
// Usage: gather_policy [nrec=10000000]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint4* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i * 0x9E3779B1u, (uint32_t)(i >> 2) * 0x85EBCA6Bu, (uint32_t)i, 1u);
}

// the permutation the sort hands the refit: perm[i] = (i * odd + c) mod n for n a power of two is a
// bijection; for other n, a multiplicative hash folded into range (a few records twice: fine here)
__global__ void k_perm(uint32_t* p, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)(((uint64_t)(i * 0x9E3779B1u + 0x7F4A7C15u) * n) >> 32);
}

template <int AUX>
__global__ __launch_bounds__(256) void k_gather_pol(const uint4* __restrict__ a, const uint32_t* __restrict__ perm,
                                                    uint32_t n, uint4* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = perm[i];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a, (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t off = t * 64u;
    const v4i s0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX);
    const v4i s1 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, AUX);
    const v4i s2 = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32, 0, AUX);
    // a 64-B record per sorted position, as the leaf records
    uint4* o = out + 4 * (size_t)i;
    o[0] = make_uint4(s0.x, s0.y, s0.z, s1.x);
    o[1] = make_uint4(s1.y, s1.z, s2.x, s2.y);
    o[2] = make_uint4(s2.z, t, s0.w, s1.w);
    o[3] = make_uint4(s2.w, 0u, 0u, 0u);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 10000000u;
    uint4 *a, *out;
    uint32_t* perm;
    CHECK(hipMalloc(&a, (size_t)n * 64));
    CHECK(hipMalloc(&out, (size_t)n * 64));
    CHECK(hipMalloc(&perm, (size_t)n * 4));
    k_fill<<<4096, 256>>>(a, (size_t)n * 4);
    k_perm<<<(n + 255) / 256, 256>>>(perm, n);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // a 512-MiB sweep between launches evicts the table from the Infinity Cache
    uint4* flush;
    const size_t fl = (size_t)512 << 20;
    CHECK(hipMalloc(&flush, fl));
    auto timed = [&](auto launch) {
        float tot = 0.f;
        for (int r = 0; r < 5; r++) {
            k_fill<<<4096, 256>>>(flush, fl / 16);
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r) tot += ms;
        }
        return tot / 4;
    };
    const uint32_t blocks = (n + 255) / 256;
#define RUN(AUX) timed([&] { k_gather_pol<AUX><<<blocks, 256>>>(a, perm, n, out); })
    const float m0 = RUN(0), m1 = RUN(1), m2 = RUN(2), m16 = RUN(16), m17 = RUN(17), m19 = RUN(19), m3 = RUN(3);
    CHECK(hipDeviceSynchronize());
    printf("{\"n\": %u, \"ms\": {\"default\": %.4f, \"sc0\": %.4f, \"nt\": %.4f, \"sc1\": %.4f, \"sc0_sc1\": %.4f, "
           "\"sc0_sc1_nt\": %.4f, \"sc0_nt\": %.4f}}\n", n, m0, m1, m2, m16, m17, m19, m3);
    return 0;
}
