// write_roofline.hip -- what HBM delivers for the write patterns of the build's refit stage
// (k_refit writes 64-B node records, leaf pseudo-records and QNodes), timed with hipEvents
// on MI355X over a 1.25-GiB region (past the 256-MiB Infinity Cache):
//   stream16   coalesced 16 B/lane stores (the leaf records in sorted order)
//   rec64      one 64-B record per lane (4 x dwordx4) at a permuted slot: a lone half line
//   pair128    one lane writes both 64-B halves of a 128-B line (slots 2i, 2i+1), lines permuted
//   rec64seq   one 64-B record per lane at slot i (lanes of a wave cover 4 KB contiguously)
//   half64     one 64-B record per lane at slot 2i (every other half line, never the sibling)
// Prints one JSON line per pattern: GB/s of bytes written.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_stream16(float4* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}
__device__ __forceinline__ void put64(float4* p, uint32_t i) {
    p[0] = make_float4((float)i, 1.f, 2.f, 3.f);
    p[1] = make_float4(4.f, 5.f, 6.f, 7.f);
    p[2] = make_float4(8.f, 9.f, 10.f, 11.f);
    p[3] = make_float4(12.f, 13.f, 14.f, 15.f);
}
// slot r = (i * 0x9E3779B1) mod nrec: a permutation of [0, nrec) (nrec a power of two)
__global__ void k_rec64(float4* __restrict__ a, uint32_t nrec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    put64(a + 4 * (size_t)((i * 0x9E3779B1u) & (nrec - 1)), i);
}
__global__ void k_pair128(float4* __restrict__ a, uint32_t nline) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nline) return;
    float4* p = a + 8 * (size_t)((i * 0x9E3779B1u) & (nline - 1));
    put64(p, i);
    put64(p + 4, i);
}
__global__ void k_rec64seq(float4* __restrict__ a, uint32_t nrec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nrec) put64(a + 4 * (size_t)i, i);
}
__global__ void k_half64(float4* __restrict__ a, uint32_t nline) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nline) put64(a + 8 * (size_t)i, i);
}

int main() {
    const size_t bytes = 1280ull << 20;   // 1.25 GiB
    float4* a;
    CHECK(hipMalloc(&a, 2 * bytes));
    CHECK(hipMemset(a, 0, 2 * bytes));
    const uint32_t nrec = 1u << 24;       // 16 Mi records of 64 B = 1 GiB (a power of two for the permutation)
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct R { const char* name; double bytes; float best; } res[5] = {
        {"stream16", (double)bytes, 1e9f}, {"rec64", 64.0 * nrec, 1e9f}, {"pair128", 64.0 * nrec, 1e9f},
        {"rec64seq", 64.0 * nrec, 1e9f}, {"half64", 64.0 * (nrec / 2), 1e9f}};
    for (int it = 0; it < 5; ++it) {
        for (int k = 0; k < 5; ++k) {
            CHECK(hipEventRecord(e0));
            switch (k) {
                case 0: k_stream16<<<8192, 256>>>(a, bytes / 16); break;
                case 1: k_rec64<<<nrec / 256, 256>>>(a, nrec); break;
                case 2: k_pair128<<<nrec / 2 / 256, 256>>>(a, nrec / 2); break;
                case 3: k_rec64seq<<<nrec / 256, 256>>>(a, nrec); break;
                case 4: k_half64<<<nrec / 2 / 256, 256>>>(a, nrec / 2); break;
            }
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < res[k].best) res[k].best = ms;
        }
    }
    for (int k = 0; k < 5; ++k)
        printf("{\"pattern\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f, \"gbs\": %.1f}\n", res[k].name, res[k].bytes,
               res[k].best, res[k].bytes / (res[k].best * 1e-3) / 1e9);
    return 0;
}
