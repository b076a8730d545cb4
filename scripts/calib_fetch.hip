// calib_fetch.hip -- calibrates rocprofv3 FETCH_SIZE against known byte counts for
// the access patterns of the trace kernels (MI355X_MICROARCH.md: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Three kernels over a 4-GiB table (past the 256-MiB Infinity Cache):
//   k_stream   coalesced 16 B/lane streaming read            (guide: FETCH = 1/2)
//   k_rec64    one 64-B record per lane (4 x dwordx4), records scattered by a
//              permutation of the table (the node-record gather of traversal)
//   k_rec64w   as k_rec64 but all 64 lanes of a wave read the same record
// Each kernel touches every byte it reads exactly once.  Prints the byte counts.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_stream(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// records r = (i * 0x9E3779B1) mod nrec, nrec a power of two: a permutation of [0, nrec)
__global__ void k_rec64(const float4* __restrict__ a, uint32_t nrec, float* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const uint32_t r = (i * 0x9E3779B1u) & (nrec - 1);
    const float4* p = a + 4 * (size_t)r;
    const float4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
    const float s = v0.x + v1.y + v2.z + v3.w;
    if (s == 1234.5f) out[0] = s;
}

__global__ void k_rec64w(const float4* __restrict__ a, uint32_t nrec, float* out) {
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= nrec) return;
    const uint32_t r = (w * 0x9E3779B1u) & (nrec - 1);
    const float4* p = a + 4 * (size_t)r;
    const float4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
    const float s = v0.x + v1.y + v2.z + v3.w;
    if (s == 1234.5f) out[0] = s;
}

int main() {
    const size_t bytes = 4ull << 30;
    float4* a;
    float* out;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(a, 0, bytes));
    const uint32_t nrec = (uint32_t)(bytes / 64);          // 64 Mi records
    const uint32_t nsub = nrec / 4;                         // rec64: 16 Mi records = 1 GiB
    for (int it = 0; it < 2; ++it) {
        k_stream<<<4096, 256>>>(a, bytes / 16, out);
        k_rec64<<<nrec / 256, 256>>>(a, nrec, out);
        k_rec64w<<<nsub * 64 / 256, 256>>>(a, nsub, out);
    }
    CHECK(hipDeviceSynchronize());
    printf("k_stream bytes %zu\nk_rec64 bytes %zu\nk_rec64w bytes %zu\n", bytes, (size_t)nrec * 64, (size_t)nsub * 64);
    return 0;
}
