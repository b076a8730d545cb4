// gather_roofline.hip -- what the memory system delivers for the traversal's access
// pattern, measured with hipEvents on MI355X.  The traversal kernels
// fetch one 64-B record per lane per step from random places of a > 256-MiB table, and
// each fetch depends on the previous one (the next node id comes out of the record).
// Kernels, all over a 1.25-GiB table of 64-B records (the C5 QNode + leaf arrays):
//   k_stream  coalesced 16 B/lane streaming read of the table    (HBM streaming peak)
//   k_gather  one random 64-B record per lane, no dependence     (random-gather peak)
//   k_chase   persistent lanes, each walking a chain of STEPS dependent random 64-B
//             records (next = hash of the loaded words): the traversal's pattern without
//             its arithmetic.  Rate = records/s, and the latency of one step under load.
// Usage: gather_roofline [waves_per_simd=8] [steps=256] [table_mib=1280]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_fill(uint4* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i * 0x9E3779B1u, (uint32_t)(i >> 2) * 0x85EBCA6Bu, (uint32_t)i, 1u);
}

__global__ void k_stream(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// record r = (i * odd) mod nrec (nrec a power of two): each record once, in random order
__global__ void k_gather(const uint4* __restrict__ a, uint32_t nrec, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const uint32_t r = (i * 0x9E3779B1u) & (nrec - 1);
    const uint4* p = a + 4 * (size_t)r;
    const uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
    const uint32_t s = v0.x ^ v1.y ^ v2.z ^ v3.w;
    if (s == 0x12345u) out[0] = s;
}

__global__ __launch_bounds__(256) void k_chase(const uint4* __restrict__ a, uint32_t nrec, uint32_t steps,
                                               uint32_t* out) {
    uint32_t r = ((blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B1u) & (nrec - 1);
    uint32_t s = 0;
    for (uint32_t k = 0; k < steps; k++) {
        const uint4* p = a + 4 * (size_t)r;
        const uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
        s ^= v1.y ^ v2.z ^ v3.w;
        r = (v0.x ^ (r * 0x85EBCA6Bu) ^ k) & (nrec - 1);   // the next record depends on this one
    }
    if (s == 0x12345u) out[0] = s ^ r;
}

// k_chase with RECW-byte records (RECW = 16, 32, 64, 128): does the rate follow the records
// (requests) or the bytes / load instructions?
template <int RECW>
__global__ __launch_bounds__(256) void k_chase_w(const uint4* __restrict__ a, uint32_t nrec, uint32_t steps,
                                                 uint32_t* out) {
    uint32_t r = ((blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B1u) & (nrec - 1);
    uint32_t s = 0;
    for (uint32_t k = 0; k < steps; k++) {
        const uint4* p = a + (RECW / 16) * (size_t)r;
        uint4 v = p[0];
        if (RECW >= 32) { const uint4 w = p[1]; v.y ^= w.x; v.z ^= w.w; }
        if (RECW >= 64) { const uint4 w = p[2], x = p[3]; v.y ^= w.x ^ x.y; v.z ^= w.w ^ x.z; }
        if (RECW >= 128) {
            const uint4 w = p[4], x = p[5], y = p[6], z = p[7];
            v.y ^= w.x ^ x.y ^ y.z ^ z.w;
            v.z ^= w.w ^ x.z ^ y.y ^ z.x;
        }
        s ^= v.y ^ v.z;
        r = (v.x ^ (r * 0x85EBCA6Bu) ^ k) & (nrec - 1);
    }
    if (s == 0x12345u) out[0] = s ^ r;
}

int main(int argc, char** argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t steps = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
    const uint32_t nrec = (uint32_t)((argc > 3 ? atoi(argv[3]) : 1280) << 14);   // MiB -> 64-B records
    uint32_t nrec2 = 1;
    while (nrec2 * 2 <= nrec) nrec2 *= 2;   // 16 Mi: power of two for the index masks
    const size_t bytes = (size_t)nrec * 64;
    uint4* a;
    uint32_t* out;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&out, 4));
    k_fill<<<4096, 256>>>(a, bytes / 16);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    auto timed = [&](auto launch, int reps) {
        launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < reps; i++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / reps;
    };
    const float ms_stream = timed([&] { k_stream<<<cus * 32, 256>>>(reinterpret_cast<const float4*>(a), bytes / 16, reinterpret_cast<float*>(out)); }, 10);
    const float ms_gather = timed([&] { k_gather<<<nrec2 / 256, 256>>>(a, nrec2, out); }, 10);
    const uint32_t blocks = (uint32_t)(cus * 4 * wps / 4);   // 4 waves per 256-thread block
    if (nrec2 < 256) return 1;
    const float ms_chase = timed([&] { k_chase<<<blocks, 256>>>(a, nrec2, steps, out); }, 5);
    // the same table as 16- and 32-B records (4x / 2x as many, same bytes)
    uint32_t n16 = 1, n32 = 1, n64 = 1, n128 = 1;
    while (n16 * 2 <= (uint32_t)(bytes / 16)) n16 *= 2;
    while (n32 * 2 <= (uint32_t)(bytes / 32)) n32 *= 2;
    while (n64 * 2 <= (uint32_t)(bytes / 64)) n64 *= 2;
    while (n128 * 2 <= (uint32_t)(bytes / 128)) n128 *= 2;
    const float ms_c16 = timed([&] { k_chase_w<16><<<blocks, 256>>>(a, n16, steps, out); }, 5);
    const float ms_c32 = timed([&] { k_chase_w<32><<<blocks, 256>>>(a, n32, steps, out); }, 5);
    const float ms_c64 = timed([&] { k_chase_w<64><<<blocks, 256>>>(a, n64, steps, out); }, 5);
    const float ms_c128 = timed([&] { k_chase_w<128><<<blocks, 256>>>(a, n128, steps, out); }, 5);
    CHECK(hipDeviceSynchronize());
    const double lanes = (double)blocks * 256;
    const double recs = lanes * steps;
    printf("{\"cus\": %d, \"table_bytes\": %zu, \"stream_gbs\": %.1f, \"gather_records_per_s\": %.4g, "
           "\"gather_record_gbs\": %.1f, \"gather_line_gbs\": %.1f, \"chase_waves_per_simd\": %d, \"chase_lanes\": %.0f, "
           "\"chase_steps\": %u, \"chase_ms\": %.4f, \"chase_records_per_s\": %.4g, \"chase_record_gbs\": %.1f, "
           "\"chase_step_latency_us\": %.3f, \"chase16_records_per_s\": %.4g, \"chase32_records_per_s\": %.4g, "
           "\"chase64w_records_per_s\": %.4g, \"chase128_records_per_s\": %.4g}\n",
           cus, bytes, bytes / (ms_stream * 1e-3) / 1e9, nrec2 / (ms_gather * 1e-3),
           nrec2 * 64.0 / (ms_gather * 1e-3) / 1e9, nrec2 * 128.0 / (ms_gather * 1e-3) / 1e9, wps, lanes, steps,
           ms_chase, recs / (ms_chase * 1e-3), recs * 64 / (ms_chase * 1e-3) / 1e9, ms_chase * 1e3 / steps,
           recs / (ms_c16 * 1e-3), recs / (ms_c32 * 1e-3), recs / (ms_c64 * 1e-3), recs / (ms_c128 * 1e-3));
    return 0;
}
