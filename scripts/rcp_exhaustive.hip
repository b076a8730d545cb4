// Exhaustive check of the correctly rounded fp32 reciprocal used by the triangle test
// (trace.hip rcp_rn): v_rcp_f32 + one fma Newton step, against the IEEE division 1.f / x,
// over every fp32 bit pattern x with 2^-126 <= |x| < 2^126 (normal x, normal 1/x), by
// exponent band.  Prints one JSON line: patterns tested, mismatches, the first few.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o scripts/rcp_exhaustive scripts/rcp_exhaustive.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_rn(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, r, 1.0f);
    return fmaf(e, r, r);
}

__global__ void k_check(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (uint32_t s = 0; s < 2; s++) {   // both signs
        const uint32_t bits = (lo + i) | (s << 31);
        const float x = __uint_as_float(bits);
        const float ref = 1.0f / x;
        const float got = rcp_rn(x);
        if (__float_as_uint(ref) != __float_as_uint(got)) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 8) first[k] = bits;
        }
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 32);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0, 32);
    const uint32_t lo = 1u << 23;            // 2^-126
    const uint32_t hi = (126u + 127u) << 23;  // 2^126
    const uint32_t chunk = 1u << 28;
    unsigned long long tested = 0;
    for (uint32_t b = lo; b < hi; b += chunk) {
        const uint32_t n = (hi - b) < chunk ? (hi - b) : chunk;
        hipLaunchKernelGGL(k_check, dim3((n + 255) / 256), dim3(256), 0, 0, b, n, bad, first);
        tested += 2ull * n;
    }
    unsigned long long hb = 0;
    uint32_t hf[8];
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(hf, first, 32, hipMemcpyDeviceToHost);
    printf("{\"tested\": %llu, \"mismatches\": %llu, \"first\": [", tested, hb);
    for (int k = 0; k < 8 && k < (int)hb; k++) printf("%s\"0x%08x\"", k ? ", " : "", hf[k]);
    printf("]}\n");
    return 0;
}
