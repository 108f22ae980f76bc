// Exhaustive check of rtow_device.hip's sqrt_pos (v_sqrt_f32 plus the two
// one-ulp FMA corrections, without sqrtf's small-input rescaling and its
// special-value selects) against the correctly rounded sqrtf, over every
// positive float bit pattern (denormals, normals, +inf).
//   hipcc --offload-arch=gfx950 -O3 -o tools/sqrt_check tools/sqrt_check.hip
// Prints the mismatch count per range (denormal / [2^-126, 2^-96) / >= 2^-96).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float sqrt_pos(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = fmaf(-sdn, s, x), rup = fmaf(-sup, s, x);
    const float t = rdn <= 0.0f ? sdn : s;
    return rup > 0.0f ? sup : t;
}

__global__ void check(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t u = lo + i;
        const float x = __uint_as_float(u);
        const float a = sqrtf(x), b = sqrt_pos(x);
        if (__float_as_uint(a) != __float_as_uint(b)) {
            const int r = u < 0x00800000u ? 0 : (u < 0x0f800000u ? 1 : 2);  // 2^-96 = 0x0f800000
            atomicAdd(&bad[r], 1ull);
            atomicMin(&first[r], u);
            atomicMax(&first[3 + r], u);
        }
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 3 * sizeof(unsigned long long));
    hipMalloc(&first, 6 * sizeof(uint32_t));
    hipMemset(bad, 0, 3 * sizeof(unsigned long long));
    uint32_t init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0, 0, 0};
    hipMemcpy(first, init, sizeof(init), hipMemcpyHostToDevice);
    const uint32_t lo = 1u, hi = 0x7f800000u;  // +denormal_min .. +inf
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, lo, hi - lo + 1u, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("kernel failed\n");
        return 1;
    }
    unsigned long long h[3];
    uint32_t f[6];
    hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    const char* names[3] = {"denormal", "[2^-126, 2^-96)", ">= 2^-96 (incl. +inf)"};
    for (int r = 0; r < 3; r++)
        std::printf("%-24s mismatches %llu (bits 0x%08x .. 0x%08x)\n", names[r], h[r], h[r] ? f[r] : 0u,
                    h[r] ? f[3 + r] : 0u);
    std::printf("checked %u positive floats\n", hi - lo + 1u);
    return 0;
}
