// tools/valu_calib.hip -- what the SQ VALU counters mean on gfx950.
//
// One kernel, a dependent-free chain of v_fma_f32 per lane, with only the
// first K lanes of every wave active inside the loop.  Run it under
// rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU ...
// for K = 64, 32, 16, 1: SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64)
// should read K/64 if the pair is the active-lane fraction ("VALUUtilization")
// it is on gfx9.  Build: hipcc --offload-arch=gfx950 -O3 -o valu_calib valu_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void fma_loop(float* out, int iters, int k_active) {
    const int lane = threadIdx.x & 63;
    float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.5f, d = 0.25f;
    if (lane < k_active) {
        for (int i = 0; i < iters; i++) {
            a = fmaf(a, b, c);
            c = fmaf(c, b, d);
            d = fmaf(d, b, a);
            b = fmaf(b, 0.999f, 1e-4f);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + c + d + b;
}

int main(int argc, char** argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 64;
    const int iters = 4096, blocks = 1024, threads = 256;
    float* out;
    if (hipMalloc(&out, sizeof(float) * blocks * threads) != hipSuccess) return 1;
    hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(threads), 0, 0, out, iters, k);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"k_active\": %d, \"waves\": %d, \"fma_per_lane\": %d}\n", k, blocks * threads / 64, iters * 4);
    hipFree(out);
    return 0;
}
