// Calibration: v_mfma_f32_32x32x2_f32 issue rate vs independent accumulators per wave
// (NACC) and waves per SIMD.  hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void k(float *out, int iters, float a0, float b0) {
    f32x16 acc[NACC];
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
    float a = a0 + threadIdx.x, b = b0 - threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16 / NACC; ++r)
#pragma unroll
            for (int i = 0; i < NACC; ++i)
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < NACC; ++i)
        for (int q = 0; q < 16; ++q) s += acc[i][q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
void run(int blocks_per_cu) {
    float *out;
    hipMalloc(&out, 256 * 256 * 8 * sizeof(float));
    const int blocks = 256 * blocks_per_cu, iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(256), 0, 0, out, 10, 1.f, 2.f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f, 2.f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 32 * 32 * 2 * 16 * (double)iters * blocks * 4;
    printf("NACC=%d waves/SIMD=%d: %.1f TF/s\n", NACC, blocks_per_cu, flops / ms / 1e9);
    hipFree(out);
}

int main() {
    for (int w = 1; w <= 2; ++w) {
        run<1>(w);
        run<2>(w);
        run<4>(w);
        run<8>(w);
    }
    return 0;
}
