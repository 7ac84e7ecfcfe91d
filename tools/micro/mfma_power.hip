// Calibration: sustained v_mfma_f32_32x32x2_f32 rate and shader clock with constant
// vs random operands (data-dependent power -> clock).  Every wave runs `iters` x 16
// MFMAs over 2 accumulators; operands rotate through 16 registers per lane filled from
// a seeded hash (random) or a constant.  Block 0 wave 0 samples s_memtime (shader
// clock) and s_memrealtime (100 MHz) around the loop.
// hipcc --offload-arch=gfx950 -O3 mfma_power.hip -o /tmp/mfma_power
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float hash_f(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
    return (float)(x & 0xffffff) / 16777216.0f - 0.5f;
}

__global__ __launch_bounds__(256) void k(float *out, uint64_t *clk, int iters, int random) {
    f32x16 acc0, acc1;
    for (int q = 0; q < 16; ++q) { acc0[q] = 0.f; acc1[q] = 0.f; }
    float a[16], b[16];
    const uint32_t seed = blockIdx.x * 256 + threadIdx.x;
    for (int i = 0; i < 16; ++i) {
        a[i] = random ? hash_f(seed * 32 + i) : 1.0f;
        b[i] = random ? hash_f(seed * 32 + 16 + i) : 0.5f;
    }
    uint64_t t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[i], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i + 1], b[i + 1], acc1, 0, 0, 0);
        }
        asm volatile("" : "+v"(a[0]), "+v"(b[0]));
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    float s = 0.f;
    for (int q = 0; q < 16; ++q) s += acc0[q] + acc1[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    float *out;
    uint64_t *clk;
    hipMalloc(&out, 256 * 2 * 256 * sizeof(float));
    hipMalloc(&clk, 2 * sizeof(uint64_t));
    for (int random = 0; random < 2; ++random)
        for (int iters : {500, 5000, 20000}) {
            const int blocks = 256 * 2;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, 10, random);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters, random);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            uint64_t c[2];
            hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
            const double flops = 2.0 * 32 * 32 * 2 * 16 * (double)iters * blocks * 4;
            printf("random=%d iters=%d: %.3f ms, %.1f TF/s, shader clock %.3f GHz\n", random, iters,
                   ms, flops / ms / 1e9, (double)c[0] / ((double)c[1] / 100e6) / 1e9);
        }
    return 0;
}
