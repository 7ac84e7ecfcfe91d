// pk_hazard.hip -- which instruction pairing corrupts packed-fp32 results on gfx950?
//
// The bf16x6 kernels built WITH packed fp32 VALU ops (v_pk_add_f32 / v_pk_mul_f32) gave
// nondeterministic wrong values whenever two waves shared a SIMD.  In
// those builds (llvm-objdump of group_l1_6.hip) the pairings that occur ONLY with packed
// ops are: a v_mov_b32_dpp immediately (0 or 1 wait states) followed by a v_pk_add_f32
// that reads its result as the high half of a register pair; a plain v_mov_b32 into one
// half of a pair right before the v_pk op; a v_pk op's result read one state later.
// Each mode below runs one of those pairings in inline asm (so the compiler cannot pad
// it), many times, in waves that share SIMDs with MFMA-heavy waves, and counts the
// lanes whose result differs from the plain-VALU answer.
//
// modes: 0 dpp-mov -> pk (0 states)      1 dpp-mov, s_nop 1, pk
//        2 v_mov -> pk (0 states)        3 pk -> v_add of the high half (0 states)
//        4 dpp-mov -> pk (0 states), no MFMA waves beside it
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/pk_hazard.hip -o tools/micro/pk_hazard
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>
__device__ __forceinline__ float probe(float x, float y) {
    float r;
    if constexpr (MODE == 0 || MODE == 4) {
        // v3 <- dpp(v1) (lane ^ 1 within the quad); v[4:5] = v[0:1] + v[2:3]; r = v5 = y + x'
        asm volatile(
            "v_mov_b32 v0, %1\n v_mov_b32 v1, %2\n v_mov_b32 v2, %1\n s_nop 4\n"
            "v_mov_b32_dpp v3, v1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_add_f32 v[4:5], v[0:1], v[2:3]\n s_nop 4\n v_mov_b32 %0, v5\n"
            : "=v"(r) : "v"(x), "v"(y) : "v0", "v1", "v2", "v3", "v4", "v5");
    } else if constexpr (MODE == 1) {
        asm volatile(
            "v_mov_b32 v0, %1\n v_mov_b32 v1, %2\n v_mov_b32 v2, %1\n s_nop 4\n"
            "v_mov_b32_dpp v3, v1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "s_nop 1\n v_pk_add_f32 v[4:5], v[0:1], v[2:3]\n s_nop 4\n v_mov_b32 %0, v5\n"
            : "=v"(r) : "v"(x), "v"(y) : "v0", "v1", "v2", "v3", "v4", "v5");
    } else if constexpr (MODE == 2) {
        // v3 <- y * 1 written by a plain VALU right before the pk read; r = v5 = y + y
        asm volatile(
            "v_mov_b32 v0, %1\n v_mov_b32 v1, %2\n v_mov_b32 v2, %1\n s_nop 4\n"
            "v_mov_b32 v3, v1\n v_pk_add_f32 v[4:5], v[0:1], v[2:3]\n s_nop 4\n v_mov_b32 %0, v5\n"
            : "=v"(r) : "v"(x), "v"(y) : "v0", "v1", "v2", "v3", "v4", "v5");
    } else {
        // v[4:5] = v[0:1] + v[2:3]; r = v5 + v5 read immediately
        asm volatile(
            "v_mov_b32 v0, %1\n v_mov_b32 v1, %2\n v_mov_b32 v2, %1\n v_mov_b32 v3, %2\n s_nop 4\n"
            "v_pk_add_f32 v[4:5], v[0:1], v[2:3]\n v_add_f32 %0, v5, v5\n s_nop 4\n"
            : "=v"(r) : "v"(x), "v"(y) : "v0", "v1", "v2", "v3", "v4", "v5");
    }
    return r;
}

template <int MODE>
__device__ __forceinline__ float expect(float x, float y, int lane) {
    if constexpr (MODE == 0 || MODE == 1 || MODE == 4) {
        const float yn = __shfl_xor(y, 1);
        return y + yn;
    } else if constexpr (MODE == 2) {
        return y + y;
    } else {
        return (y + y) + (y + y);
    }
}

// even waves probe, odd waves run MFMAs (both on every SIMD: 8 waves per 512-thread block,
// 2 blocks per CU)
template <int MODE>
__global__ __launch_bounds__(512) void kern(int iters, unsigned *bad, float *sink) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float x = 1.0f + 0.001f * (float)(blockIdx.x * 512 + threadIdx.x);
    float y = 3.0f + 0.01f * (float)lane + 0.1f * (float)w;
    unsigned nbad = 0;
    if ((w & 1) == 0 || MODE == 4) {
        for (int i = 0; i < iters; ++i) {
            const float r = probe<MODE>(x, y);
            const float e = expect<MODE>(x, y, lane);
            nbad += (r != e) ? 1u : 0u;
            y = y + 0.5f;
            if (y > 1000.f) y = 3.0f + 0.01f * (float)lane;
        }
    } else {
        f32x16 acc = {};
        bf16x8 a, b;
        for (int q = 0; q < 8; ++q) { a[q] = (short)(0x3f80 + lane); b[q] = (short)(0x3f80 + q); }
        for (int i = 0; i < iters; ++i)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        float s = 0.f;
        for (int q = 0; q < 16; ++q) s += acc[q];
        sink[blockIdx.x * 512 + threadIdx.x] = s;
    }
    if (nbad) atomicAdd(bad, nbad);
}

template <int MODE>
unsigned run(int blocks, int iters, unsigned *dbad, float *sink) {
    hipMemset(dbad, 0, 4);
    hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(512), 0, 0, iters, dbad, sink);
    unsigned h = 0;
    hipMemcpy(&h, dbad, 4, hipMemcpyDeviceToHost);
    return h;
}

int main(int argc, char **argv) {
    const int blocks = 512, iters = argc > 1 ? atoi(argv[1]) : 20000;
    unsigned *dbad;
    float *sink;
    hipMalloc(&dbad, 4);
    hipMalloc(&sink, (size_t)blocks * 512 * 4);
    const unsigned long probes = (unsigned long)blocks * 4 * 64 * iters;
    printf("mode 0 dpp-mov -> pk, 0 states   : %u bad of %lu\n", run<0>(blocks, iters, dbad, sink), probes);
    printf("mode 1 dpp-mov, s_nop 1, pk      : %u bad of %lu\n", run<1>(blocks, iters, dbad, sink), probes);
    printf("mode 2 v_mov -> pk, 0 states     : %u bad of %lu\n", run<2>(blocks, iters, dbad, sink), probes);
    printf("mode 3 pk -> v_add, 0 states     : %u bad of %lu\n", run<3>(blocks, iters, dbad, sink), probes);
    printf("mode 4 dpp-mov -> pk, no MFMA    : %u bad of %lu\n", run<4>(blocks, iters, dbad, sink), 2 * probes);
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
