// Calibration: fp32-accurate GEMM on bf16 MFMA by a 3-way bf16 split of each fp32
// operand (x = hi + mid + lo, truncation split: exact for normal fp32), against the
// native f32-input MFMA (v_mfma_f32_32x32x2_f32).
//   part 1: accuracy of one 32x32xK tile vs an fp64 host product (error / sum|a b|)
//   part 2: throughput of an accumulator-chained C -> C layer stack per wave, A
//           fragments streamed from an L2-resident table (the fused kernels' shape)
// hipcc --offload-arch=gfx950 -O3 split_mfma.hip -o /tmp/split_mfma
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);        \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// truncation split of 8 consecutive fp32 values into three packed bf16x8
__device__ __forceinline__ void split8(const float (&x)[8], u32x4 &h, u32x4 &m, u32x4 &l) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t hb[2], mb[2], lb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t xb = __float_as_uint(x[2 * i + j]);
            const float hf = __uint_as_float(xb & 0xffff0000u);
            const float r = x[2 * i + j] - hf;
            const uint32_t rb = __float_as_uint(r);
            const float mf = __uint_as_float(rb & 0xffff0000u);
            const float lf = r - mf;
            hb[j] = xb;
            mb[j] = rb;
            lb[j] = __float_as_uint(lf);
        }
        h[i] = __builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u);
        m[i] = __builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u);
        l[i] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
    }
}

__device__ __forceinline__ f32x16 mf(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// NT terms: 3 (hh, hm, mh), 6 (+ hl, mm, lh), 9 (all); small terms first
template <int NT>
__device__ __forceinline__ f32x16 split_mma(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
    if constexpr (NT >= 9) {
        c = mf(a[2], b[2], c);
        c = mf(a[1], b[2], c);
        c = mf(a[2], b[1], c);
    }
    if constexpr (NT >= 6) {
        c = mf(a[0], b[2], c);
        c = mf(a[1], b[1], c);
        c = mf(a[2], b[0], c);
    }
    c = mf(a[0], b[1], c);
    c = mf(a[1], b[0], c);
    c = mf(a[0], b[0], c);
    return c;
}

// ---------------------------------------------------------------- part 1: accuracy
// A [32][K] row-major, B [K][32] row-major, C [32][32]
template <int MODE>  // 0: f32 MFMA; 3/6/9: split terms
__global__ void tile_kernel(const float *A, const float *B, float *C, int K) {
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    f32x16 acc;
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    if (MODE == 0) {
        for (int k = 0; k < K; k += 2)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * K + k + h], B[(k + h) * 32 + r], acc, 0, 0, 0);
    } else {
        for (int k = 0; k < K; k += 16) {
            float xa[8], xb[8];
            for (int j = 0; j < 8; ++j) {
                xa[j] = A[r * K + k + 8 * h + j];
                xb[j] = B[(k + 8 * h + j) * 32 + r];
            }
            u32x4 a[3], b[3];
            split8(xa, a[0], a[1], a[2]);
            split8(xb, b[0], b[1], b[2]);
            acc = split_mma<MODE>(a, b, acc);
        }
    }
    for (int q = 0; q < 16; ++q) C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = acc[q];
}

static double urand(uint64_t &s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return ((s >> 11) * (1.0 / 9007199254740992.0));
}
static double nrand(uint64_t &s) {
    double u1 = urand(s) + 1e-300, u2 = urand(s);
    return sqrt(-2 * log(u1)) * cos(6.283185307179586 * u2);
}

static void accuracy() {
    const int Ks[] = {32, 128, 512};
    const char *dist[] = {"w~N/sqrtK x relu(N)", "w~N x N", "w~U x U*1e3"};
    for (int d = 0; d < 3; ++d)
        for (int K : Ks) {
            std::vector<float> A(32 * K), B(K * 32);
            uint64_t s = 1234 + K * 7 + d;
            for (auto &v : A) v = d == 0 ? nrand(s) / sqrt((double)K) : d == 1 ? nrand(s) : urand(s) * 2 - 1;
            for (auto &v : B) v = d == 0 ? fmax(nrand(s), 0.0) : d == 1 ? nrand(s) : (urand(s) * 2 - 1) * 1e3;
            float *dA, *dB, *dC;
            CK(hipMalloc(&dA, A.size() * 4));
            CK(hipMalloc(&dB, B.size() * 4));
            CK(hipMalloc(&dC, 32 * 32 * 4));
            CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
            CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
            std::vector<double> ref(1024), den(1024);
            for (int i = 0; i < 32; ++i)
                for (int j = 0; j < 32; ++j) {
                    double a = 0, b = 0;
                    for (int k = 0; k < K; ++k) {
                        a += (double)A[i * K + k] * B[k * 32 + j];
                        b += fabs((double)A[i * K + k] * B[k * 32 + j]);
                    }
                    ref[i * 32 + j] = a;
                    den[i * 32 + j] = b;
                }
            // fp32 sequential fmaf on the host (what a CPU fp32 chain gives)
            double seq_max = 0, seq_mean = 0;
            for (int i = 0; i < 32; ++i)
                for (int j = 0; j < 32; ++j) {
                    float a = 0.f;
                    for (int k = 0; k < K; ++k) a = fmaf(A[i * K + k], B[k * 32 + j], a);
                    const double e = fabs(a - ref[i * 32 + j]) / den[i * 32 + j];
                    seq_max = fmax(seq_max, e);
                    seq_mean += e / 1024;
                }
            printf("%-22s K=%4d  host fmaf   max %.2e mean %.2e\n", dist[d], K, seq_max, seq_mean);
            for (int mode : {0, 3, 6, 9}) {
                if (mode == 0) hipLaunchKernelGGL(tile_kernel<0>, 1, 64, 0, 0, dA, dB, dC, K);
                if (mode == 3) hipLaunchKernelGGL(tile_kernel<3>, 1, 64, 0, 0, dA, dB, dC, K);
                if (mode == 6) hipLaunchKernelGGL(tile_kernel<6>, 1, 64, 0, 0, dA, dB, dC, K);
                if (mode == 9) hipLaunchKernelGGL(tile_kernel<9>, 1, 64, 0, 0, dA, dB, dC, K);
                std::vector<float> C(1024);
                CK(hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost));
                double mx = 0, mean = 0;
                for (int i = 0; i < 1024; ++i) {
                    const double e = fabs(C[i] - ref[i]) / den[i];
                    mx = fmax(mx, e);
                    mean += e / 1024;
                }
                printf("%-22s K=%4d  %-10s  max %.2e mean %.2e\n", dist[d], K,
                       mode == 0 ? "f32 mfma" : mode == 3 ? "bf16x3" : mode == 6 ? "bf16x6" : "bf16x9", mx,
                       mean);
            }
            CK(hipFree(dA));
            CK(hipFree(dB));
            CK(hipFree(dC));
        }
}

// ---------------------------------------------------------------- part 2: throughput
// Each wave runs LAYERS layers of C -> C on its own 32-row tile, weights of layer
// l % NL from a global table; ReLU between layers.
constexpr int NL = 4, LAYERS = 32;

template <int C>
__global__ __launch_bounds__(256, 2) void chain_f32(const float *__restrict__ tbl, float *out, int reps) {
    constexpr int T = C / 32, NS = C / 2;  // k-steps of 2
    const int lane = threadIdx.x & 63;
    f32x16 act[T];
    for (int t = 0; t < T; ++t)
        for (int q = 0; q < 16; ++q) act[t][q] = (lane + q + t) * 1e-3f;
    for (int rep = 0; rep < reps; ++rep)
        for (int l = 0; l < LAYERS; ++l) {
            const float4 *w = reinterpret_cast<const float4 *>(tbl + (size_t)(l % NL) * T * NS * 64);
            f32x16 acc[T];
            for (int t = 0; t < T; ++t)
                for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
            float4 cur[T], nxt[T];
#pragma unroll
            for (int co = 0; co < T; ++co) cur[co] = w[(co * NS / 4) * 64 + lane];
#pragma unroll
            for (int g = 0; g < NS / 4; ++g) {
                if (g + 1 < NS / 4) {
#pragma unroll
                    for (int co = 0; co < T; ++co) nxt[co] = w[(co * NS / 4 + g + 1) * 64 + lane];
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int st = g * 4 + s;
                    const float b = act[st >> 4][st & 15];
#pragma unroll
                    for (int co = 0; co < T; ++co)
                        acc[co] = __builtin_amdgcn_mfma_f32_32x32x2f32((&cur[co].x)[s], b, acc[co], 0, 0, 0);
                }
#pragma unroll
                for (int co = 0; co < T; ++co) cur[co] = nxt[co];
            }
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int q = 0; q < 16; ++q) act[t][q] = fmaxf(acc[t][q], 0.f);
        }
    float s = 0.f;
    for (int t = 0; t < T; ++t)
        for (int q = 0; q < 16; ++q) s += act[t][q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C, int NT>
__global__ __launch_bounds__(256, 2) void chain_split(const u32x4 *__restrict__ tbl, float *out, int reps) {
    constexpr int T = C / 32, NC = C / 16;  // k-chunks of 16
    const int lane = threadIdx.x & 63;
    f32x16 act[T];
    for (int t = 0; t < T; ++t)
        for (int q = 0; q < 16; ++q) act[t][q] = (lane + q + t) * 1e-3f;
    for (int rep = 0; rep < reps; ++rep)
        for (int l = 0; l < LAYERS; ++l) {
            // [co][chunk][piece][lane] u32x4
            const u32x4 *w = tbl + (size_t)(l % NL) * T * NC * 3 * 64;
            f32x16 acc[T];
            for (int t = 0; t < T; ++t)
                for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
            u32x4 cur[T][3], nxt[T][3];
#pragma unroll
            for (int co = 0; co < T; ++co)
#pragma unroll
                for (int p = 0; p < 3; ++p) cur[co][p] = w[((co * NC) * 3 + p) * 64 + lane];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (c + 1 < NC) {
#pragma unroll
                    for (int co = 0; co < T; ++co)
#pragma unroll
                        for (int p = 0; p < 3; ++p) nxt[co][p] = w[((co * NC + c + 1) * 3 + p) * 64 + lane];
                }
                float x[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = act[c >> 1][8 * (c & 1) + j];
                u32x4 b[3];
                split8(x, b[0], b[1], b[2]);
#pragma unroll
                for (int co = 0; co < T; ++co) acc[co] = split_mma<NT>(cur[co], b, acc[co]);
#pragma unroll
                for (int co = 0; co < T; ++co)
#pragma unroll
                    for (int p = 0; p < 3; ++p) cur[co][p] = nxt[co][p];
            }
#pragma unroll
            for (int t = 0; t < T; ++t)
#pragma unroll
                for (int q = 0; q < 16; ++q) act[t][q] = fmaxf(acc[t][q], 0.f);
        }
    float s = 0.f;
    for (int t = 0; t < T; ++t)
        for (int q = 0; q < 16; ++q) s += act[t][q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
static void timeit(const char *name, int C, F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch(1);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    launch(reps);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double waves = 256.0 * 8 * 4;  // blocks * waves per block
    const double flops = 2.0 * 32 * C * C * LAYERS * reps * waves;
    printf("%-16s C=%3d: %.3f ms  %.1f TF (fp32-equivalent)\n", name, C, ms, flops / ms / 1e9);
}

template <int C>
static void throughput() {
    constexpr int T = C / 32;
    float *tf, *out;
    u32x4 *ts;
    const size_t nf = (size_t)NL * T * (C / 2) * 64, ns = (size_t)NL * T * (C / 16) * 3 * 64;
    CK(hipMalloc(&tf, nf * 4));
    CK(hipMalloc(&ts, ns * 16));
    CK(hipMalloc(&out, 256 * 8 * 256 * 4 * 4));
    std::vector<float> hf(nf);
    uint64_t s = 99;
    for (auto &v : hf) v = (urand(s) * 2 - 1) / sqrt((double)C);
    CK(hipMemcpy(tf, hf.data(), nf * 4, hipMemcpyHostToDevice));
    std::vector<uint32_t> hs(ns * 4);
    for (auto &v : hs) {
        const float f = (urand(s) * 2 - 1) / sqrt((double)C);
        const uint32_t b = __builtin_bit_cast(uint32_t, f) >> 16;
        v = b | (b << 16);
    }
    CK(hipMemcpy(ts, hs.data(), ns * 16, hipMemcpyHostToDevice));
    const int blocks = 256 * 8;
    timeit("f32 mfma", C, [&](int r) { hipLaunchKernelGGL(chain_f32<C>, blocks, 256, 0, 0, tf, out, r); });
    timeit("bf16x6", C, [&](int r) { hipLaunchKernelGGL((chain_split<C, 6>), blocks, 256, 0, 0, ts, out, r); });
    timeit("bf16x9", C, [&](int r) { hipLaunchKernelGGL((chain_split<C, 9>), blocks, 256, 0, 0, ts, out, r); });
    timeit("bf16x3", C, [&](int r) { hipLaunchKernelGGL((chain_split<C, 3>), blocks, 256, 0, 0, ts, out, r); });
    CK(hipFree(tf));
    CK(hipFree(ts));
    CK(hipFree(out));
}

int main() {
    accuracy();
    throughput<64>();
    throughput<128>();
    return 0;
}
