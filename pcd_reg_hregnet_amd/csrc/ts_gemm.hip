// ts_gemm.hip -- tall-skinny fp32 GEMM for the training step's 1x1 convs.
//
// out[r][n] = act(scale[n] * sum_k A[r][k] W'[n][k] + shift[n]) for R in the 10^5..10^6 rows of
// the level-1 / level-2 grouped rows and K, N <= a few hundred channels (the conv forward
// y = x W^T of every train-mode layer and its input gradient dx = dy W, train.py; reference
// layers.py:115-130, 183-198 in .train()).  hreg_gemm stages both operands through LDS tile
// by tile and ran these shapes at 2-3 TB/s; here a workgroup keeps the whole W' column group
// (<= 64 KB) in LDS for its life and its four waves stream 32-row tiles of A straight from
// HBM into MFMA operand registers (one K-group of 64 ahead), with no barrier in the loop.
//
// W' is W [N][K] (w_trans 0) or the transpose of a [K][N] matrix (w_trans 1: the input
// gradient dy W_layer reads the layer's own weight, no transposed copy).
//
// Products: v_mfma_f32_32x32x2_f32 with A as the first operand (tile rows = MFMA rows) and W'
// as the second (output channels = MFMA columns), hreg_gemm's orientation: lane (j, h) holds
// column j of each output tile for rows (q & 3) + 8 (q >> 2) + 4 h, so one dword store
// writes two full 128-B row segments.  k-order: within each 16-deep sub-chunk, lane half h
// takes k = 16 sub + 8 h + s at k-step s -- exactly hreg_gemm's, so every output is the
// same fp32 sum as hreg_gemm's (tests/test_gpu_train.py checks bitwise equality).
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TS_LDS_FLOATS = 16384;  // W' column group: NT * 32 rows x (K16 + 4) floats
constexpr int TS_GRP = 4;             // 16-deep sub-chunks per A load group (k = 64)
constexpr int TS_PRE_FLOATS = 2048;   // (PRE) the input's BatchNorm parameters: K <= 512

// (SEG, r6) A assembled from column segments instead of one matrix: columns [kend[s-1], kend[s])
// are segment s's row r / div[s] (stride ld[s]); every kend a multiple of 16, so a lane's 8-column
// load never straddles two segments.  The descriptor tail's cat([x2 repeated over k rows, x1,
// att_map]) (layers.py:204-206) without materialising it: the same values in the same k order,
// so the same sums as the concatenated matrix.
struct TsSeg {
    const float *base[3];
    int ld[3], div[3], kend[3];
};

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// (PRE, r6) A is the previous layer's pre-BatchNorm output: every A value is replaced on load by
// bn_act(A, mean[k], invstd[k], gamma[k], beta[k], ReLU) -- hreg_bn_apply's arithmetic, so the
// products are those of the materialised activation (train.py _ConvStats)
struct TsPre {
    const float *mean, *invstd, *gamma, *beta;
};

// (OSEG, r6) the output as column segments: columns [nend[s-1], nend[s]) go to segment s's
// matrix (stride ld[s]); every nend a multiple of 32, so an output tile writes one segment (the
// descriptor tail's input gradient straight into its x2 / x1 / att_map blocks)
struct TsOut {
    float *base[3];
    int ld[3], nend[3];
};

// STATS: the train-mode BatchNorm statistics of the output ride along in the epilogue (the
// col_reduce pass over y it replaces): every lane keeps fp64 sums of its column's values and
// squares (exact products) over its rows, in its fixed tile order; the lane halves, then the
// four waves (in order, through LDS) combine, and each workgroup writes its partial
// [blockIdx.x][N][2] for col_finalize (train.hip) to sum over workgroups in order.
template <int NT, bool TAIL, bool FULL, bool STATS = false, bool SEG = false, bool PRE = false, bool OSEG = false>
__global__ __launch_bounds__(256, 2) void ts_gemm_kernel(const float *__restrict__ A, int lda, int R, int K,
                                                         const float *__restrict__ W, int w_trans, int N,
                                                         const float *__restrict__ scale,
                                                         const float *__restrict__ shift, int relu,
                                                         float *__restrict__ out, int ldo,
                                                         double *__restrict__ part = nullptr, TsSeg sg = {},
                                                         TsPre pre = {}, TsOut os = {}) {
    extern __shared__ __attribute__((aligned(16))) float Ws[];
    const int K16 = (K + 15) & ~15, KP = K16 + 4, nsub = K16 / 16;
    const int ngrp = (nsub + TS_GRP - 1) / TS_GRP;
    const int n0 = blockIdx.y * NT * 32;
    constexpr int NR = NT * 32;
    // stage W' [NR][K16] (zero beyond N / K)
    if (!w_trans) {
        for (int i = threadIdx.x; i < NR * (K16 / 4); i += 256) {
            const int nn = i / (K16 / 4), k = (i - nn * (K16 / 4)) * 4;
            const int n = n0 + nn;
            const float4 v = (n < N && k < K) ? ld4(W + (size_t)n * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4 *>(Ws + nn * KP + k) = v;
        }
    } else {
        for (int i = threadIdx.x; i < NR * K16; i += 256) {
            const int k = i / NR, nn = i - k * NR;
            const int n = n0 + nn;
            Ws[nn * KP + k] = (n < N && k < K) ? W[(size_t)k * N + n] : 0.f;
        }
    }
    // the epilogue's shift / scale from LDS (a global load there would make the tile's
    // stores wait for the next group's prefetch: vmcnt counts in order)
    float *Sh = Ws + NR * KP, *Sc = Sh + NR;
    for (int i = threadIdx.x; i < NR; i += 256) {
        const int n = n0 + i;
        Sh[i] = (shift && n < N) ? shift[n] : 0.f;
        if (FULL) Sc[i] = (scale && n < N) ? scale[n] : 1.f;
    }
    // (PRE) the input's BatchNorm parameters per k, past the statistics' partials (zero past K:
    // finite values the zero columns of W' cancel)
    float *Pm = Sh + 2 * NR + (STATS ? 16 * NR : 0);
    if constexpr (PRE) {
        for (int i = threadIdx.x; i < K16; i += 256) {
            const bool ok = i < K;
            Pm[i] = ok ? pre.mean[i] : 0.f;
            Pm[K16 + i] = ok ? pre.invstd[i] : 0.f;
            Pm[2 * K16 + i] = ok ? pre.gamma[i] : 0.f;
            Pm[3 * K16 + i] = ok ? pre.beta[i] : 0.f;
        }
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int ntiles = (R + 31) / 32;
    const int tstride = gridDim.x * 4;
    int t = blockIdx.x * 4 + wave;
    // A through a buffer descriptor: unconditional loads (rows clamped to R - 1; a sub-chunk
    // past the row reads the next row -- finite values the zero columns of W' cancel, masked
    // exactly in the tail sub-chunk -- or, past the buffer, 0), so no load sits in a branch
    // and the waits stay counted
    const uint32_t abytes = (uint32_t)((size_t)R * lda * sizeof(float));
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(A), (short)0, (int)abytes, 0x00020000);
    auto load_group = [&](int tt, int g, float4 (&v)[2 * TS_GRP]) {
        int r = tt * 32 + j;
        r = r < R ? r : R - 1;
        if constexpr (SEG) {
#pragma unroll
            for (int u = 0; u < TS_GRP; ++u) {
                const int k0 = (g * TS_GRP + u) * 16;  // (uniform) sub-chunk -> its segment
                const int s = k0 < sg.kend[0] ? 0 : k0 < sg.kend[1] ? 1 : 2;
                const int kb = s == 0 ? 0 : sg.kend[s - 1];
                const int kk = k0 < K ? k0 - kb + 8 * h : 8 * h;  // (past K: a valid row, masked by W' = 0)
                const float *src = sg.base[s] + (size_t)(r / sg.div[s]) * sg.ld[s] + kk;
                v[2 * u] = *reinterpret_cast<const float4 *>(src);
                v[2 * u + 1] = *reinterpret_cast<const float4 *>(src + 4);
            }
            return;
        }
#pragma unroll
        for (int u = 0; u < TS_GRP; ++u) {
            const int k = (g * TS_GRP + u) * 16 + 8 * h;
            const uint32_t off = (uint32_t)(r * lda + k) * 4u;
            v[2 * u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
            v[2 * u + 1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 16, 0, 0));
        }
    };

    f32x16 acc[NT];
    double st1[NT], st2[NT];
#pragma unroll
    for (int co = 0; co < NT; ++co) st1[co] = st2[co] = 0.0;
    float4 bufA[2 * TS_GRP], bufB[2 * TS_GRP];
    int g = 0;
    // one (tile, group) step: the next step's A into `nx` while this step's (`cu`) MFMAs run
    // (ping-pong buffers, two steps per loop trip: no register copy, so the wait for `nx`
    // falls at its use one step later; past the last tile the prefetch reads a clamped tile)
    auto step = [&](float4 (&cu)[2 * TS_GRP], float4 (&nx)[2 * TS_GRP]) {
        int t2 = t, g2 = g + 1;
        if (g2 == ngrp) {
            g2 = 0;
            t2 += tstride;
        }
        load_group(t2 < ntiles ? t2 : t, g2, nx);
        if (g == 0) {
#pragma unroll
            for (int co = 0; co < NT; ++co)
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[co][q] = 0.f;
        }
#pragma unroll
        for (int u = 0; u < TS_GRP; ++u) {
            const int sub = g * TS_GRP + u;
            if (sub < nsub) {
                float bv[8] = {cu[2 * u].x,     cu[2 * u].y,     cu[2 * u].z,     cu[2 * u].w,
                               cu[2 * u + 1].x, cu[2 * u + 1].y, cu[2 * u + 1].z, cu[2 * u + 1].w};
                if constexpr (PRE) {
                    const float *pk = Pm + sub * 16 + 8 * h;
                    const float4 m0 = ld4(pk), m1 = ld4(pk + 4), i0 = ld4(pk + K16), i1 = ld4(pk + K16 + 4),
                                 g0 = ld4(pk + 2 * K16), g1 = ld4(pk + 2 * K16 + 4), b0 = ld4(pk + 3 * K16),
                                 b1 = ld4(pk + 3 * K16 + 4);
                    const float mv[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
                    const float iv[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
                    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
                    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) bv[e] = bn_act(bv[e], mv[e], iv[e], gv[e], bb[e], 1);
                }
                if (TAIL && sub == nsub - 1) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) bv[e] = sub * 16 + 8 * h + e < K ? bv[e] : 0.f;
                }
                // W' fragments one output tile ahead of their MFMAs
                const float *wr = Ws + j * KP + sub * 16 + 8 * h;
                float4 w0 = ld4(wr), w1 = ld4(wr + 4);
#pragma unroll
                for (int co = 0; co < NT; ++co) {
                    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
                    if (co + 1 < NT) {
                        w0 = ld4(wr + (co + 1) * 32 * KP);
                        w1 = ld4(wr + (co + 1) * 32 * KP + 4);
                    }
#pragma unroll
                    for (int s = 0; s < 8; ++s)
                        acc[co] = __builtin_amdgcn_mfma_f32_32x32x2f32(bv[s], wv[s], acc[co], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (g == ngrp - 1) {
            // lane (j, h), register q: row (q & 3) + 8 (q >> 2) + 4 h of the tile, column j of
            // output tile co -- each dword store instruction writes two 128-B row segments
            // (full rate; 16-B stores of a row-per-lane layout wrote 32-B pieces at ~3 TB/s)
#pragma unroll
            for (int co = 0; co < NT; ++co) {
                const int nl = co * 32 + j, n = n0 + nl;
                float *obase = out;
                int old_ = ldo, ncol = n;
                if constexpr (OSEG) {
                    const int nt0 = n0 + co * 32;  // (uniform) the tile's segment
                    const int sgi = nt0 < os.nend[0] ? 0 : nt0 < os.nend[1] ? 1 : 2;
                    obase = os.base[sgi];
                    old_ = os.ld[sgi];
                    ncol = n - (sgi == 0 ? 0 : os.nend[sgi - 1]);
                }
                if (n < N) {
                    const float sh = Sh[nl];
                    const float sc = FULL ? Sc[nl] : 1.f;
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int r = t * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                        if (r < R) {
                            float v = acc[co][q];
                            if constexpr (FULL) {
                                v = fadd_rn(fmul_rn(v, sc), sh);
                                if (relu) v = fmaxf(v, 0.f);
                            } else {
                                v = fadd_rn(v, sh);
                            }
                            obase[(size_t)r * old_ + ncol] = v;
                            if constexpr (STATS) {
                                const double d = (double)v;
                                st1[co] += d;
                                st2[co] = fma(d, d, st2[co]);
                            }
                        }
                    }
                }
            }
        }
        t = t2;
        g = g2;
    };
    if (t < ntiles) load_group(t, 0, bufA);
    while (t < ntiles) {
        step(bufA, bufB);
        if (t >= ntiles) break;
        step(bufB, bufA);
    }
    if constexpr (STATS) {
        double *red = reinterpret_cast<double *>(Ws + NR * KP + 2 * NR);  // [4 waves][NR][2]
#pragma unroll
        for (int co = 0; co < NT; ++co) {
            const double o1 = __shfl_xor(st1[co], 32), o2 = __shfl_xor(st2[co], 32);
            if (h == 0) {
                red[(wave * NR + co * 32 + j) * 2 + 0] = st1[co] + o1;
                red[(wave * NR + co * 32 + j) * 2 + 1] = st2[co] + o2;
            }
        }
        __syncthreads();
        for (int nl = threadIdx.x; nl < NR; nl += 256) {
            const int n = n0 + nl;
            if (n < N) {
                double a = red[nl * 2], b = red[nl * 2 + 1];
#pragma unroll
                for (int w = 1; w < 4; ++w) {
                    a += red[(w * NR + nl) * 2];
                    b += red[(w * NR + nl) * 2 + 1];
                }
                part[((size_t)blockIdx.x * N + n) * 2 + 0] = a;
                part[((size_t)blockIdx.x * N + n) * 2 + 1] = b;
            }
        }
    }
}

// output tiles per workgroup for this K (W' column group within TS_LDS_FLOATS), 0: unsupported
int ts_nt(int K, int N, bool stats) {
    // (+ the tile's shift / scale, 2 floats per column, and with the statistics their wave
    // partials: 4 waves x 2 doubles = 16 floats per column, as ts_launch reserves them; the
    // plain kernel keeps its historical 8-float margin).  The whole request then stays
    // within TS_LDS_FLOATS (64 KB), which ts_grid_x's workgroups-per-CU count assumes.
    const int KP = ((K + 15) & ~15) + 4 + 2 + (stats ? 16 : 8);
    int nt = TS_LDS_FLOATS / (32 * KP);
    if (nt > 8) nt = 8;
    const int need = (N + 31) / 32;
    nt = nt < need ? nt : need;
    // instantiated: 1, 2, 4, 8 (3 / 6 tiles took 224 / 256+ VGPRs): round up when W' still fits
    const int cap = TS_LDS_FLOATS / (32 * KP);
    if (nt == 3) nt = 4 <= cap ? 4 : 2;
    else if (nt > 4 && nt < 8) nt = 8 <= cap ? 8 : 4;
    return nt;
}

// workgroups along the rows: persistent (tiles assigned statically), so exactly as many as
// fit at once -- three per CU up to 168 VGPRs (<= 4 tiles; 2 with the statistics), else two
int ts_grid_x(int R, int K, int N, bool stats) {
    const int nt = ts_nt(K, N, stats);
    const int gy = (N + nt * 32 - 1) / (nt * 32);
    const int tiles = (R + 31) / 32;
    const int gx = (tiles + 3) / 4;
    const int per_cu = nt >= 8 || (stats && nt >= 4) ? 2 : 3;
    const int cap = 256 * per_cu / gy > 0 ? 256 * per_cu / gy : 1;
    return gx < cap ? gx : cap;
}

}  // namespace

// (train.hip) the statistics' finalisation over S partials [S][C][2] (+ the running update)
int hreg_bn_finalize_stats(const double *part, int S, int R, int C, float eps, float *mean, float *invstd,
                           float *var_unbiased, float momentum, float *running_mean, float *running_var,
                           hipStream_t st);

extern "C" int hreg_ts_gemm_supported(int R, int K, int N, int stats) {
    // (the A extent is addressed through a buffer descriptor: < 2 GB); stats: the budget of
    // hreg_ts_gemm_bn (16 more floats of LDS per column), else the plain kernel's own
    return R > 0 && K > 0 && N > 0 && (K & 3) == 0 && (N & 3) == 0 && ts_nt(K, N, stats != 0) > 0 &&
           (size_t)R * K * sizeof(float) < ((size_t)1 << 31);
}

namespace {

// launch (STATS: the workgroups' statistic partials into part, see ts_gemm_kernel); returns
// the number of workgroups along the rows (the partials' count), or a negative HREG_ERR_*
template <bool STATS, bool SEG = false, bool PRE = false, bool OSEG = false>
int ts_launch(const float *A, int lda, int R, int K, const float *W, int w_trans, int N, const float *scale,
              const float *shift, int relu, float *out, int ldo, double *part, hipStream_t st, TsSeg sg = {},
              TsPre pre = {}, TsOut os = {}) {
    if (!A || !W || !out || R <= 0 || K <= 0 || N <= 0 || lda < K || ldo < N || (K & 3) || (N & 3) ||
        (lda & 3) || (ldo & 3) || ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W) |
                                     reinterpret_cast<uintptr_t>(out)) & 15))
        return -HREG_ERR_INVALID;
    if (SEG && (K & 15)) return -HREG_ERR_INVALID;
    if ((size_t)R * lda * sizeof(float) >= ((size_t)1 << 31)) return -HREG_ERR_UNSUPPORTED;
    const int nt = ts_nt(K, N, STATS);
    if (nt <= 0) return -HREG_ERR_UNSUPPORTED;
    const int gx = ts_grid_x(R, K, N, STATS);
    const int gy = (N + nt * 32 - 1) / (nt * 32);
    const size_t lds0 = ((size_t)nt * 32 * (((K + 15) & ~15) + 4) + 2 * nt * 32 + (STATS ? 16 * nt * 32 : 0)) *
                        sizeof(float);
    if (lds0 > TS_LDS_FLOATS * sizeof(float)) return -HREG_ERR_UNSUPPORTED;  // (ts_nt's budget)
    // (PRE: + the input's 4 x K16 BatchNorm parameters, <= TS_PRE_FLOATS beyond the budget)
    const size_t lds = lds0 + (PRE ? (size_t)4 * ((K + 15) & ~15) * sizeof(float) : 0);
    if (PRE && 4 * ((K + 15) & ~15) > TS_PRE_FLOATS) return -HREG_ERR_UNSUPPORTED;
    const bool tail = (K & 15) != 0, full = scale != nullptr || relu;
    if (STATS && full) return -HREG_ERR_UNSUPPORTED;
#define TS_CASE(NTT, TT, FF)                                                                                   \
    if (nt == NTT && tail == TT && full == FF) {                                                              \
        hipLaunchKernelGGL((ts_gemm_kernel<NTT, TT, FF, STATS, SEG, PRE, OSEG>), dim3(gx, gy), dim3(256), lds, st, A, \
                           lda, R, K, W, w_trans, N, scale, shift, relu, out, ldo, part, sg, pre, os);         \
        if (hipGetLastError() != hipSuccess) return -HREG_ERR_LAUNCH;                                          \
        return gx;                                                                                             \
    }
#define TS_NT_CASE(NTT) TS_CASE(NTT, false, false) TS_CASE(NTT, true, false)                           \
    if constexpr (!STATS) { TS_CASE(NTT, false, true) TS_CASE(NTT, true, true) }
    TS_NT_CASE(1) TS_NT_CASE(2) TS_NT_CASE(4)
    if constexpr (!PRE) { TS_NT_CASE(8) }  // (PRE at 8 tiles spills: <= 4, ts_pre_ok)
#undef TS_NT_CASE
#undef TS_CASE
    return -HREG_ERR_UNSUPPORTED;
}

}  // namespace

extern "C" int hreg_ts_gemm(const float *A, int lda, int R, int K, const float *W, int w_trans, int N,
                            const float *scale, const float *shift, int relu, float *out, int ldo, void *stream) {
    if (R == 0 && A && W && out) return HREG_OK;
    const int rc = ts_launch<false>(A, lda, R, K, W, w_trans, N, scale, shift, relu, out, ldo, nullptr,
                                    as_stream(stream));
    return rc < 0 ? -rc : HREG_OK;
}

// hreg_ts_gemm (no scale / shift / activation) with the output [R][N] split by columns into up to
// three matrices: columns [0, n1) -> out0 (stride ld0), [n1, n2) -> out1, [n2, N) -> out2; n1, n2
// multiples of 32 (n2 = N: two segments).  The same values as hreg_ts_gemm's (r6: the descriptor
// tail's input gradient written straight into its x2-block / x1 / att_map gradients).
extern "C" int hreg_ts_gemm_split_out(const float *A, int lda, int R, int K, const float *W, int w_trans, int N,
                                      float *out0, int ld0, int n1, float *out1, int ld1, int n2, float *out2,
                                      int ld2, void *stream) {
    if (!out0 || !out1 || n1 <= 0 || n2 < n1 || n2 > N || (n1 & 31) || ((n2 & 31) && n2 != N) ||
        (n2 < N && !out2) || ld0 < n1 || ld1 < n2 - n1 || (n2 < N && ld2 < N - n2) || ((ld0 | ld1 | ld2) & 3) ||
        ((reinterpret_cast<uintptr_t>(out0) | reinterpret_cast<uintptr_t>(out1) | reinterpret_cast<uintptr_t>(out2)) & 15))
        return HREG_ERR_INVALID;
    if (R == 0 && A && W) return HREG_OK;
    TsOut os;
    os.base[0] = out0; os.ld[0] = ld0; os.nend[0] = n1;
    os.base[1] = out1; os.ld[1] = ld1; os.nend[1] = n2;
    os.base[2] = out2 ? out2 : out1; os.ld[2] = out2 ? ld2 : ld1; os.nend[2] = N;
    // (out / ldo: the validity checks of the plain form; the tiles are written through os)
    const int rc = ts_launch<false, false, false, true>(A, lda, R, K, W, w_trans, N, nullptr, nullptr, 0, out0, N,
                                                        nullptr, as_stream(stream), {}, {}, os);
    return rc < 0 ? -rc : HREG_OK;
}

extern "C" size_t hreg_ts_gemm_bn_ws_bytes(int R, int K, int N) {
    if (R <= 0 || K <= 0 || N <= 0 || ts_nt(K, N, true) <= 0) return 0;
    return (size_t)ts_grid_x(R, K, N, true) * N * 2 * sizeof(double);
}

extern "C" int hreg_ts_gemm_bn(const float *A, int lda, int R, int K, const float *W, int w_trans, int N,
                               const float *shift, float *out, int ldo, float eps, float momentum, void *ws,
                               float *mean, float *invstd, float *var_unbiased, float *running_mean,
                               float *running_var, void *stream) {
    if (!ws || !mean || !invstd || R <= 0 || ((running_mean == nullptr) != (running_var == nullptr)) ||
        (running_mean && !var_unbiased))
        return HREG_ERR_INVALID;
    hipStream_t st = as_stream(stream);
    const int S = ts_launch<true>(A, lda, R, K, W, w_trans, N, nullptr, shift, 0, out, ldo,
                                  static_cast<double *>(ws), st);
    if (S < 0) return -S;
    return hreg_bn_finalize_stats(static_cast<const double *>(ws), S, R, N, eps, mean, invstd, var_unbiased,
                                  momentum, running_mean, running_var, st);
}

// hreg_ts_gemm_bn with A = the previous layer's pre-BatchNorm output y_in [R][K]: every value of
// A enters as bn_act(y_in, pre_mean, pre_invstd, pre_gamma, pre_beta, pre_relu) (hreg_bn_apply's
// arithmetic), so out, the statistics and the running update are those of hreg_bn_apply followed
// by hreg_ts_gemm_bn, without the activation's write and read (r6, train.py _ConvStats).
extern "C" int hreg_ts_gemm_bn_pre(const float *A, int lda, int R, int K, const float *W, int N,
                                   const float *shift, float *out, int ldo, float eps, float momentum, void *ws,
                                   float *mean, float *invstd, float *var_unbiased, float *running_mean,
                                   float *running_var, const float *pre_mean, const float *pre_invstd,
                                   const float *pre_gamma, const float *pre_beta, int pre_relu, void *stream) {
    if (!ws || !mean || !invstd || R <= 0 || ((running_mean == nullptr) != (running_var == nullptr)) ||
        (running_mean && !var_unbiased) || !pre_mean || !pre_invstd || !pre_gamma || !pre_beta)
        return HREG_ERR_INVALID;
    if (!pre_relu) return HREG_ERR_UNSUPPORTED;  // (the chains' activations are all ReLU)
    hipStream_t st = as_stream(stream);
    TsPre pre{pre_mean, pre_invstd, pre_gamma, pre_beta};
    const int S = ts_launch<true, false, true>(A, lda, R, K, W, 0, N, nullptr, shift, 0, out, ldo,
                                               static_cast<double *>(ws), st, {}, pre);
    if (S < 0) return -S;
    return hreg_bn_finalize_stats(static_cast<const double *>(ws), S, R, N, eps, mean, invstd, var_unbiased,
                                  momentum, running_mean, running_var, st);
}

extern "C" int hreg_ts_gemm_pre_supported(int R, int K, int N) {
    return hreg_ts_gemm_supported(R, K, N, 1) && 4 * ((K + 15) & ~15) <= TS_PRE_FLOATS && ts_nt(K, N, true) <= 4;
}

// hreg_ts_gemm_bn over the descriptor tail's rows without the concatenation (r6): A = cat([x2
// repeated over the k rows of each group, x1, att]) (layers.py:204-206), x2 [R/k][C1], x1 [R][C1],
// att [R][Ca]; C1, Ca multiples of 16.  The same sums as hreg_ts_gemm_bn on the materialised
// [R][2 C1 + Ca] matrix (the same values in the same k order).
extern "C" int hreg_ts_gemm_bn_tail(const float *x2, int k, const float *x1, int C1, const float *att, int Ca,
                                    int R, const float *W, int N, const float *shift, float *out, int ldo,
                                    float eps, float momentum, void *ws, float *mean, float *invstd,
                                    float *var_unbiased, float *running_mean, float *running_var, void *stream) {
    if (!x2 || !x1 || !att || !ws || !mean || !invstd || R <= 0 || k <= 0 || R % k || (C1 & 15) || (Ca & 15) ||
        ((running_mean == nullptr) != (running_var == nullptr)) || (running_mean && !var_unbiased) ||
        ((reinterpret_cast<uintptr_t>(x2) | reinterpret_cast<uintptr_t>(x1) | reinterpret_cast<uintptr_t>(att)) & 15))
        return HREG_ERR_INVALID;
    const int K = 2 * C1 + Ca;
    TsSeg sg;
    sg.base[0] = x2; sg.ld[0] = C1; sg.div[0] = k; sg.kend[0] = C1;
    sg.base[1] = x1; sg.ld[1] = C1; sg.div[1] = 1; sg.kend[1] = 2 * C1;
    sg.base[2] = att; sg.ld[2] = Ca; sg.div[2] = 1; sg.kend[2] = K;
    hipStream_t st = as_stream(stream);
    // (A / lda: the validity checks of the plain form; the segments are read through sg)
    const int S = ts_launch<true, true>(x1, K, R, K, W, 0, N, nullptr, shift, 0, out, ldo, static_cast<double *>(ws),
                                        st, sg);
    if (S < 0) return -S;
    return hreg_bn_finalize_stats(static_cast<const double *>(ws), S, R, N, eps, mean, invstd, var_unbiased,
                                  momentum, running_mean, running_var, st);
}
