// train.hip -- training-step building blocks.
//
// The reference trains with train-mode BatchNorm (batch statistics) after every 1x1
// conv (layers.py:115-130, 183-198, 246-268, 417-431; train/train_reg_v0.py:241-296)
// and Adam (train_reg_v0.py:246).  Here:
//   column statistics   mean / invstd / unbiased var of y [R][C] per channel
//   bn_apply            out = act(gamma * (y - mean) * invstd + beta)
//   bn_backward         dgamma, dbeta and dy of (BN + optional ReLU)
//   col_sum             sum over rows (conv bias gradients)
//   gemm_tn             out[n][k] = sum_r A[r][n] B[r][k] (weight gradients dW = dY^T X)
//   transpose           W [N][K] -> W^T (the input gradient dX = dY W runs on hreg_gemm)
//   adam_step           torch.optim.Adam's update (L2 weight decay 0, amsgrad off)
//   bn_running_update   running_mean / running_var momentum update
// Every reduction over rows is split over workgroups with partial results in a
// caller workspace and summed in a fixed order afterwards: no atomics, the same bits
// every run (the reference's cuDNN BN / GEMM backward are not deterministic).
#include "common.h"

namespace {

constexpr int CR_THREADS = 256;  // column lanes x row lanes (column width 16, 32 or 64)

// column width of a col_reduce workgroup: the smallest of 16 / 32 / 64 covering C, so
// that narrow activations (C = 32 at level 1) keep every lane busy
inline int cr_width_log2(int C) { return C <= 16 ? 4 : (C <= 32 ? 5 : 6); }

// per-column sums over rows [r0, r1): MODE 0: (y, y^2); MODE 1: (g, g*xhat) with
// g = dout * [out > 0 if relu], xhat = (y - mean) * invstd; MODE 2: (x, 0).
// double accumulators (the variance is E[y^2] - E[y]^2); row lanes combined in order.
// MK (MODE 1): the ReLU mask -- 0 none, 1 from out, 2 recomputed from y (compile-time, so
// the batched loads carry no branches)
template <int MODE, int MK = 0>
__global__ __launch_bounds__(CR_THREADS) void col_reduce_kernel(
    const float *__restrict__ x, const float *__restrict__ out, const float *__restrict__ y,
    const float *__restrict__ mean, const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, int relu, int R, int C, int rows_per_split, int cw_log2,
    double *__restrict__ partial) {
    __shared__ double s0[CR_THREADS], s1[CR_THREADS];
    const int cw = 1 << cw_log2, nrl = CR_THREADS >> cw_log2;
    const int cl = threadIdx.x & (cw - 1), rl = threadIdx.x >> cw_log2;
    const int c = blockIdx.x * cw + cl;
    const int r0 = blockIdx.y * rows_per_split;
    const int r1 = min(R, r0 + rows_per_split);
    double a = 0.0, b = 0.0;
    if (c < C) {
        float mu = 0.f, is = 0.f, ga = 0.f, be = 0.f;
        if (MODE == 1) {
            mu = mean[c];
            is = invstd[c];
            if (relu && !out) { ga = gamma[c]; be = beta[c]; }
        }
        int r = r0 + rl;
        if constexpr (MODE == 1) {
            // eight rows' loads issued before their (in-order) accumulation: the loop body's
            // two streams and the mask branch otherwise leave one load in flight per wave
            for (; r + 7 * nrl < r1; r += 8 * nrl) {
                float gv[8], yv[8], ov[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const size_t i = (size_t)(r + u * nrl) * C + c;
                    gv[u] = x[i];
                    yv[u] = y[i];
                    ov[u] = MK == 1 ? out[i] : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    float g = gv[u];
                    const float xh = fmul_rn(fsub_rn(yv[u], mu), is);
                    if (MK != 0) {
                        const bool on = MK == 2 ? fadd_rn(fmul_rn(xh, ga), be) > 0.f : ov[u] > 0.f;
                        if (!on) g = 0.f;
                    }
                    a += (double)g;
                    b += (double)g * (double)xh;
                }
            }
        }
#pragma unroll 4
        for (; r < r1; r += nrl) {
            const size_t i = (size_t)r * C + c;
            if (MODE == 0) {
                const double v = x[i];
                a += v;
                b += v * v;
            } else if (MODE == 1) {
                float g = x[i];
                const float xh = fmul_rn(fsub_rn(y[i], mu), is);
                if (relu) {
                    // the forward's ReLU mask: out > 0, or recomputed bit-identically
                    // from y as bn_apply computed out (no third stream to read)
                    const bool on = out ? out[i] > 0.f : fadd_rn(fmul_rn(xh, ga), be) > 0.f;
                    if (!on) g = 0.f;
                }
                a += (double)g;
                b += (double)g * (double)xh;
            } else {
                a += (double)x[i];
            }
        }
    }
    s0[threadIdx.x] = a;
    s1[threadIdx.x] = b;
    __syncthreads();
    if (rl == 0 && c < C) {
        double ta = 0.0, tb = 0.0;
        for (int q = 0; q < nrl; ++q) {
            ta += s0[q * cw + cl];
            tb += s1[q * cw + cl];
        }
        partial[((size_t)blockIdx.y * C + c) * 2 + 0] = ta;
        partial[((size_t)blockIdx.y * C + c) * 2 + 1] = tb;
    }
}

// column totals over the splits (8 columns x 32 split lanes per workgroup: lane l sums
// splits l, l+32, ... in order, then the 32 lanes in order), then MODE's finalisation
constexpr int FIN_COLS = 8, FIN_LANES = 32;

// acc0 / acc1 (MODE 1, 2; optional): the totals are also added to these (a parameter's
// .grad accumulating over its uses, as autograd's accumulation would: one fp32 add each)
// MODE 0: acc0 / acc1 (optional) = running mean / var, updated with `momentum` as
// bn_running_kernel does (from the fp32 mean and unbiased variance just written)
template <int MODE>
__global__ __launch_bounds__(FIN_COLS * FIN_LANES) void col_finalize_kernel(
    const double *__restrict__ partial, int S, int R, int C, float eps, float *__restrict__ o0,
    float *__restrict__ o1, float *__restrict__ o2, float *__restrict__ acc0 = nullptr,
    float *__restrict__ acc1 = nullptr, float momentum = 0.f) {
    __shared__ double s0[FIN_COLS * FIN_LANES], s1[FIN_COLS * FIN_LANES];
    const int cl = threadIdx.x % FIN_COLS, sl = threadIdx.x / FIN_COLS;
    const int c = blockIdx.x * FIN_COLS + cl;
    double a = 0.0, b = 0.0;
    if (c < C) {
#pragma unroll 4
        for (int s = sl; s < S; s += FIN_LANES) {
            a += partial[((size_t)s * C + c) * 2 + 0];
            b += partial[((size_t)s * C + c) * 2 + 1];
        }
    }
    s0[threadIdx.x] = a;
    s1[threadIdx.x] = b;
    __syncthreads();
    if (sl != 0 || c >= C) return;
    a = 0.0;
    b = 0.0;
    for (int q = 0; q < FIN_LANES; ++q) {
        a += s0[q * FIN_COLS + cl];
        b += s1[q * FIN_COLS + cl];
    }
    if (MODE == 0) {
        // mean, invstd (biased variance, used to normalise), unbiased variance (running stat)
        const double m = a / R;
        double var = b / R - m * m;
        if (var < 0.0) var = 0.0;
        o0[c] = (float)m;
        o1[c] = (float)(1.0 / sqrt(var + (double)eps));
        const float vu = (float)(R > 1 ? var * R / (R - 1) : var);
        if (o2) o2[c] = vu;
        if (acc0) {
            acc0[c] = fadd_rn(fmul_rn(1.f - momentum, acc0[c]), fmul_rn(momentum, (float)m));
            acc1[c] = fadd_rn(fmul_rn(1.f - momentum, acc1[c]), fmul_rn(momentum, vu));
        }
    } else if (MODE == 1) {
        o0[c] = (float)b;  // dgamma = sum g * xhat
        o1[c] = (float)a;  // dbeta = sum g
        if (acc0) acc0[c] = fadd_rn(acc0[c], (float)b);
        if (acc1) acc1[c] = fadd_rn(acc1[c], (float)a);
    } else {
        if (o0) o0[c] = (float)a;
        if (acc0) acc0[c] = fadd_rn(acc0[c], (float)a);
    }
}

// bn_apply / bn_backward on float4 groups of 4 channels (C % 4 == 0, C <= BN4_MAXC: every
// layer of the path), 32-bit indexing, the per-channel parameters staged in LDS (one
// ds_read_b128 per parameter and float4 instead of 4 scattered global loads); the
// per-element arithmetic of the scalar kernels (same results)
constexpr int BN4_MAXC = 512;

template <int NP>
__device__ __forceinline__ void stage_params(float4 (*sp)[BN4_MAXC / 4], const float *const (&src)[NP], int C4) {
    for (int k = threadIdx.x; k < NP * C4; k += blockDim.x) {
        const int a = k / C4, c4 = k - a * C4;
        const float *p = src[a] + 4 * c4;
        sp[a][c4] = make_float4(p[0], p[1], p[2], p[3]);
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void bn_apply4_kernel(const float4 *__restrict__ y, const float *__restrict__ mean,
                                                        const float *__restrict__ invstd,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta, int relu, int total4,
                                                        int C4, float4 *__restrict__ out) {
    __shared__ float4 sp[4][BN4_MAXC / 4];
    stage_params<4>(sp, {mean, invstd, gamma, beta}, C4);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
        const int c4 = i % C4;
        const float4 yv = y[i], mu = sp[0][c4], is = sp[1][c4], ga = sp[2][c4], be = sp[3][c4];
        const float *yp = &yv.x, *mp = &mu.x, *ip = &is.x, *gp = &ga.x, *bp = &be.x;
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = bn_act(yp[u], mp[u], ip[u], gp[u], bp[u], relu);
        out[i] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

__global__ __launch_bounds__(256) void bn_backward4_kernel(
    const float4 *__restrict__ dout, const float4 *__restrict__ out, const float4 *__restrict__ y,
    const float *__restrict__ mean, const float *__restrict__ invstd, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ dgamma, const float *__restrict__ dbeta, int relu,
    int total4, int R, int C4, float4 *__restrict__ dy) {
    __shared__ float4 sp[6][BN4_MAXC / 4];
    const float *zero_beta = beta ? beta : mean;  // (beta is only read for the recomputed mask)
    stage_params<6>(sp, {mean, invstd, gamma, zero_beta, dgamma, dbeta}, C4);
    const float invR = 1.0f / (float)R;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += gridDim.x * blockDim.x) {
        const int c4 = i % C4;
        const float4 gv4 = dout[i], yv4 = y[i];
        const float4 ov4 = relu && out ? out[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 mu = sp[0][c4], is = sp[1][c4], ga = sp[2][c4], be = sp[3][c4], dg = sp[4][c4],
                     db = sp[5][c4];
        const float *gp = &gv4.x, *yp = &yv4.x, *op = &ov4.x, *mp = &mu.x, *ip = &is.x, *gap = &ga.x,
                    *bp = &be.x, *dgp = &dg.x, *dbp = &db.x;
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float g = gp[u];
            const float xh = fmul_rn(fsub_rn(yp[u], mp[u]), ip[u]);
            if (relu && !(out ? op[u] > 0.f : fadd_rn(fmul_rn(xh, gap[u]), bp[u]) > 0.f)) g = 0.f;
            const float t = fsub_rn(fsub_rn(g, fmul_rn(dbp[u], invR)), fmul_rn(xh, fmul_rn(dgp[u], invR)));
            o[u] = fmul_rn(fmul_rn(t, ip[u]), gap[u]);
        }
        dy[i] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

__global__ void bn_apply_kernel(const float *__restrict__ y, const float *__restrict__ mean,
                                const float *__restrict__ invstd, const float *__restrict__ gamma,
                                const float *__restrict__ beta, int relu, size_t total, int C,
                                float *__restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        out[i] = bn_act(y[i], mean[c], invstd[c], gamma[c], beta[c], relu);
    }
}

// dy = gamma * invstd * (g - dbeta / R - xhat * dgamma / R)
__global__ void bn_backward_kernel(const float *__restrict__ dout, const float *__restrict__ out,
                                   const float *__restrict__ y, const float *__restrict__ mean,
                                   const float *__restrict__ invstd, const float *__restrict__ gamma,
                                   const float *__restrict__ beta, const float *__restrict__ dgamma,
                                   const float *__restrict__ dbeta, int relu, size_t total, int R, int C,
                                   float *__restrict__ dy) {
    const float invR = 1.0f / (float)R;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        float g = dout[i];
        const float xh = fmul_rn(fsub_rn(y[i], mean[c]), invstd[c]);
        if (relu && !(out ? out[i] > 0.f : fadd_rn(fmul_rn(xh, gamma[c]), beta[c]) > 0.f)) g = 0.f;
        const float t = fsub_rn(fsub_rn(g, fmul_rn(dbeta[c], invR)), fmul_rn(xh, fmul_rn(dgamma[c], invR)));
        dy[i] = fmul_rn(fmul_rn(t, invstd[c]), gamma[c]);
    }
}

__global__ void bn_running_kernel(const float *__restrict__ mean, const float *__restrict__ var_unb,
                                  int C, float momentum, float *__restrict__ rmean,
                                  float *__restrict__ rvar) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    rmean[c] = fadd_rn(fmul_rn(1.f - momentum, rmean[c]), fmul_rn(momentum, mean[c]));
    rvar[c] = fadd_rn(fmul_rn(1.f - momentum, rvar[c]), fmul_rn(momentum, var_unb[c]));
}

// ---------------------------------------------------------------- gemm_tn
// out[n][k] = sum_r A[r][n] * B[r][k] (weight gradients: tall, skinny operands, HBM-bound).
// A workgroup owns a (32 TNN) x (32 TNK) output tile (TNN, TNK in {1, 2}: no MFMAs on tiles
// past N / K) and a range of rows; each of its 4 waves keeps the tile in TNN x TNK
// v_mfma_f32_32x32x2_f32 accumulators and takes every 4th block of 16 rows, loading its
// operands straight from global memory: at k-step s lane (h, j) needs A[r][n0 + j (+32)] and
// B[r][k0 + j (+32)] with r = 2s + h, so each load instruction reads two 128-byte row
// segments and no LDS staging or barrier sits in the loop.  The next block's operands load
// while this block's MFMAs run (ping-pong registers); loads go through buffer descriptors
// with no bounds tests -- a split's blocks lie inside its rows (splits are multiples of 64
// rows), rows past R read 0, and columns past N / K only feed accumulator entries that are
// never stored.  The waves' tiles are added in wave order through LDS at the end; split z of
// the rows writes ws[z][N][K] and tn_reduce_kernel sums the splits in order (same bits every
// run, and the same sums as the unpipelined form).
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int TN_ROWS = 64;  // rows per workgroup iteration (16 per wave)

template <int TNN, int TNK>
__global__ __launch_bounds__(256) void gemm_tn_kernel(const float *__restrict__ A, int lda,
                                                      const float *__restrict__ Bm, int ldb, int R,
                                                      int N, int K, int rows_per_split,
                                                      float *__restrict__ ws) {
    __shared__ float red[3][(32 * TNN) * (32 * TNK)];
    constexpr int TW = 32 * TNK;  // tile width (k)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int n0 = blockIdx.x * 32 * TNN, k0 = blockIdx.y * TW;
    const int r0 = blockIdx.z * rows_per_split;
    const int r1 = min(R, r0 + rows_per_split);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(A), (short)0,
                                                      (int)((size_t)R * lda * sizeof(float)), 0x00020000);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Bm), (short)0,
                                                      (int)((size_t)R * ldb * sizeof(float)), 0x00020000);
    f32x16 acc[TNN][TNK];
#pragma unroll
    for (int a = 0; a < TNN; ++a)
#pragma unroll
        for (int b = 0; b < TNK; ++b)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;
    typedef float Blk[TNN + TNK][8];
    auto load = [&](int base, Blk &v) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const uint32_t r = (uint32_t)(base + 2 * s + h);
#pragma unroll
            for (int a = 0; a < TNN; ++a)
                v[a][s] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(ra, (r * (uint32_t)lda + n0 + 32 * a + j) * 4u, 0, 0));
#pragma unroll
            for (int b = 0; b < TNK; ++b)
                v[TNN + b][s] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rb, (r * (uint32_t)ldb + k0 + 32 * b + j) * 4u, 0, 0));
        }
    };
    auto mma = [&](const Blk &v) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int a = 0; a < TNN; ++a)
#pragma unroll
                for (int b = 0; b < TNK; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(v[a][s], v[TNN + b][s], acc[a][b], 0, 0, 0);
    };
    // blocks in pairs, no exit between them (a mid-loop exit made the compiler keep two copies
    // of the accumulators): an odd count's last partner block is zeroed, adding 0 * 0 (the
    // prefetch past the split's last block reads rows that are never used, or 0 past R)
    Blk p0, p1;
    const int base0 = r0 + 16 * w;
    const int nblk = base0 < r1 ? (r1 - base0 + TN_ROWS - 1) / TN_ROWS : 0;
    if (nblk) load(base0, p0);
    for (int i = 0; i < nblk; i += 2) {
        load(base0 + (i + 1) * TN_ROWS, p1);
        mma(p0);
        load(base0 + (i + 2) * TN_ROWS, p0);
        if (i + 1 >= nblk) {
#pragma unroll
            for (int c = 0; c < TNN + TNK; ++c)
#pragma unroll
                for (int s = 0; s < 8; ++s) p1[c][s] = 0.f;
        }
        mma(p1);
    }
    // acc[a][b][q]: tile row n = 32 a + (q&3) + 8(q>>2) + 4h, column k = 32 b + j
    if (w > 0) {
        float *o = red[w - 1];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int n = (q & 3) + 8 * (q >> 2) + 4 * h;
#pragma unroll
            for (int a = 0; a < TNN; ++a)
#pragma unroll
                for (int b = 0; b < TNK; ++b) o[(32 * a + n) * TW + 32 * b + j] = acc[a][b][q];
        }
    }
    __syncthreads();
    if (w != 0) return;
    float *o = ws + (size_t)blockIdx.z * N * K;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int n = (q & 3) + 8 * (q >> 2) + 4 * h;
#pragma unroll
        for (int a = 0; a < TNN; ++a)
#pragma unroll
            for (int b = 0; b < TNK; ++b) {
                const int nn = 32 * a + n, kk = 32 * b + j;
                float v = acc[a][b][q];
                v = fadd_rn(v, red[0][nn * TW + kk]);
                v = fadd_rn(v, red[1][nn * TW + kk]);
                v = fadd_rn(v, red[2][nn * TW + kk]);
                if (n0 + nn < N && k0 + kk < K) o[(size_t)(n0 + nn) * K + k0 + kk] = v;
            }
    }
}

// gemm_tn_kernel with the operands staged through LDS (r6): each 64-row step of a workgroup
// is loaded by all 256 threads as 16-byte row segments (4 + 4 buffer_load_dwordx4 per thread
// at 64 x 64 instead of 32 + 32 dword loads per lane, which kept the weight-gradient GEMMs at
// ~2.4 TB/s), one step ahead in registers; each wave then reads its 16 rows' MFMA operands
// from LDS.  Wave w still takes rows 16 w .. 16 w + 15 of every step in the same k-step order,
// so every output is the same sum as gemm_tn_kernel's (that kernel stays for row strides or
// bases that are not 16-byte aligned).
// (SEG, r6) B = column segments: columns [kend[s-1], kend[s]) are segment s's row r / div[s]
// (rows[s] rows, stride ld[s]); every kend a multiple of 64, so a 64-wide k-block reads one segment
// (the descriptor tail's cat([x2 repeated over k rows, x1, att_map]) without materialising it)
struct TnSeg {
    const float *base[3];
    int ld[3], div[3], kend[3], rows[3];
};
// (PREB, r6) B is the previous layer's pre-BatchNorm output: each staged B value is
// bn_act(B, mean[k], invstd[k], gamma[k], beta[k], ReLU) (hreg_bn_apply's arithmetic; rows past
// R stay 0), so the sums are those over the materialised activation
struct TnPre {
    const float *mean, *invstd, *gamma, *beta;
};

template <int TNN, int TNK, bool SEG = false, bool PREB = false>
__global__ __launch_bounds__(256) void gemm_tn4_kernel(const float *__restrict__ A, int lda,
                                                       const float *__restrict__ Bm, int ldb, int R,
                                                       int N, int K, int rows_per_split,
                                                       float *__restrict__ ws, TnSeg sg = {}, TnPre pb = {}) {
    constexpr int WA = 32 * TNN, WB = 32 * TNK, TW = WB;  // tile widths (floats)
    constexpr int FA = WA / 4, FB = WB / 4;               // float4 per row
    constexpr int LA = TN_ROWS * FA / 256, LB = TN_ROWS * FB / 256;  // float4 loads per thread
    constexpr int STAGE = TN_ROWS * (WA + WB);
    constexpr int RED = 3 * WA * WB;
    __shared__ __attribute__((aligned(16))) float lds[STAGE > RED ? STAGE : RED];
    float *As = lds, *Bs = lds + TN_ROWS * WA;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int n0 = blockIdx.x * WA, k0 = blockIdx.y * WB;
    const int r0 = blockIdx.z * rows_per_split;
    const int r1 = min(R, r0 + rows_per_split);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(A), (short)0,
                                                      (int)((size_t)R * lda * sizeof(float)), 0x00020000);
    int bdiv = 1, bcol = k0;  // B row divisor and this block's first column in its source
    const float *Bsrc = Bm;
    int brows = R;
    if constexpr (SEG) {
        const int s = k0 < sg.kend[0] ? 0 : k0 < sg.kend[1] ? 1 : 2;  // (uniform)
        Bsrc = sg.base[s];
        ldb = sg.ld[s];
        bdiv = sg.div[s];
        bcol = k0 - (s == 0 ? 0 : sg.kend[s - 1]);
        brows = sg.rows[s];
    }
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Bsrc), (short)0,
                                                      (int)((size_t)brows * ldb * sizeof(float)), 0x00020000);
    typedef float v4f __attribute__((ext_vector_type(4)));
    f32x16 acc[TNN][TNK];
#pragma unroll
    for (int a = 0; a < TNN; ++a)
#pragma unroll
        for (int b = 0; b < TNK; ++b)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;
    v4f ga[LA], gb[LB];
    // (PREB) this thread's 4 B columns are the same in every staged row (256 % FB == 0)
    v4f pm = {}, pi = {}, pg = {}, pbe = {};
    int gbase = 0;
    if constexpr (PREB) {
        static_assert(256 % FB == 0, "B column per thread");
        const int c0 = bcol + 4 * (tid % FB);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool ok = c0 + u < K;
            pm[u] = ok ? pb.mean[c0 + u] : 0.f;
            pi[u] = ok ? pb.invstd[c0 + u] : 0.f;
            pg[u] = ok ? pb.gamma[c0 + u] : 0.f;
            pbe[u] = ok ? pb.beta[c0 + u] : 0.f;
        }
    }
    // rows past R read 0 (buffer bounds); columns past N / K feed only accumulator entries that
    // are never stored (the tile's columns stay inside the row: lda >= N, ldb >= K, 4 | lda, ldb)
    auto gload = [&](int base) {
        gbase = base;
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int e = tid + 256 * i, r = e / FA, c4 = e - r * FA;
            const uint32_t off = ((uint32_t)(base + r) * (uint32_t)lda + n0 + 4 * c4) * 4u;
            ga[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            const int e = tid + 256 * i, r = e / FB, c4 = e - r * FB;
            const uint32_t br = SEG ? (uint32_t)(base + r) / (uint32_t)bdiv : (uint32_t)(base + r);
            const uint32_t off = (br * (uint32_t)ldb + bcol + 4 * c4) * 4u;
            gb[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0));
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int i = 0; i < LA; ++i) *reinterpret_cast<v4f *>(As + 4 * (tid + 256 * i)) = ga[i];
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            v4f v = gb[i];
            if constexpr (PREB) {
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = bn_act(v[u], pm[u], pi[u], pg[u], pbe[u], 1);
                if (gbase + TN_ROWS > R) {  // (the last step: rows past R stay 0)
                    const bool live = gbase + (tid + 256 * i) / FB < R;
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] = live ? v[u] : 0.f;
                }
            }
            *reinterpret_cast<v4f *>(Bs + 4 * (tid + 256 * i)) = v;
        }
    };
    const int nit = r1 > r0 ? (r1 - r0 + TN_ROWS - 1) / TN_ROWS : 0;
    if (nit) gload(r0);
    for (int it = 0; it < nit; ++it) {
        __syncthreads();  // the previous step's operand reads are done
        lstore();
        __syncthreads();
        if (it + 1 < nit) gload(r0 + (it + 1) * TN_ROWS);
        // k-step s of wave w: rows 16 w + 2 s + h (gemm_tn_kernel's order)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int r = 16 * w + 2 * s + h;
            float va[TNN], vb[TNK];
#pragma unroll
            for (int a = 0; a < TNN; ++a) va[a] = As[r * WA + 32 * a + j];
#pragma unroll
            for (int b = 0; b < TNK; ++b) vb[b] = Bs[r * WB + 32 * b + j];
#pragma unroll
            for (int a = 0; a < TNN; ++a)
#pragma unroll
                for (int b = 0; b < TNK; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(va[a], vb[b], acc[a][b], 0, 0, 0);
        }
    }
    __syncthreads();  // the staging buffer becomes the cross-wave reduction buffer
    // acc[a][b][q]: tile row n = 32 a + (q&3) + 8(q>>2) + 4h, column k = 32 b + j
    if (w > 0) {
        float *o = lds + (w - 1) * WA * WB;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int n = (q & 3) + 8 * (q >> 2) + 4 * h;
#pragma unroll
            for (int a = 0; a < TNN; ++a)
#pragma unroll
                for (int b = 0; b < TNK; ++b) o[(32 * a + n) * TW + 32 * b + j] = acc[a][b][q];
        }
    }
    __syncthreads();
    if (w != 0) return;
    float *o = ws + (size_t)blockIdx.z * N * K;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int n = (q & 3) + 8 * (q >> 2) + 4 * h;
#pragma unroll
        for (int a = 0; a < TNN; ++a)
#pragma unroll
            for (int b = 0; b < TNK; ++b) {
                const int nn = 32 * a + n, kk = 32 * b + j;
                float v = acc[a][b][q];
                v = fadd_rn(v, lds[0 * WA * WB + nn * TW + kk]);
                v = fadd_rn(v, lds[1 * WA * WB + nn * TW + kk]);
                v = fadd_rn(v, lds[2 * WA * WB + nn * TW + kk]);
                if (n0 + nn < N && k0 + kk < K) o[(size_t)(n0 + nn) * K + k0 + kk] = v;
            }
    }
}

// out[i] = beta * out[i] + sum_z ws[z][i], z in order.  With many splits a workgroup
// takes 16 outputs x 16 split lanes (lane l sums z = l, l+16, ... in order, then the 16
// lanes in order); with few, one thread per output.
template <int LANES>
__global__ __launch_bounds__(256) void tn_reduce_kernel(const float *__restrict__ ws, int S, size_t NK,
                                                        float beta, float *__restrict__ out) {
    if (LANES == 1) {
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NK;
             i += (size_t)gridDim.x * blockDim.x) {
            float s = 0.f;
            for (int z = 0; z < S; ++z) s = fadd_rn(s, ws[(size_t)z * NK + i]);
            out[i] = beta != 0.f ? fadd_rn(fmul_rn(beta, out[i]), s) : s;
        }
        return;
    }
    constexpr int OUTS = 256 / LANES;
    __shared__ float part[256];
    const int ol = threadIdx.x % OUTS, sl = threadIdx.x / OUTS;
    const size_t i = (size_t)blockIdx.x * OUTS + ol;
    float s = 0.f;
    if (i < NK) {
#pragma unroll 4
        for (int z = sl; z < S; z += LANES) s = fadd_rn(s, ws[(size_t)z * NK + i]);
    }
    part[threadIdx.x] = s;
    __syncthreads();
    if (sl != 0 || i >= NK) return;
    float t = 0.f;
    for (int q = 0; q < LANES; ++q) t = fadd_rn(t, part[q * OUTS + ol]);
    out[i] = beta != 0.f ? fadd_rn(fmul_rn(beta, out[i]), t) : t;
}

__global__ void transpose_kernel(const float *__restrict__ in, int R, int C, float *__restrict__ out) {
    __shared__ float t[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    for (int i = threadIdx.y; i < 32; i += blockDim.y) {
        const int r = r0 + i, c = c0 + threadIdx.x;
        t[i][threadIdx.x] = (r < R && c < C) ? in[(size_t)r * C + c] : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.y; i < 32; i += blockDim.y) {
        const int c = c0 + i, r = r0 + threadIdx.x;
        if (c < C && r < R) out[(size_t)c * R + r] = t[threadIdx.x][i];
    }
}

// torch.optim.Adam (torch/optim/adam.py, foreach path, weight_decay 0), same order:
//   m = lerp(m, g, 1 - b1) = m + (1 - b1)(g - m);  v = b2 v + ((1 - b2) g) g
//   denom = sqrt(v) / sqrt(1 - b2^t) + eps;  p += (-lr / (1 - b1^t)) * (m / denom)
// scal (optional): {step_size, bc2_sqrt} read from device memory (a captured graph's replays
// take each step's bias corrections from there, hreg_adam_step_dev)
__global__ void adam_kernel(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                            float *__restrict__ v, size_t n, float lr, float b1, float b2, float eps,
                            float step_size, float bc2_sqrt, const float *__restrict__ scal = nullptr) {
    if (scal) {
        step_size = scal[0];
        bc2_sqrt = scal[1];
    }
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const float gi = g[i];
        const float mi = fadd_rn(m[i], fmul_rn(1.f - b1, fsub_rn(gi, m[i])));
        const float vi = fadd_rn(fmul_rn(b2, v[i]), fmul_rn(fmul_rn(1.f - b2, gi), gi));
        m[i] = mi;
        v[i] = vi;
        const float denom = fadd_rn(sqrtf(vi) / bc2_sqrt, eps);
        p[i] = fadd_rn(p[i], fmul_rn(-step_size, mi / denom));
    }
}

__global__ void add_into_kernel(const float4 *__restrict__ x, float4 *__restrict__ y, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 a = x[i];
        float4 b = y[i];
        b.x = fadd_rn(b.x, a.x); b.y = fadd_rn(b.y, a.y); b.z = fadd_rn(b.z, a.z); b.w = fadd_rn(b.w, a.w);
        y[i] = b;
    }
}

__global__ void add_into_tail_kernel(const float *__restrict__ x, float *__restrict__ y, size_t i0, size_t n) {
    for (size_t i = i0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        y[i] = fadd_rn(y[i], x[i]);
}

// row splits so that col_blocks x S reaches `target` workgroups (2048 = 8 per CU: a
// streaming reduction needs several waves per SIMD in flight to reach HBM rate; for
// the weight-gradient GEMM too, despite the extra N x K partials: A/B 235 vs 232
// train pairs/s against a 512 target)
int splits_for(int R, int col_blocks, int min_rows, int target = 2048, int cap = 1024) {
    int S = 1;
    while (col_blocks * S < target && R / (S * 2) >= min_rows && S < cap) S *= 2;
    return S;
}

unsigned grid1d(size_t n) {
    size_t b = (n + 255) / 256;
    return (unsigned)(b > 4096 ? 4096 : (b ? b : 1));
}

}  // namespace

static int cr_blocks(int C) {
    const int cw = 1 << cr_width_log2(C);
    return (C + cw - 1) / cw;
}

// row splits of a col_reduce launch; the BN backward's two-stream reduction (MODE 1) takes
// up to 4096 (a wave keeps only 16 loads in flight: more workgroups, not longer loops)
static int cr_splits(int R, int C, bool bwd) { return splits_for(R, cr_blocks(C), 256, 2048, bwd ? 4096 : 1024); }

// partials [S][C][2] doubles, then 2C floats (hreg_bn_backward's own dgamma / dbeta when
// it accumulates into the caller's)
static size_t cr_partial_bytes(int R, int C) {
    const int S = cr_splits(R, C, true);  // (>= every mode's)
    return (size_t)S * C * 2 * sizeof(double);
}

extern "C" size_t hreg_col_reduce_ws_bytes(int R, int C) {
    if (R <= 0 || C <= 0) return 0;
    return cr_partial_bytes(R, C) + (size_t)2 * C * sizeof(float);
}

extern "C" int hreg_bn_stats(const float *y, int R, int C, float eps, void *ws, float *mean,
                             float *invstd, float *var_unbiased, void *stream) {
    if (!y || !ws || !mean || !invstd || R <= 0 || C <= 0) return HREG_ERR_INVALID;
    const int cb = cr_blocks(C), S = splits_for(R, cb, 256);
    const int rps = (R + S - 1) / S;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(col_reduce_kernel<0>, dim3(cb, S), dim3(CR_THREADS), 0, st, y, nullptr, nullptr,
                       nullptr, nullptr, nullptr, nullptr, 0, R, C, rps, cr_width_log2(C), (double *)ws);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(col_finalize_kernel<0>, dim3((C + FIN_COLS - 1) / FIN_COLS), dim3(FIN_COLS * FIN_LANES), 0, st,
                       (const double *)ws, S, R, C, eps, mean, invstd, var_unbiased);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// statistics of S column partials [S][C][2] (sum y, sum y^2; ts_gemm.hip's fused epilogue)
int hreg_bn_finalize_stats(const double *part, int S, int R, int C, float eps, float *mean, float *invstd,
                           float *var_unbiased, float momentum, float *running_mean, float *running_var,
                           hipStream_t st) {
    hipLaunchKernelGGL(col_finalize_kernel<0>, dim3((C + FIN_COLS - 1) / FIN_COLS), dim3(FIN_COLS * FIN_LANES), 0, st,
                       part, S, R, C, eps, mean, invstd, var_unbiased, running_mean, running_var, momentum);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_bn_apply(const float *y, int R, int C, const float *mean, const float *invstd,
                             const float *gamma, const float *beta, int relu, float *out,
                             void *stream) {
    if (!y || !mean || !invstd || !gamma || !beta || !out || R < 0 || C <= 0) return HREG_ERR_INVALID;
    const size_t total = (size_t)R * C;
    if (!total) return HREG_OK;
    if (C % 4 == 0 && C <= BN4_MAXC && total / 4 < (size_t)INT32_MAX && !(reinterpret_cast<uintptr_t>(y) & 15) &&
        !(reinterpret_cast<uintptr_t>(out) & 15))
        hipLaunchKernelGGL(bn_apply4_kernel, dim3(grid1d(total / 4)), dim3(256), 0, as_stream(stream),
                           reinterpret_cast<const float4 *>(y), mean, invstd, gamma, beta, relu, (int)(total / 4),
                           C / 4, reinterpret_cast<float4 *>(out));
    else
        hipLaunchKernelGGL(bn_apply_kernel, dim3(grid1d(total)), dim3(256), 0, as_stream(stream), y, mean,
                           invstd, gamma, beta, relu, total, C, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_bn_backward(const float *dout, const float *out, const float *y, int R, int C,
                                const float *mean, const float *invstd, const float *gamma,
                                const float *beta, int relu, void *ws, float *dy, float *dgamma,
                                float *dbeta, int accumulate, void *stream) {
    if (!dout || !y || !mean || !invstd || !gamma || !ws || !dy || !dgamma || !dbeta || R <= 0 ||
        C <= 0 || (relu && !out && !beta))
        return HREG_ERR_INVALID;
    const int cb = cr_blocks(C), S = cr_splits(R, C, true);
    const int rps = (R + S - 1) / S;
    hipStream_t st = as_stream(stream);
    auto red = !relu ? col_reduce_kernel<1, 0> : out ? col_reduce_kernel<1, 1> : col_reduce_kernel<1, 2>;
    hipLaunchKernelGGL(red, dim3(cb, S), dim3(CR_THREADS), 0, st, dout, out, y, mean, invstd, gamma, beta, relu, R,
                       C, rps, cr_width_log2(C), (double *)ws);
    HREG_CHECK_LAUNCH();
    // accumulate: this call's dgamma / dbeta (read by the dy pass) go to the workspace tail
    // and are added to the caller's
    float *dg = dgamma, *db = dbeta;
    if (accumulate) {
        dg = reinterpret_cast<float *>(static_cast<char *>(ws) + cr_partial_bytes(R, C));
        db = dg + C;
    }
    hipLaunchKernelGGL(col_finalize_kernel<1>, dim3((C + FIN_COLS - 1) / FIN_COLS), dim3(FIN_COLS * FIN_LANES), 0, st,
                       (const double *)ws, S, R, C, 0.f, dg, db, nullptr, accumulate ? dgamma : nullptr,
                       accumulate ? dbeta : nullptr);
    HREG_CHECK_LAUNCH();
    dgamma = dg;
    dbeta = db;
    const size_t total = (size_t)R * C;
    if (C % 4 == 0 && C <= BN4_MAXC && total / 4 < (size_t)INT32_MAX &&
        !((reinterpret_cast<uintptr_t>(dout) | reinterpret_cast<uintptr_t>(out) |
           reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(dy)) & 15))
        hipLaunchKernelGGL(bn_backward4_kernel, dim3(grid1d(total / 4)), dim3(256), 0, st,
                           reinterpret_cast<const float4 *>(dout), reinterpret_cast<const float4 *>(out),
                           reinterpret_cast<const float4 *>(y), mean, invstd, gamma, beta, dgamma, dbeta, relu,
                           (int)(total / 4), R, C / 4, reinterpret_cast<float4 *>(dy));
    else
        hipLaunchKernelGGL(bn_backward_kernel, dim3(grid1d(total)), dim3(256), 0, st, dout, out, y, mean,
                           invstd, gamma, beta, dgamma, dbeta, relu, total, R, C, dy);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_bn_running_update(const float *mean, const float *var_unbiased, int C,
                                      float momentum, float *running_mean, float *running_var,
                                      void *stream) {
    if (!mean || !var_unbiased || !running_mean || !running_var || C <= 0) return HREG_ERR_INVALID;
    hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, as_stream(stream), mean,
                       var_unbiased, C, momentum, running_mean, running_var);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_col_sum(const float *x, int R, int C, void *ws, float *out, int accumulate,
                            void *stream) {
    if (!x || !ws || !out || R <= 0 || C <= 0) return HREG_ERR_INVALID;
    const int cb = cr_blocks(C), S = splits_for(R, cb, 256);
    const int rps = (R + S - 1) / S;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(col_reduce_kernel<2>, dim3(cb, S), dim3(CR_THREADS), 0, st, x, nullptr, nullptr,
                       nullptr, nullptr, nullptr, nullptr, 0, R, C, rps, cr_width_log2(C), (double *)ws);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(col_finalize_kernel<2>, dim3((C + FIN_COLS - 1) / FIN_COLS), dim3(FIN_COLS * FIN_LANES), 0, st,
                       (const double *)ws, S, R, C, 0.f, accumulate ? nullptr : out, nullptr, nullptr,
                       accumulate ? out : nullptr);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

static int tn_splits(int R, int N, int K) {
    return splits_for(R, ((N + 63) / 64) * ((K + 63) / 64), 512);
}

extern "C" size_t hreg_gemm_tn_ws_bytes(int R, int N, int K) {
    if (R <= 0 || N <= 0 || K <= 0) return 0;
    return (size_t)tn_splits(R, N, K) * N * K * sizeof(float);
}

static int gemm_tn_launch(const float *A, int lda, const float *B, int ldb, int R, int N, int K, float beta,
                          void *ws, float *out, void *stream, int S) {
    if (!A || !B || !ws || !out || R <= 0 || N <= 0 || K <= 0 || lda < N || ldb < K || S <= 0)
        return HREG_ERR_INVALID;
    if ((size_t)R * lda * sizeof(float) >= ((size_t)1 << 31) || (size_t)R * ldb * sizeof(float) >= ((size_t)1 << 31))
        return HREG_ERR_UNSUPPORTED;  // (buffer-descriptor addressing)
    int rps = (R + S - 1) / S;
    rps = (rps + TN_ROWS - 1) / TN_ROWS * TN_ROWS;
    hipStream_t st = as_stream(stream);
    // 64-wide output tiles as before (same splits, same sums); a 32-wide dimension runs one
    // tile of MFMAs across it instead of two
    const int tnn = N <= 32 ? 1 : 2, tnk = K <= 32 ? 1 : 2;
    const dim3 grid((N + 32 * tnn - 1) / (32 * tnn), (K + 32 * tnk - 1) / (32 * tnk), S);
    // 16-byte row segments through LDS when the rows allow them (gemm_tn4_kernel: the same sums)
    // (r6, train bench paired on one box: 422 / 426 vs 413 / 419 pairs/s, gpurun_out/r6tn)
    const bool v4 = !(lda & 3) && !(ldb & 3) && !(reinterpret_cast<uintptr_t>(A) & 15) &&
                    !(reinterpret_cast<uintptr_t>(B) & 15);
#define TN_LAUNCH(KER, a, b)                                                                           \
    hipLaunchKernelGGL((KER<a, b>), grid, dim3(256), 0, st, A, lda, B, ldb, R, N, K, rps, (float *)ws)
#define TN_CASE(a, b)                        \
    if (v4) TN_LAUNCH(gemm_tn4_kernel, a, b); \
    else TN_LAUNCH(gemm_tn_kernel, a, b)
    if (tnn == 1 && tnk == 1) {
        TN_CASE(1, 1);
    } else if (tnn == 1) {
        TN_CASE(1, 2);
    } else if (tnk == 1) {
        TN_CASE(2, 1);
    } else {
        TN_CASE(2, 2);
    }
#undef TN_CASE
#undef TN_LAUNCH
    HREG_CHECK_LAUNCH();
    const size_t NK = (size_t)N * K;
    if (S >= 16)
        hipLaunchKernelGGL(tn_reduce_kernel<16>, dim3((unsigned)((NK + 15) / 16)), dim3(256), 0, st,
                           (const float *)ws, S, NK, beta, out);
    else
        hipLaunchKernelGGL(tn_reduce_kernel<1>, dim3(grid1d(NK)), dim3(256), 0, st, (const float *)ws,
                           S, NK, beta, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_gemm_tn(const float *A, int lda, const float *B, int ldb, int R, int N, int K,
                            float beta, void *ws, float *out, void *stream) {
    return gemm_tn_launch(A, lda, B, ldb, R, N, K, beta, ws, out, stream, R > 0 ? tn_splits(R, N, K) : 1);
}

// hreg_gemm_tn with B = the previous layer's pre-BatchNorm output: B enters as
// bn_act(B, pre_mean, pre_invstd, pre_gamma, pre_beta, pre_relu) per column (the weight gradient
// dW = dY^T act(y_in) of train.py _ConvStats without the activation materialised); the same
// splits and sums as hreg_gemm_tn over the materialised B.  16-byte aligned rows only.
extern "C" int hreg_gemm_tn_pre(const float *A, int lda, const float *B, int ldb, int R, int N, int K, float beta,
                                void *ws, float *out, const float *pre_mean, const float *pre_invstd,
                                const float *pre_gamma, const float *pre_beta, int pre_relu, void *stream) {
    if (!A || !B || !ws || !out || R <= 0 || N <= 0 || K <= 0 || lda < N || ldb < K || !pre_mean || !pre_invstd ||
        !pre_gamma || !pre_beta)
        return HREG_ERR_INVALID;
    if (!pre_relu) return HREG_ERR_UNSUPPORTED;  // (the chains' activations are all ReLU)
    if ((lda & 3) || (ldb & 3) || ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) ||
        (size_t)R * lda * sizeof(float) >= ((size_t)1 << 31) || (size_t)R * ldb * sizeof(float) >= ((size_t)1 << 31))
        return HREG_ERR_UNSUPPORTED;
    const int S = tn_splits(R, N, K);
    int rps = (R + S - 1) / S;
    rps = (rps + TN_ROWS - 1) / TN_ROWS * TN_ROWS;
    hipStream_t st = as_stream(stream);
    const int tnn = N <= 32 ? 1 : 2, tnk = K <= 32 ? 1 : 2;
    const dim3 grid((N + 32 * tnn - 1) / (32 * tnn), (K + 32 * tnk - 1) / (32 * tnk), S);
    const TnPre pre{pre_mean, pre_invstd, pre_gamma, pre_beta};
#define TNP_CASE(a, b)                                                                                          \
    hipLaunchKernelGGL((gemm_tn4_kernel<a, b, false, true>), grid, dim3(256), 0, st, A, lda, B, ldb, R, N, K, rps, \
                       (float *)ws, TnSeg{}, pre)
    if (tnn == 1 && tnk == 1) TNP_CASE(1, 1);
    else if (tnn == 1) TNP_CASE(1, 2);
    else if (tnk == 1) TNP_CASE(2, 1);
    else TNP_CASE(2, 2);
#undef TNP_CASE
    HREG_CHECK_LAUNCH();
    const size_t NK = (size_t)N * K;
    if (S >= 16)
        hipLaunchKernelGGL(tn_reduce_kernel<16>, dim3((unsigned)((NK + 15) / 16)), dim3(256), 0, st,
                           (const float *)ws, S, NK, beta, out);
    else
        hipLaunchKernelGGL(tn_reduce_kernel<1>, dim3(grid1d(NK)), dim3(256), 0, st, (const float *)ws,
                           S, NK, beta, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// hreg_gemm_tn with B = cat([x2 repeated over the k rows of each group, x1, att]) (the descriptor
// tail, layers.py:204-206) read in place: x2 [R/k][C1], x1 [R][C1], att [R][Ca], C1 and Ca
// multiples of 64; out [N][2 C1 + Ca] (r6).  The same sums as hreg_gemm_tn on the materialised
// matrix (the same values in the same row order per wave).  ws: hreg_gemm_tn_ws_bytes(R, N, 2C1+Ca).
extern "C" int hreg_gemm_tn_tail(const float *A, int lda, const float *x2, int k, const float *x1, int C1,
                                 const float *att, int Ca, int R, int N, float beta, void *ws, float *out,
                                 void *stream) {
    const int K = 2 * C1 + Ca;
    if (!A || !x2 || !x1 || !att || !ws || !out || R <= 0 || N <= 0 || k <= 0 || R % k || lda < N || (lda & 3) ||
        (C1 & 63) || (Ca & 63) ||
        ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(x2) | reinterpret_cast<uintptr_t>(x1) |
          reinterpret_cast<uintptr_t>(att)) & 15))
        return HREG_ERR_INVALID;
    if ((size_t)R * lda * sizeof(float) >= ((size_t)1 << 31) || (size_t)R * Ca * sizeof(float) >= ((size_t)1 << 31) ||
        (size_t)R * C1 * sizeof(float) >= ((size_t)1 << 31))
        return HREG_ERR_UNSUPPORTED;
    const int S = tn_splits(R, N, K);
    int rps = (R + S - 1) / S;
    rps = (rps + TN_ROWS - 1) / TN_ROWS * TN_ROWS;
    TnSeg sg;
    sg.base[0] = x2; sg.ld[0] = C1; sg.div[0] = k; sg.kend[0] = C1; sg.rows[0] = R / k;
    sg.base[1] = x1; sg.ld[1] = C1; sg.div[1] = 1; sg.kend[1] = 2 * C1; sg.rows[1] = R;
    sg.base[2] = att; sg.ld[2] = Ca; sg.div[2] = 1; sg.kend[2] = K; sg.rows[2] = R;
    hipStream_t st = as_stream(stream);
    const int tnn = N <= 32 ? 1 : 2;  // (gemm_tn_launch's tiles: the same sums as its launch)
    const dim3 grid((N + 32 * tnn - 1) / (32 * tnn), K / 64, S);
    if (tnn == 1)
        hipLaunchKernelGGL((gemm_tn4_kernel<1, 2, true>), grid, dim3(256), 0, st, A, lda, x1, C1, R, N, K, rps,
                           (float *)ws, sg);
    else
        hipLaunchKernelGGL((gemm_tn4_kernel<2, 2, true>), grid, dim3(256), 0, st, A, lda, x1, C1, R, N, K, rps,
                           (float *)ws, sg);
    HREG_CHECK_LAUNCH();
    const size_t NK = (size_t)N * K;
    if (S >= 16)
        hipLaunchKernelGGL(tn_reduce_kernel<16>, dim3((unsigned)((NK + 15) / 16)), dim3(256), 0, st,
                           (const float *)ws, S, NK, beta, out);
    else
        hipLaunchKernelGGL(tn_reduce_kernel<1>, dim3(grid1d(NK)), dim3(256), 0, st, (const float *)ws, S, NK, beta,
                           out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// tools only (tools/tn_split_sweep.py): the same GEMM with S row splits (ws: S * N * K floats)
extern "C" int hreg_debug_gemm_tn_s(const float *A, int lda, const float *B, int ldb, int R, int N, int K,
                                    float beta, void *ws, float *out, void *stream, int S) {
    return gemm_tn_launch(A, lda, B, ldb, R, N, K, beta, ws, out, stream, S);
}

extern "C" int hreg_transpose(const float *in, int R, int C, float *out, void *stream) {
    if (!in || !out || R < 0 || C < 0) return HREG_ERR_INVALID;
    if (!R || !C) return HREG_OK;
    hipLaunchKernelGGL(transpose_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(32, 8), 0,
                       as_stream(stream), in, R, C, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_add_into(const float *x, float *y, size_t n, void *stream) {
    if (!x || !y) return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    hipStream_t st = as_stream(stream);
    const bool al = !((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15);
    const size_t n4 = al ? n / 4 : 0;
    if (n4) {
        hipLaunchKernelGGL(add_into_kernel, dim3(grid1d(n4)), dim3(256), 0, st, reinterpret_cast<const float4 *>(x),
                           reinterpret_cast<float4 *>(y), n4);
        HREG_CHECK_LAUNCH();
    }
    if (4 * n4 < n) {  // the < 4 tail of aligned buffers, or everything of unaligned ones
        hipLaunchKernelGGL(add_into_tail_kernel, dim3(grid1d(n - 4 * n4)), dim3(256), 0, st, x, y, 4 * n4, n);
        HREG_CHECK_LAUNCH();
    }
    return HREG_OK;
}

extern "C" int hreg_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                              size_t n, float lr, float beta1, float beta2, float eps, int step,
                              void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || step < 1) return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
    hipLaunchKernelGGL(adam_kernel, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), param, grad,
                       exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, (float)(lr / bc1),
                       (float)sqrt(bc2));
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// Adam with the step's bias corrections {lr / (1 - b1^t), sqrt(1 - b2^t)} (fp32, computed on
// the host in double as hreg_adam_step does) read from device memory at run time
extern "C" int hreg_adam_step_dev(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, size_t n,
                                  float lr, float beta1, float beta2, float eps, const float *scalars,
                                  void *stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !scalars) return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    hipLaunchKernelGGL(adam_kernel, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), param, grad, exp_avg,
                       exp_avg_sq, n, lr, beta1, beta2, eps, 0.f, 1.f, scalars);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
