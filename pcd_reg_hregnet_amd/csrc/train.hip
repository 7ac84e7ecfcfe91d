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

constexpr int CR_THREADS = 256;  // 64 columns x 4 row lanes

// per-column sums over rows [r0, r1): MODE 0: (y, y^2); MODE 1: (g, g*xhat) with
// g = dout * [out > 0 if relu], xhat = (y - mean) * invstd; MODE 2: (x, 0).
// double accumulators (the variance is E[y^2] - E[y]^2).
template <int MODE>
__global__ __launch_bounds__(CR_THREADS) void col_reduce_kernel(
    const float *__restrict__ x, const float *__restrict__ out, const float *__restrict__ y,
    const float *__restrict__ mean, const float *__restrict__ invstd, int relu, int R, int C,
    int rows_per_split, double *__restrict__ partial) {
    __shared__ double s0[4][64], s1[4][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int rl = threadIdx.x >> 6;
    const int r0 = blockIdx.y * rows_per_split;
    const int r1 = min(R, r0 + rows_per_split);
    double a = 0.0, b = 0.0;
    if (c < C) {
        float mu = 0.f, is = 0.f;
        if (MODE == 1) { mu = mean[c]; is = invstd[c]; }
        for (int r = r0 + rl; r < r1; r += 4) {
            const size_t i = (size_t)r * C + c;
            if (MODE == 0) {
                const double v = x[i];
                a += v;
                b += v * v;
            } else if (MODE == 1) {
                float g = x[i];
                if (relu && !(out[i] > 0.f)) g = 0.f;
                const float xh = fmul_rn(fsub_rn(y[i], mu), is);
                a += (double)g;
                b += (double)g * (double)xh;
            } else {
                a += (double)x[i];
            }
        }
    }
    s0[rl][threadIdx.x & 63] = a;
    s1[rl][threadIdx.x & 63] = b;
    __syncthreads();
    if (rl == 0 && c < C) {
        const int l = threadIdx.x;
        const double ta = ((s0[0][l] + s0[1][l]) + s0[2][l]) + s0[3][l];
        const double tb = ((s1[0][l] + s1[1][l]) + s1[2][l]) + s1[3][l];
        partial[((size_t)blockIdx.y * C + c) * 2 + 0] = ta;
        partial[((size_t)blockIdx.y * C + c) * 2 + 1] = tb;
    }
}

// column totals over the splits, in split order, then MODE's finalisation
template <int MODE>
__global__ void col_finalize_kernel(const double *__restrict__ partial, int S, int R, int C,
                                    float eps, float *__restrict__ o0, float *__restrict__ o1,
                                    float *__restrict__ o2) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double a = 0.0, b = 0.0;
    for (int s = 0; s < S; ++s) {
        a += partial[((size_t)s * C + c) * 2 + 0];
        b += partial[((size_t)s * C + c) * 2 + 1];
    }
    if (MODE == 0) {
        // mean, invstd (biased variance, used to normalise), unbiased variance (running stat)
        const double m = a / R;
        double var = b / R - m * m;
        if (var < 0.0) var = 0.0;
        o0[c] = (float)m;
        o1[c] = (float)(1.0 / sqrt(var + (double)eps));
        if (o2) o2[c] = (float)(R > 1 ? var * R / (R - 1) : var);
    } else if (MODE == 1) {
        o0[c] = (float)b;  // dgamma = sum g * xhat
        o1[c] = (float)a;  // dbeta = sum g
    } else {
        o0[c] = (float)a;
    }
}

__global__ void bn_apply_kernel(const float *__restrict__ y, const float *__restrict__ mean,
                                const float *__restrict__ invstd, const float *__restrict__ gamma,
                                const float *__restrict__ beta, int relu, size_t total, int C,
                                float *__restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const float xh = fmul_rn(fsub_rn(y[i], mean[c]), invstd[c]);
        float v = fadd_rn(fmul_rn(xh, gamma[c]), beta[c]);
        if (relu) v = fmaxf(v, 0.f);
        out[i] = v;
    }
}

// dy = gamma * invstd * (g - dbeta / R - xhat * dgamma / R)
__global__ void bn_backward_kernel(const float *__restrict__ dout, const float *__restrict__ out,
                                   const float *__restrict__ y, const float *__restrict__ mean,
                                   const float *__restrict__ invstd, const float *__restrict__ gamma,
                                   const float *__restrict__ dgamma, const float *__restrict__ dbeta,
                                   int relu, size_t total, int R, int C, float *__restrict__ dy) {
    const float invR = 1.0f / (float)R;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        float g = dout[i];
        if (relu && !(out[i] > 0.f)) g = 0.f;
        const float xh = fmul_rn(fsub_rn(y[i], mean[c]), invstd[c]);
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
// out[n][k] = sum_r A[r][n] * B[r][k]: a 64 x 64 output tile per workgroup (4 waves,
// one 32 x 32 v_mfma_f32_32x32x2_f32 tile each), rows in chunks of 32 staged in LDS
// as loaded (row-major, coalesced), k-step s of a chunk = rows 2s, 2s+1 (lane half
// h takes row 2s+h).  Split over rows: split z writes its partial tile to
// ws[z][N][K]; tn_reduce_kernel sums the splits in order.
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int TN_BR = 32, TN_LDS = 64 + 32;  // row stride padded: halves hit distinct banks

__global__ __launch_bounds__(256) void gemm_tn_kernel(const float *__restrict__ A, int lda,
                                                      const float *__restrict__ Bm, int ldb, int R,
                                                      int N, int K, int rows_per_split,
                                                      float *__restrict__ ws) {
    __shared__ float As[TN_BR][TN_LDS], Bs[TN_BR][TN_LDS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int n0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
    const int r0 = blockIdx.z * rows_per_split;
    const int r1 = min(R, r0 + rows_per_split);
    const int h = lane >> 5, j = lane & 31;
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    for (int rc = r0; rc < r1; rc += TN_BR) {
        // stage 32 rows x 64 columns of A and B (8 floats per thread each)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = tid + i * 256;  // 0 .. 2047
            const int rr = e >> 6, cc = e & 63;
            const int r = rc + rr;
            const bool okr = r < r1;
            As[rr][cc] = (okr && n0 + cc < N) ? A[(size_t)r * lda + n0 + cc] : 0.f;
            Bs[rr][cc] = (okr && k0 + cc < K) ? Bm[(size_t)r * ldb + k0 + cc] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < TN_BR / 2; ++s) {
            const float a = As[2 * s + h][wm * 32 + j];
            const float b = Bs[2 * s + h][wn * 32 + j];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    // acc[q]: row n = (q&3) + 8(q>>2) + 4h of the wave tile, column k = j
    float *o = ws + (size_t)blockIdx.z * N * K;
    const int k = k0 + wn * 32 + j;
    if (k < K) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int n = n0 + wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
            if (n < N) o[(size_t)n * K + k] = acc[q];
        }
    }
}

__global__ void tn_reduce_kernel(const float *__restrict__ ws, int S, size_t NK, float beta,
                                 float *__restrict__ out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NK;
         i += (size_t)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int z = 0; z < S; ++z) s = fadd_rn(s, ws[(size_t)z * NK + i]);
        out[i] = beta != 0.f ? fadd_rn(fmul_rn(beta, out[i]), s) : s;
    }
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
__global__ void adam_kernel(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                            float *__restrict__ v, size_t n, float lr, float b1, float b2, float eps,
                            float step_size, float bc2_sqrt) {
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

int splits_for(int R, int col_blocks, int min_rows) {
    int S = 1;
    while (col_blocks * S < 512 && R / (S * 2) >= min_rows && S < 1024) S *= 2;
    return S;
}

unsigned grid1d(size_t n) {
    size_t b = (n + 255) / 256;
    return (unsigned)(b > 4096 ? 4096 : (b ? b : 1));
}

}  // namespace

extern "C" size_t hreg_col_reduce_ws_bytes(int R, int C) {
    if (R <= 0 || C <= 0) return 0;
    const int S = splits_for(R, (C + 63) / 64, 256);
    return (size_t)S * C * 2 * sizeof(double);
}

extern "C" int hreg_bn_stats(const float *y, int R, int C, float eps, void *ws, float *mean,
                             float *invstd, float *var_unbiased, void *stream) {
    if (!y || !ws || !mean || !invstd || R <= 0 || C <= 0) return HREG_ERR_INVALID;
    const int cb = (C + 63) / 64, S = splits_for(R, cb, 256);
    const int rps = (R + S - 1) / S;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(col_reduce_kernel<0>, dim3(cb, S), dim3(CR_THREADS), 0, st, y, nullptr, nullptr,
                       nullptr, nullptr, 0, R, C, rps, (double *)ws);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(col_finalize_kernel<0>, dim3((C + 255) / 256), dim3(256), 0, st,
                       (const double *)ws, S, R, C, eps, mean, invstd, var_unbiased);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_bn_apply(const float *y, int R, int C, const float *mean, const float *invstd,
                             const float *gamma, const float *beta, int relu, float *out,
                             void *stream) {
    if (!y || !mean || !invstd || !gamma || !beta || !out || R < 0 || C <= 0) return HREG_ERR_INVALID;
    const size_t total = (size_t)R * C;
    if (!total) return HREG_OK;
    hipLaunchKernelGGL(bn_apply_kernel, dim3(grid1d(total)), dim3(256), 0, as_stream(stream), y, mean,
                       invstd, gamma, beta, relu, total, C, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_bn_backward(const float *dout, const float *out, const float *y, int R, int C,
                                const float *mean, const float *invstd, const float *gamma, int relu,
                                void *ws, float *dy, float *dgamma, float *dbeta, void *stream) {
    if (!dout || !y || !mean || !invstd || !gamma || !ws || !dy || !dgamma || !dbeta || R <= 0 ||
        C <= 0 || (relu && !out))
        return HREG_ERR_INVALID;
    const int cb = (C + 63) / 64, S = splits_for(R, cb, 256);
    const int rps = (R + S - 1) / S;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(col_reduce_kernel<1>, dim3(cb, S), dim3(CR_THREADS), 0, st, dout, out, y, mean,
                       invstd, relu, R, C, rps, (double *)ws);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(col_finalize_kernel<1>, dim3((C + 255) / 256), dim3(256), 0, st,
                       (const double *)ws, S, R, C, 0.f, dgamma, dbeta, nullptr);
    HREG_CHECK_LAUNCH();
    const size_t total = (size_t)R * C;
    hipLaunchKernelGGL(bn_backward_kernel, dim3(grid1d(total)), dim3(256), 0, st, dout, out, y, mean,
                       invstd, gamma, dgamma, dbeta, relu, total, R, C, dy);
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

extern "C" int hreg_col_sum(const float *x, int R, int C, void *ws, float *out, void *stream) {
    if (!x || !ws || !out || R <= 0 || C <= 0) return HREG_ERR_INVALID;
    const int cb = (C + 63) / 64, S = splits_for(R, cb, 256);
    const int rps = (R + S - 1) / S;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(col_reduce_kernel<2>, dim3(cb, S), dim3(CR_THREADS), 0, st, x, nullptr, nullptr,
                       nullptr, nullptr, 0, R, C, rps, (double *)ws);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(col_finalize_kernel<2>, dim3((C + 255) / 256), dim3(256), 0, st,
                       (const double *)ws, S, R, C, 0.f, out, nullptr, nullptr);
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

extern "C" int hreg_gemm_tn(const float *A, int lda, const float *B, int ldb, int R, int N, int K,
                            float beta, void *ws, float *out, void *stream) {
    if (!A || !B || !ws || !out || R <= 0 || N <= 0 || K <= 0 || lda < N || ldb < K)
        return HREG_ERR_INVALID;
    const int S = tn_splits(R, N, K);
    int rps = (R + S - 1) / S;
    rps = (rps + TN_BR - 1) / TN_BR * TN_BR;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(gemm_tn_kernel, dim3((N + 63) / 64, (K + 63) / 64, S), dim3(256), 0, st, A, lda,
                       B, ldb, R, N, K, rps, (float *)ws);
    HREG_CHECK_LAUNCH();
    const size_t NK = (size_t)N * K;
    hipLaunchKernelGGL(tn_reduce_kernel, dim3(grid1d(NK)), dim3(256), 0, st, (const float *)ws, S, NK,
                       beta, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_transpose(const float *in, int R, int C, float *out, void *stream) {
    if (!in || !out || R < 0 || C < 0) return HREG_ERR_INVALID;
    if (!R || !C) return HREG_OK;
    hipLaunchKernelGGL(transpose_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(32, 8), 0,
                       as_stream(stream), in, R, C, out);
    HREG_CHECK_LAUNCH();
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
