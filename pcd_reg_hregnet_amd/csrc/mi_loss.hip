// mi_loss.hip -- the Model_V2 training losses:
// ChamferDistanceLoss (losses/chamfer_loss.py:10-36 over the third-party
// chamfer_distance extension, not vendored: its published semantics are the
// nearest-neighbour squared distance in each direction) and the scalar parts of
// DeepMILoss's Jensen-Shannon estimator (losses/mi_loss_v2.py:42-79).  The
// discriminator convs themselves run on hreg_gemm / hreg_gemm_tn (mi_losses.py).
// Every reduction runs in a fixed order (one block, or per-block partials summed in
// block order): the same bits every run.
#include "common.h"

namespace {

constexpr int CH_THREADS = 256;
constexpr int CH_TILE = 1024;  // reference points staged in LDS per pass

// nearest squared distance from each query of cloud q to cloud p (both scaled by
// 1/scale first, chamfer_loss.py:27-28); ties keep the lowest index.
// grid (ceil(nq / 256), nb)
__global__ __launch_bounds__(CH_THREADS) void nn_dist_kernel(const float *__restrict__ q, const float *__restrict__ p,
                                                             int nq, int np, float scale,
                                                             float *__restrict__ dist, int32_t *__restrict__ idx) {
    __shared__ float sx[CH_TILE], sy[CH_TILE], sz[CH_TILE];
    const int b = blockIdx.y;
    const int i = blockIdx.x * CH_THREADS + threadIdx.x;
    float qx = 0.f, qy = 0.f, qz = 0.f;
    if (i < nq) {
        const float *v = q + ((size_t)b * nq + i) * 3;
        qx = v[0] / scale; qy = v[1] / scale; qz = v[2] / scale;
    }
    float best = __int_as_float(0x7f800000);
    int bi = -1;
    const float *P = p + (size_t)b * np * 3;
    for (int t0 = 0; t0 < np; t0 += CH_TILE) {
        const int nt = min(CH_TILE, np - t0);
        __syncthreads();
        for (int k = threadIdx.x; k < nt; k += CH_THREADS) {
            sx[k] = P[(size_t)(t0 + k) * 3] / scale;
            sy[k] = P[(size_t)(t0 + k) * 3 + 1] / scale;
            sz[k] = P[(size_t)(t0 + k) * 3 + 2] / scale;
        }
        __syncthreads();
        for (int k = 0; k < nt; ++k) {
            const float d = sqdist3(qx, qy, qz, sx[k], sy[k], sz[k]);
            if (d < best) { best = d; bi = t0 + k; }
        }
    }
    if (i < nq) {
        dist[(size_t)b * nq + i] = best;
        if (idx) idx[(size_t)b * nq + i] = bi;
    }
}

// chamfer_distance (chamfer_loss.py:10-16) per pair: (mean_i sqrt(d01_i) +
// mean_j sqrt(d10_j)) / 2, then the reduction (:29-34) over the batch.
// One block; per pair the sums run thread-strided, then tree-free in thread order.
__global__ __launch_bounds__(256) void chamfer_reduce_kernel(const float *__restrict__ d01,
                                                             const float *__restrict__ d10, int nb, int n,
                                                             int m, int reduction, float *__restrict__ per_pair,
                                                             float *__restrict__ out) {
    __shared__ float part[256];
    __shared__ float pair_val;
    float acc = 0.f;
    for (int b = 0; b < nb; ++b) {
        float s = 0.f;
        for (int i = threadIdx.x; i < n; i += 256) s = fadd_rn(s, sqrtf(d01[(size_t)b * n + i]));
        part[threadIdx.x] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = 0.f;
            for (int k = 0; k < 256; ++k) t = fadd_rn(t, part[k]);
            pair_val = t / (float)n;
        }
        __syncthreads();
        float s2 = 0.f;
        for (int j = threadIdx.x; j < m; j += 256) s2 = fadd_rn(s2, sqrtf(d10[(size_t)b * m + j]));
        part[threadIdx.x] = s2;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = 0.f;
            for (int k = 0; k < 256; ++k) t = fadd_rn(t, part[k]);
            const float v = fadd_rn(pair_val, t / (float)m) / 2.0f;
            if (per_pair) per_pair[b] = v;
            acc = fadd_rn(acc, v);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && out) out[0] = reduction == HREG_REDUCE_MEAN ? acc / (float)nb : acc;
}

__device__ __forceinline__ float softplus(float z) { return z > 20.f ? z : log1pf(expf(z)); }
__device__ __forceinline__ float sigmoidf(float z) { return 1.0f / fadd_rn(1.0f, expf(-z)); }

// DeepMILoss JS terms (mi_loss_v2.py:56-64): t_joint = T(c, x), t_marg = T(c, x');
// Ej = -mean softplus(-t_joint), Em = mean softplus(t_marg), loss = 0.5 (Em - Ej).
// out[0] = loss, out[1] = Ej, out[2] = Em; g_joint / g_marg = d loss / d t (optional).
// One block, thread-strided partial sums reduced in thread order.
__global__ __launch_bounds__(256) void js_kernel(const float *__restrict__ tj, const float *__restrict__ tm, int n,
                                                 float *__restrict__ out, float *__restrict__ gj,
                                                 float *__restrict__ gm) {
    __shared__ float pj[256], pm[256];
    float sj = 0.f, sm = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) {
        sj = fadd_rn(sj, softplus(-tj[i]));
        sm = fadd_rn(sm, softplus(tm[i]));
        if (gj) gj[i] = -0.5f * sigmoidf(-tj[i]) / (float)n;
        if (gm) gm[i] = 0.5f * sigmoidf(tm[i]) / (float)n;
    }
    pj[threadIdx.x] = sj;
    pm[threadIdx.x] = sm;
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, c = 0.f;
        for (int k = 0; k < 256; ++k) {
            a = fadd_rn(a, pj[k]);
            c = fadd_rn(c, pm[k]);
        }
        const float Ej = -(a / (float)n), Em = c / (float)n;
        out[0] = 0.5f * (Em - Ej);
        out[1] = Ej;
        out[2] = Em;
    }
}

// t[r] = act(dot(h[r], w) + b): the single-output conv/linear closing each
// discriminator (conv3 32->1 + ReLU, mi_loss_v2.py:33,39; l0 Linear C->1, :13,22).
// One wave per row.
__global__ __launch_bounds__(256) void rowdot_kernel(const float *__restrict__ h, int R, int C,
                                                     const float *__restrict__ w, const float *__restrict__ b,
                                                     int relu, float *__restrict__ t) {
    const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s = fadd_rn(s, fmul_rn(h[(size_t)r * C + c], w[c]));
    s = wave_sum_f32(s);
    if (b) s = fadd_rn(s, b[0]);
    if (relu) s = fmaxf(s, 0.f);
    if (lane == 0) t[r] = s;
}

// backward of rowdot: g' = g * [t > 0] (relu); dh[r][c] = g'[r] w[c];
// grid-stride over rows x channels
__global__ void rowdot_dh_kernel(const float *__restrict__ g, const float *__restrict__ t, int relu, int R,
                                 int C, const float *__restrict__ w, float *__restrict__ dh) {
    const size_t n = (size_t)R * C;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const size_t r = e / C;
        const int c = (int)(e - r * C);
        const float gr = (!relu || t[r] > 0.f) ? g[r] : 0.f;
        dh[e] = fmul_rn(gr, w[c]);
    }
}

// dw[c] = sum_r g'[r] h[r][c], db = sum_r g'[r]; one block per channel (and one for
// db), rows thread-strided, partials reduced in thread order
__global__ __launch_bounds__(256) void rowdot_dw_kernel(const float *__restrict__ g, const float *__restrict__ t,
                                                        int relu, int R, int C, const float *__restrict__ h,
                                                        float *__restrict__ dw, float *__restrict__ db) {
    __shared__ float part[256];
    const int c = blockIdx.x;  // c == C: the bias
    float s = 0.f;
    for (int r = threadIdx.x; r < R; r += 256) {
        const float gr = (!relu || t[r] > 0.f) ? g[r] : 0.f;
        s = fadd_rn(s, c < C ? fmul_rn(gr, h[(size_t)r * C + c]) : gr);
    }
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f;
        for (int k = 0; k < 256; ++k) a = fadd_rn(a, part[k]);
        if (c < C) {
            if (dw) dw[c] = a;
        } else if (db) {
            db[0] = a;
        }
    }
}

// dx = dy * [y > 0] (ReLU backward of the discriminator convs)
__global__ void relu_bwd_kernel(const float *__restrict__ dy, const float *__restrict__ y, size_t n,
                                float *__restrict__ dx) {
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
        dx[e] = y[e] > 0.f ? dy[e] : 0.f;
}

int grid1d(size_t n) {
    size_t g = (n + 255) / 256;
    return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int hreg_chamfer(const float *p0, const float *p1, int nb, int n, int m, float scale, int reduction,
                            float *d01, float *d10, int32_t *idx01, int32_t *idx10, float *per_pair, float *out,
                            void *stream) {
    if (!p0 || !p1 || !d01 || !d10 || nb <= 0 || n <= 0 || m <= 0 || !(scale > 0.f) || nb > 65535)
        return HREG_ERR_INVALID;
    if (reduction != HREG_REDUCE_MEAN && reduction != HREG_REDUCE_SUM && reduction != HREG_REDUCE_NONE)
        return HREG_ERR_INVALID;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(nn_dist_kernel, dim3((n + CH_THREADS - 1) / CH_THREADS, nb), dim3(CH_THREADS), 0, st, p0,
                       p1, n, m, scale, d01, idx01);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(nn_dist_kernel, dim3((m + CH_THREADS - 1) / CH_THREADS, nb), dim3(CH_THREADS), 0, st, p1,
                       p0, m, n, scale, d10, idx10);
    HREG_CHECK_LAUNCH();
    if (per_pair || out) {
        hipLaunchKernelGGL(chamfer_reduce_kernel, dim3(1), dim3(256), 0, st, d01, d10, nb, n, m, reduction,
                           per_pair, reduction == HREG_REDUCE_NONE ? nullptr : out);
        HREG_CHECK_LAUNCH();
    }
    return HREG_OK;
}

extern "C" int hreg_js_loss(const float *t_joint, const float *t_marg, int n, float *out, float *g_joint,
                            float *g_marg, void *stream) {
    if (!t_joint || !t_marg || !out || n <= 0) return HREG_ERR_INVALID;
    hipLaunchKernelGGL(js_kernel, dim3(1), dim3(256), 0, as_stream(stream), t_joint, t_marg, n, out, g_joint,
                       g_marg);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_rowdot(const float *h, int R, int C, const float *w, const float *b, int relu, float *t,
                           void *stream) {
    if (!h || !w || !t || R < 0 || C <= 0) return HREG_ERR_INVALID;
    if (!R) return HREG_OK;
    hipLaunchKernelGGL(rowdot_kernel, dim3((R + 3) / 4), dim3(256), 0, as_stream(stream), h, R, C, w, b, relu, t);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_rowdot_bwd(const float *g, const float *t, int relu, const float *h, int R, int C,
                               const float *w, float *dh, float *dw, float *db, void *stream) {
    if (!g || !h || !w || R < 0 || C <= 0 || (relu && !t)) return HREG_ERR_INVALID;
    if (!R) return HREG_OK;
    hipStream_t st = as_stream(stream);
    if (dh) {
        hipLaunchKernelGGL(rowdot_dh_kernel, dim3(grid1d((size_t)R * C)), dim3(256), 0, st, g, t, relu, R, C, w,
                           dh);
        HREG_CHECK_LAUNCH();
    }
    if (dw || db) {
        hipLaunchKernelGGL(rowdot_dw_kernel, dim3(C + 1), dim3(256), 0, st, g, t, relu, R, C, h, dw, db);
        HREG_CHECK_LAUNCH();
    }
    return HREG_OK;
}

extern "C" int hreg_relu_bwd(const float *dy, const float *y, size_t n, float *dx, void *stream) {
    if (!dy || !y || !dx) return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), dy, y, n, dx);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
