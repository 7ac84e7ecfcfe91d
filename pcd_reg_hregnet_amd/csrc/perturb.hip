// perturb.hip -- the data side in front of the path: the
// decalibration perturbation of TruckScenesPerturbation.lidar_to_lidar
// (dataset/man_dataset.py:606-631) over a batch of clouds, its SE(3) algebra
// (transform/rodrigues.py SO3/SE3), the twist generator of UniformTransformSE3
// (transform/dataset_transforms.py:65-145) and the range filter of
// PointCloudFilter (dataset/dataset_utils.py:113-127).
//
// Twists x = (w, v) in R^6 (rotation first).  One thread per transform for the
// algebra (a handful of flops); the point transform is one thread per point with
// the cloud's matrix recomputed per thread from its twist (no second launch).
// Float operations follow the reference's expression order (-ffp-contract=off);
// sin/cos/acos/tan are the device libm, so results agree with torch's CPU libm to
// a few ulp, not bitwise (tests: tests/test_gpu_perturb.py).
#include "common.h"

namespace {

constexpr float SINC_EPS = 0.01f;  // rodrigues.py:8,103,135 and inv_vecs_Xg_ig :414

// sinc1 = sin(t)/t, sinc2 = (1-cos t)/t^2, sinc3 = (t - sin t)/t^3 with the
// reference's O(t^8) Taylor branches for |t| < 0.01 (rodrigues.py:5-19,100-114,132-145)
__device__ float sinc1(float t) {
    if (fabsf(t) < SINC_EPS) {
        const float t2 = t * t;
        return 1.0f - t2 / 6.0f * (1.0f - t2 / 20.0f * (1.0f - t2 / 42.0f));
    }
    return sinf(t) / t;
}
__device__ float sinc2(float t) {
    const float t2 = t * t;
    if (fabsf(t) < SINC_EPS) return 0.5f * (1.0f - t2 / 12.0f * (1.0f - t2 / 30.0f * (1.0f - t2 / 56.0f)));
    return (1.0f - cosf(t)) / t2;
}
__device__ float sinc3(float t) {
    if (fabsf(t) < SINC_EPS) {
        const float t2 = t * t;
        return (1.0f / 6.0f) * (1.0f - t2 / 20.0f * (1.0f - t2 / 42.0f * (1.0f - t2 / 72.0f)));
    }
    return (t - sinf(t)) / (t * t * t);
}

__device__ float norm3(const float *w) { return sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]); }

// W = mat(w) (rodrigues.py:265-276), S = W W
__device__ void skew(const float *w, float *W) {
    W[0] = 0.f;   W[1] = -w[2]; W[2] = w[1];
    W[3] = w[2];  W[4] = 0.f;   W[5] = -w[0];
    W[6] = -w[1]; W[7] = w[0];  W[8] = 0.f;
}
__device__ void mul3(const float *A, const float *B, float *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

// R = I + sinc1(t) W + sinc2(t) S (SO3.exp, rodrigues.py:304-314); with V != null
// also V = I + sinc2(t) W + sinc3(t) S (SE3.exp, rodrigues.py:526-545)
__device__ void so3_exp(const float *w, float *R, float *V) {
    const float t = norm3(w);
    float W[9], S[9];
    skew(w, W);
    mul3(W, W, S);
    const float s1 = sinc1(t), s2 = sinc2(t);
    for (int i = 0; i < 9; ++i) R[i] = ((i % 4 == 0) ? 1.f : 0.f) + s1 * W[i] + s2 * S[i];
    if (V) {
        const float s3 = sinc3(t);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4 == 0) ? 1.f : 0.f) + s2 * W[i] + s3 * S[i];
    }
}

// g [16] row-major = SE3.exp(x)
__device__ void se3_exp(const float *x, float *g) {
    float R[9], V[9];
    so3_exp(x, R, V);
    for (int i = 0; i < 3; ++i) {
        g[i * 4 + 0] = R[i * 3 + 0];
        g[i * 4 + 1] = R[i * 3 + 1];
        g[i * 4 + 2] = R[i * 3 + 2];
        g[i * 4 + 3] = V[i * 3] * x[3] + V[i * 3 + 1] * x[4] + V[i * 3 + 2] * x[5];
    }
    g[12] = 0.f; g[13] = 0.f; g[14] = 0.f; g[15] = 1.f;
}

// w = SO3.log(R) (rodrigues.py:330-370): t = acos((tr - 1)/2); |sinc1(t)| > 1e-7 ->
// vec((R - R^T) / (2 sinc1)); <= 1e-7 (t = pi) -> the sign-fixed sqrt branch; a NaN
// angle (tr slightly > 3 from rounding) matches neither mask and leaves w = 0, as there.
__device__ void so3_log(const float *R, float *w) {
    const float tr = (R[0] + R[4]) + R[8];
    const float c = (tr - 1.0f) / 2.0f;
    const float t = acosf(c);
    const float sc = sinc1(t);
    w[0] = w[1] = w[2] = 0.f;
    if (fabsf(sc) > 1.0e-7f) {
        const float d = 2.0f * sc;
        w[0] = (R[7] - R[5]) / d;
        w[1] = (R[2] - R[6]) / d;
        w[2] = (R[3] - R[1]) / d;
    } else if (fabsf(sc) <= 1.0e-7f) {
        const float t2 = t * t;
        const float a00 = (R[0] + 1.f) * t2 / 2.f, a11 = (R[4] + 1.f) * t2 / 2.f, a22 = (R[8] + 1.f) * t2 / 2.f;
        const float a02 = R[2] * t2 / 2.f, a12 = R[5] * t2 / 2.f;
        float sgn3 = a02 > 0.f ? 1.f : a02 < 0.f ? -1.f : 0.f;
        if (sgn3 == 0.f) sgn3 = 1.f;
        float sgn23 = a12 > 0.f ? 1.f : a12 < 0.f ? -1.f : 0.f;
        if (sgn23 == 0.f) sgn23 = 1.f;
        w[0] = sqrtf(a00);
        w[1] = sqrtf(a11) * (sgn23 * sgn3);
        w[2] = sqrtf(a22) * sgn3;
    }
}

// x = SE3.log(g) (rodrigues.py:571-582): v = H p, H = inv_vecs_Xg_ig(w) =
// I - X/2 + eta S, eta = (1 - (t/2)/tan(t/2)) / t^2 (Taylor below 0.01, :400-420)
__device__ void se3_log(const float *g, float *x) {
    const float R[9] = {g[0], g[1], g[2], g[4], g[5], g[6], g[8], g[9], g[10]};
    float w[3];
    so3_log(R, w);
    const float t = norm3(w);
    float eta;
    if (t < SINC_EPS) {
        const float t2 = t * t;
        eta = ((t2 / 40.f + 1.f) * t2 / 42.f + 1.f) * t2 / 720.f + 1.0f / 12.0f;
    } else {
        eta = (1.f - (t / 2.f) / tanf(t / 2.f)) / (t * t);
    }
    float X[9], S[9];
    skew(w, X);
    mul3(X, X, S);
    float H[9];
    for (int i = 0; i < 9; ++i) H[i] = ((i % 4 == 0) ? 1.f : 0.f) - 0.5f * X[i] + eta * S[i];
    const float p[3] = {g[3], g[7], g[11]};
    x[0] = w[0]; x[1] = w[1]; x[2] = w[2];
    for (int i = 0; i < 3; ++i) x[3 + i] = H[i * 3] * p[0] + H[i * 3 + 1] * p[1] + H[i * 3 + 2] * p[2];
}

__global__ void se3_exp_kernel(const float *__restrict__ x, int n, float *__restrict__ g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float xi[6], gi[16];
    for (int c = 0; c < 6; ++c) xi[c] = x[(size_t)i * 6 + c];
    se3_exp(xi, gi);
    for (int c = 0; c < 16; ++c) g[(size_t)i * 16 + c] = gi[c];
}

__global__ void se3_log_kernel(const float *__restrict__ g, int n, float *__restrict__ x) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float gi[16], xi[6];
    for (int c = 0; c < 16; ++c) gi[c] = g[(size_t)i * 16 + c];
    se3_log(gi, xi);
    for (int c = 0; c < 6; ++c) x[(size_t)i * 6 + c] = xi[c];
}

// UniformTransformSE3.generate_transform (dataset_transforms.py:79-126) from its random
// draws s = (w draw 3, t draw 3) and (amp, tran) per twist:
//   uniform:          w = (2s - 1) amp,     t = (2s - 1) tran
//   gaussian:         w = s / |s| amp,      t = (s tran) / |s tran| tran
//   inverse_gaussian: w = s / |s| amp,      t = s / |s| tran
// then G = [so3.exp(w) | t] and x = se3.log(G).
__global__ void twist_kernel(const float *__restrict__ s, const float *__restrict__ amp_tran, int n,
                             int dist, float *__restrict__ x) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float amp = amp_tran[(size_t)i * 2], tran = amp_tran[(size_t)i * 2 + 1];
    float w[3], t[3];
    const float *si = s + (size_t)i * 6;
    if (dist == HREG_TWIST_UNIFORM) {
        for (int c = 0; c < 3; ++c) {
            w[c] = (2.f * si[c] - 1.f) * amp;
            t[c] = (2.f * si[3 + c] - 1.f) * tran;
        }
    } else {
        const float nw = norm3(si);
        float u[3];
        for (int c = 0; c < 3; ++c) u[c] = dist == HREG_TWIST_GAUSSIAN ? si[3 + c] * tran : si[3 + c];
        const float nt = norm3(u);
        for (int c = 0; c < 3; ++c) {
            w[c] = si[c] / nw * amp;
            t[c] = u[c] / nt * tran;
        }
    }
    float R[9], G[16];
    so3_exp(w, R, nullptr);
    for (int r = 0; r < 3; ++r) {
        G[r * 4 + 0] = R[r * 3 + 0];
        G[r * 4 + 1] = R[r * 3 + 1];
        G[r * 4 + 2] = R[r * 3 + 2];
        G[r * 4 + 3] = t[r];
    }
    G[12] = G[13] = G[14] = 0.f;
    G[15] = 1.f;
    float xi[6];
    se3_log(G, xi);
    for (int c = 0; c < 6; ++c) x[(size_t)i * 6 + c] = xi[c];
}

// uncalibed = SE3.transform(exp(x_b), pcd_b) (man_dataset.py:617-625,
// rodrigues.py:585-596: R a + p); cloud b's igt = exp(x_b) and gt = igt^-1 (the
// training loop's torch.inverse(igt), train_reg_v0.py:268-271) by thread 0 of the
// cloud's first block.  grid (ceil(N/256), B).
__global__ void perturb_kernel(const float *__restrict__ pts, const float *__restrict__ x, int N,
                               float *__restrict__ out, float *__restrict__ igt, float *__restrict__ gt) {
    const int b = blockIdx.y;
    float xb[6], g[16];
    for (int c = 0; c < 6; ++c) xb[c] = x[(size_t)b * 6 + c];
    se3_exp(xb, g);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) {
        const float *p = pts + ((size_t)b * N + i) * 3;
        float *o = out + ((size_t)b * N + i) * 3;
        for (int r = 0; r < 3; ++r) o[r] = (g[r * 4] * p[0] + g[r * 4 + 1] * p[1] + g[r * 4 + 2] * p[2]) + g[r * 4 + 3];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (igt)
            for (int c = 0; c < 16; ++c) igt[(size_t)b * 16 + c] = g[c];
        if (gt) {
            float *q = gt + (size_t)b * 16;
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) q[r * 4 + c] = g[c * 4 + r];
                q[r * 4 + 3] = -(g[r] * g[3] + g[4 + r] * g[7] + g[8 + r] * g[11]);
            }
            q[12] = q[13] = q[14] = 0.f;
            q[15] = 1.f;
        }
    }
}

// PointCloudFilter.remove_points_by_range (dataset_utils.py:113-127): keep the points
// with ||p|| < max_range, in order.  ||p|| as np.linalg.norm computes it for float32
// rows: sqrt((x*x + y*y) + z*z).  One 1024-thread workgroup per cloud; chunks of
// 1024 points compacted with a ballot/popcount prefix (wave) + LDS (waves).
constexpr int RF_THREADS = 1024;
__global__ __launch_bounds__(RF_THREADS) void range_filter_kernel(
    const float *__restrict__ pts, const float *__restrict__ inten, int N, float max_range,
    float *__restrict__ out, float *__restrict__ out_inten, int32_t *__restrict__ counts) {
    __shared__ int wsum[RF_THREADS / 64];
    __shared__ int base_s;
    const int b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float *P = pts + (size_t)b * N * 3;
    float *O = out + (size_t)b * N * 3;
    if (threadIdx.x == 0) base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < N; c0 += RF_THREADS) {
        const int i = c0 + threadIdx.x;
        bool keep = false;
        float px = 0.f, py = 0.f, pz = 0.f;
        if (i < N) {
            px = P[(size_t)i * 3]; py = P[(size_t)i * 3 + 1]; pz = P[(size_t)i * 3 + 2];
            keep = sqrtf((px * px + py * py) + pz * pz) < max_range;
        }
        const uint64_t m = __ballot(keep);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = base_s;
        for (int k = 0; k < w; ++k) off += wsum[k];
        if (keep) {
            const int dst = off + before;
            O[(size_t)dst * 3] = px; O[(size_t)dst * 3 + 1] = py; O[(size_t)dst * 3 + 2] = pz;
            if (inten) out_inten[(size_t)b * N + dst] = inten[(size_t)b * N + i];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int k = 0; k < RF_THREADS / 64; ++k) tot += wsum[k];
            base_s += tot;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[b] = base_s;
}

}  // namespace

extern "C" int hreg_se3_exp(const float *x, int n, float *g, void *stream) {
    if (!x || !g || n < 0) return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    hipLaunchKernelGGL(se3_exp_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), x, n, g);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_se3_log(const float *g, int n, float *x, void *stream) {
    if (!x || !g || n < 0) return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    hipLaunchKernelGGL(se3_log_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), g, n, x);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_twists_from_samples(const float *samples, const float *amp_tran, int n, int distribution,
                                        float *x, void *stream) {
    if (!samples || !amp_tran || !x || n < 0) return HREG_ERR_INVALID;
    if (distribution != HREG_TWIST_UNIFORM && distribution != HREG_TWIST_GAUSSIAN &&
        distribution != HREG_TWIST_INVERSE_GAUSSIAN)
        return HREG_ERR_INVALID;
    if (!n) return HREG_OK;
    hipLaunchKernelGGL(twist_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), samples, amp_tran,
                       n, distribution, x);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_perturb_clouds(const float *pts, const float *x, int nb, int n, float *out, float *igt,
                                   float *gt, void *stream) {
    if (!pts || !x || !out || nb < 0 || n < 0 || nb > 65535) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(perturb_kernel, dim3(n > 0 ? (n + 255) / 256 : 1, nb), dim3(256), 0, as_stream(stream),
                       pts, x, n, out, igt, gt);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_range_filter(const float *pts, const float *intensity, int nb, int n, float max_range,
                                 float *out, float *out_intensity, int32_t *counts, void *stream) {
    if (!counts || nb < 0 || n < 0 || (n > 0 && (!pts || !out)) || (intensity && !out_intensity))
        return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    if (!n) {  // empty clouds (torch gives null data pointers): every count is 0
        if (hipMemsetAsync(counts, 0, sizeof(int32_t) * nb, as_stream(stream)) != hipSuccess)
            return HREG_ERR_LAUNCH;
        return HREG_OK;
    }
    hipLaunchKernelGGL(range_filter_kernel, dim3(nb), dim3(RF_THREADS), 0, as_stream(stream), pts, intensity, n,
                       max_range, out, out_intensity, counts);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
