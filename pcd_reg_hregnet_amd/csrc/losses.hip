// losses.hip -- transformation_loss (losses/losses.py:97-164) and its metrics on the GPU.
//
// Per pair b (one thread each, pairs strided over one 256-thread block):
//   E = R_pred^T R_gt                                  (losses.py:117-123, 136)
//   resi_R = ||E - I||_F                               (losses.py:123)
//   euler  = matrix_to_euler_angles(E, "XYZ") in deg  (losses.py:139-140; pytorch3d 0.7.8
//            transforms/rotation_conversions.py: (atan2(-E12, E22), asin(E02), atan2(-E01, E00)))
//   geo    = deg(acos(clamp((tr E - 1) / 2, -1, 1)))   (losses.py:143-147)
//   dt     = t_pred - t_gt, eucl = ||dt||              (losses.py:153-159)
// then batch means with a fixed-order LDS tree (deterministic, no atomics):
//   scalars = {alpha * loss_R + loss_t, loss_R = mean resi_R, loss_t = mean eucl}
//   R_err[3] = mean |euler|, T_err[3] = mean |dt|.
#include "common.h"

namespace {

constexpr int LOSS_THREADS = 256;
constexpr int NSUM = 8;  // resi_R, eucl, |euler| x3, |dt| x3
constexpr float RAD2DEG = 57.29577951308232f;

__global__ void __launch_bounds__(LOSS_THREADS)
transformation_loss_kernel(const float *__restrict__ pR, const float *__restrict__ pt,
                           const float *__restrict__ gR, const float *__restrict__ gt, int nb,
                           float alpha, float *__restrict__ scalars, float *__restrict__ R_err,
                           float *__restrict__ T_err, float *__restrict__ geo,
                           float *__restrict__ eucl) {
    __shared__ float red[NSUM][LOSS_THREADS];
    float acc[NSUM];
#pragma unroll
    for (int s = 0; s < NSUM; ++s) acc[s] = 0.f;
    for (int b = threadIdx.x; b < nb; b += LOSS_THREADS) {
        const float *R = pR + (size_t)b * 9, *G = gR + (size_t)b * 9;
        float E[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                float s = 0.f;
                for (int q = 0; q < 3; ++q) s = fadd_rn(s, fmul_rn(R[q * 3 + i], G[q * 3 + j]));
                E[i][j] = s;
            }
        float fro = 0.f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                const float d = fsub_rn(E[i][j], i == j ? 1.f : 0.f);
                fro = fadd_rn(fro, fmul_rn(d, d));
            }
        acc[0] = fadd_rn(acc[0], sqrtf(fro));
        const float ex = atan2f(-E[1][2], E[2][2]);
        const float ey = asinf(E[0][2]);
        const float ez = atan2f(-E[0][1], E[0][0]);
        acc[2] = fadd_rn(acc[2], fabsf(fmul_rn(ex, RAD2DEG)));
        acc[3] = fadd_rn(acc[3], fabsf(fmul_rn(ey, RAD2DEG)));
        acc[4] = fadd_rn(acc[4], fabsf(fmul_rn(ez, RAD2DEG)));
        const float tr = fadd_rn(fadd_rn(E[0][0], E[1][1]), E[2][2]);
        const float c = fminf(fmaxf(fsub_rn(tr, 1.f) / 2.f, -1.f), 1.f);
        if (geo) geo[b] = fmul_rn(acosf(c), RAD2DEG);
        float n2 = 0.f;
        for (int q = 0; q < 3; ++q) {
            const float d = fsub_rn(pt[(size_t)b * 3 + q], gt[(size_t)b * 3 + q]);
            n2 = fadd_rn(n2, fmul_rn(d, d));
            acc[5 + q] = fadd_rn(acc[5 + q], fabsf(d));
        }
        const float e = sqrtf(n2);
        if (eucl) eucl[b] = e;
        acc[1] = fadd_rn(acc[1], e);
    }
#pragma unroll
    for (int s = 0; s < NSUM; ++s) red[s][threadIdx.x] = acc[s];
    __syncthreads();
    for (int w = LOSS_THREADS / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
#pragma unroll
            for (int s = 0; s < NSUM; ++s)
                red[s][threadIdx.x] = fadd_rn(red[s][threadIdx.x], red[s][threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float inv = (float)nb;
        const float loss_R = red[0][0] / inv, loss_t = red[1][0] / inv;
        if (scalars) {
            scalars[0] = fadd_rn(fmul_rn(alpha, loss_R), loss_t);
            scalars[1] = loss_R;
            scalars[2] = loss_t;
        }
        for (int q = 0; q < 3; ++q) {
            if (R_err) R_err[q] = red[2 + q][0] / inv;
            if (T_err) T_err[q] = red[5 + q][0] / inv;
        }
    }
}

}  // namespace

extern "C" int hreg_transformation_loss(const float *pred_R, const float *pred_t, const float *gt_R,
                                        const float *gt_t, int nb, float alpha, float *scalars,
                                        float *R_err, float *T_err, float *geodesic, float *eucl,
                                        void *stream) {
    if (!pred_R || !pred_t || !gt_R || !gt_t || nb <= 0) return HREG_ERR_INVALID;
    hipLaunchKernelGGL(transformation_loss_kernel, dim3(1), dim3(LOSS_THREADS), 0, as_stream(stream),
                       pred_R, pred_t, gt_R, gt_t, nb, alpha, scalars, R_err, T_err, geodesic, eucl);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// ---------------------------------------------------------------- calibration metrics
// CalibEval.add_batch (metrics/calibeval.py:72-113) per pair b (one thread each):
//   E = pred_tf . gt_tf (4 x 4, calibeval.py:83)
//   err_euler = deg(matrix_to_euler_angles(E[:3,:3], "XYZ")), err_t = E[:3,3]
//   pred_euler = deg(matrix_to_euler_angles(pred_tf[:3,:3])), pred_t = pred_tf[:3,3]
//   theta = deg(acos(clamp((tr E[:3,:3] - 1) / 2, -1, 1))), tnorm = ||E[:3,3]|| (:197-214)
// per_pair[b] = {err_euler 3, err_t 3, pred_euler 3, pred_t 3}; batch_geo = {mean theta,
// mean tnorm} with a fixed-order LDS tree (the reference's .mean().item()).
namespace {

__device__ __forceinline__ void euler_xyz_deg(const float (&M)[3][3], float *out) {
    out[0] = fmul_rn(atan2f(-M[1][2], M[2][2]), RAD2DEG);
    out[1] = fmul_rn(asinf(M[0][2]), RAD2DEG);
    out[2] = fmul_rn(atan2f(-M[0][1], M[0][0]), RAD2DEG);
}

__global__ void __launch_bounds__(LOSS_THREADS)
calib_metrics_kernel(const float *__restrict__ pred_tf, const float *__restrict__ gt_tf, int nb,
                     float *__restrict__ per_pair, float *__restrict__ batch_geo) {
    __shared__ float red[2][LOSS_THREADS];
    float th_sum = 0.f, tn_sum = 0.f;
    for (int b = threadIdx.x; b < nb; b += LOSS_THREADS) {
        const float *P = pred_tf + (size_t)b * 16, *G = gt_tf + (size_t)b * 16;
        float E[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                float s = 0.f;
                for (int q = 0; q < 4; ++q) s = fadd_rn(s, fmul_rn(P[i * 4 + q], G[q * 4 + j]));
                E[i][j] = s;
            }
        float Er[3][3], Pr[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                Er[i][j] = E[i][j];
                Pr[i][j] = P[i * 4 + j];
            }
        float *o = per_pair + (size_t)b * 12;
        euler_xyz_deg(Er, o);
        for (int q = 0; q < 3; ++q) o[3 + q] = E[q][3];
        euler_xyz_deg(Pr, o + 6);
        for (int q = 0; q < 3; ++q) o[9 + q] = P[q * 4 + 3];
        const float tr = fadd_rn(fadd_rn(E[0][0], E[1][1]), E[2][2]);
        const float c = fminf(fmaxf(fsub_rn(tr, 1.f) / 2.f, -1.f), 1.f);
        th_sum = fadd_rn(th_sum, fmul_rn(acosf(c), RAD2DEG));
        float n2 = 0.f;
        for (int q = 0; q < 3; ++q) n2 = fadd_rn(n2, fmul_rn(E[q][3], E[q][3]));
        tn_sum = fadd_rn(tn_sum, sqrtf(n2));
    }
    red[0][threadIdx.x] = th_sum;
    red[1][threadIdx.x] = tn_sum;
    __syncthreads();
    for (int w = LOSS_THREADS / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[0][threadIdx.x] = fadd_rn(red[0][threadIdx.x], red[0][threadIdx.x + w]);
            red[1][threadIdx.x] = fadd_rn(red[1][threadIdx.x], red[1][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        batch_geo[0] = red[0][0] / (float)nb;
        batch_geo[1] = red[1][0] / (float)nb;
    }
}

}  // namespace

extern "C" int hreg_calib_metrics(const float *pred_tf, const float *gt_tf, int nb, float *per_pair,
                                  float *batch_geo, void *stream) {
    if (!pred_tf || !gt_tf || !per_pair || !batch_geo || nb <= 0) return HREG_ERR_INVALID;
    hipLaunchKernelGGL(calib_metrics_kernel, dim3(1), dim3(LOSS_THREADS), 0, as_stream(stream), pred_tf,
                       gt_tf, nb, per_pair, batch_geo);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
