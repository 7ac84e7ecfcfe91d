// icp.hip -- point-to-point ICP refinement after the network (reference
// test/test_v4.py:140-158: open3d registration_icp from the finest predicted pose,
// max_correspondence_distance 1.0, TransformationEstimationPointToPoint,
// ICPConvergenceCriteria(relative_fitness 1e-6, relative_rmse 1e-6, max_iteration 2000)).
// open3d is not in this environment (parity unpinned against it); the algorithm is its
// published RegistrationICP loop:
//   result_0 = correspondences(T_0);  for i < max_iteration:
//     T_{i+1} = Kabsch(result_i) * T_i;  result_{i+1} = correspondences(T_{i+1});
//     stop when |fitness_{i+1} - fitness_i| < rel_fitness and |rmse_{i+1} - rmse_i| < rel_rmse;
//   correspondences: every source point's nearest target point strictly within the
//   distance (fitness = matches / n_src, inlier_rmse = sqrt(sum d^2 / matches)).
//
// MI355X layout: both clouds are spatially indexed once (knn.hip hreg_spatial_index:
// points sorted by Morton cell, a bounding box per 64 sorted points).  A wave owns 64
// consecutive sorted SOURCE points (a rigid motion keeps them together), transforms
// them (fp64 pose, fp32 search), and visits only the target blocks whose box lies within
// the radius of the wave's transformed bounding box (exact: the box-to-box bound uses the
// distance's own fp32 operations, so it never exceeds a member's computed distance);
// each candidate block is staged in the wave's LDS slot and read back as broadcasts.
// One workgroup per pair then reduces the matches in fp64 (two passes: means, then the
// cross-covariance), runs the 3x3 SVD (svd3.h) and the convergence test on the device,
// so the host only polls the done flags every few iterations.
#include "common.h"
#include "svd3.h"

namespace {

constexpr int ICP_WAVES = 4;
constexpr int ST_DOUBLES = 32;  // per pair: T[12] | prev fit, rmse | fit, rmse | iter, done, ...
// state layout (doubles): 0..11 T (row-major 3x4), 12 prev fitness, 13 prev rmse, 14 fitness,
// 15 rmse, 16 updates applied, 17 done (0 / 1), 18 matches
constexpr int S_PF = 12, S_PR = 13, S_F = 14, S_R = 15, S_IT = 16, S_DONE = 17, S_CNT = 18;

__host__ __device__ inline size_t np_of(int n) {
    size_t np = 64;
    while (np < (size_t)n) np <<= 1;
    return np;
}

struct Layout {
    const float4 *ss, *sb;  // source sorted points / boxes
    const float4 *ts, *tb;  // target
    int32_t *corr;          // [nb][np_src] target index per sorted source slot, -1 none
    double *state;          // [nb][ST_DOUBLES]
};

Layout layout_of(void *ws, int nb, int ns, int nt) {
    const size_t nps = np_of(ns), npt = np_of(nt);
    char *p = static_cast<char *>(ws);
    Layout L;
    L.ss = reinterpret_cast<const float4 *>(p);
    L.sb = L.ss + (size_t)nb * nps;
    p += (size_t)nb * (nps + nps / 64 * 2) * sizeof(float4);
    L.ts = reinterpret_cast<const float4 *>(p);
    L.tb = L.ts + (size_t)nb * npt;
    p += (size_t)nb * (npt + npt / 64 * 2) * sizeof(float4);
    L.corr = reinterpret_cast<int32_t *>(p);
    p += ((size_t)nb * nps * sizeof(int32_t) + 255) / 256 * 256;
    L.state = reinterpret_cast<double *>(p);
    return L;
}

__device__ __forceinline__ float wmin(float v) { return -wave_max_f32(-v); }

// p = R s + t in fp64 with a fixed operation order, rounded to fp32 for the search
__device__ __forceinline__ void xform(const double *T, float sx, float sy, float sz, double &px,
                                      double &py, double &pz) {
    const double x = sx, y = sy, z = sz;
    px = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[0], x), __dmul_rn(T[1], y)), __dmul_rn(T[2], z)), T[3]);
    py = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[4], x), __dmul_rn(T[5], y)), __dmul_rn(T[6], z)), T[7]);
    pz = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(T[8], x), __dmul_rn(T[9], y)), __dmul_rn(T[10], z)), T[11]);
}

// per-axis gap between two intervals (0 when they overlap), fp32 (monotone: never above
// the computed |q - p| of members)
__device__ __forceinline__ float gap(float alo, float ahi, float blo, float bhi) {
    return fmaxf(fmaxf(fsub_rn(blo, ahi), fsub_rn(alo, bhi)), 0.f);
}

__global__ __launch_bounds__(ICP_WAVES * 64) void icp_nn_kernel(Layout L, int nb, int ns, int nt,
                                                                float r2) {
    __shared__ float4 stage[ICP_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t nps = np_of(ns), npt = np_of(nt);
    const int sblk = (ns + 63) / 64, tblk = (nt + 63) / 64;
    const int pair = blockIdx.y;
    const int b = blockIdx.x * ICP_WAVES + w;
    if (b >= sblk) return;
    const double *T = L.state + (size_t)pair * ST_DOUBLES;
    if (T[S_DONE] != 0.0) return;
    const int i = b * 64 + lane;
    const bool valid = i < ns;
    const float4 s = L.ss[(size_t)pair * nps + (valid ? i : 0)];
    double px, py, pz;
    xform(T, s.x, s.y, s.z, px, py, pz);
    const float qx = (float)px, qy = (float)py, qz = (float)pz;
    const float inf = __builtin_huge_valf();
    const float lx = wmin(valid ? qx : inf), ly = wmin(valid ? qy : inf), lz = wmin(valid ? qz : inf);
    const float hx = wave_max_f32(valid ? qx : -inf), hy = wave_max_f32(valid ? qy : -inf),
                hz = wave_max_f32(valid ? qz : -inf);
    const float4 *TS = L.ts + (size_t)pair * npt;
    const float4 *TB = L.tb + (size_t)pair * (npt / 64) * 2;
    float best = inf;
    int bid = 0x7fffffff;
    for (int c0 = 0; c0 < tblk; c0 += 64) {
        const int c = c0 + lane;
        bool cand = false;
        if (c < tblk) {
            const float4 lo = TB[c * 2], hi = TB[c * 2 + 1];
            const float gx = gap(lx, hx, lo.x, hi.x), gy = gap(ly, hy, lo.y, hi.y), gz = gap(lz, hz, lo.z, hi.z);
            cand = fadd_rn(fadd_rn(fmul_rn(gx, gx), fmul_rn(gy, gy)), fmul_rn(gz, gz)) < r2;
        }
        uint64_t m = __ballot(cand);
        while (m) {
            const int blk = c0 + (int)__builtin_ctzll(m);
            m &= m - 1;
            const int j = blk * 64 + lane;
            stage[w][lane] = j < nt ? TS[j] : make_float4(inf, inf, inf, __int_as_float(0x7fffffff));
            __builtin_amdgcn_wave_barrier();
#pragma unroll 8
            for (int e = 0; e < 64; ++e) {
                const float4 t = stage[w][e];
                const float d = sqdist3(qx, qy, qz, t.x, t.y, t.z);
                const int id = __float_as_int(t.w);
                if (d < best || (d == best && id < bid)) { best = d; bid = id; }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (valid) L.corr[(size_t)pair * nps + i] = best < r2 ? bid : -1;
}

// one workgroup per pair: fitness / rmse of the current matches, the convergence test,
// and (not converged) the Kabsch update T <- [R_u | t_u] T
__global__ __launch_bounds__(256) void icp_update_kernel(Layout L, const float *__restrict__ tgt,
                                                         int nb, int ns, int nt, double rel_fit,
                                                         double rel_rmse, int max_iter) {
    __shared__ double red[4][16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int pair = blockIdx.x;
    const size_t nps = np_of(ns);
    double *T = L.state + (size_t)pair * ST_DOUBLES;
    if (T[S_DONE] != 0.0) return;
    const float4 *SS = L.ss + (size_t)pair * nps;
    const int32_t *C = L.corr + (size_t)pair * nps;
    const float *P = tgt + (size_t)pair * nt * 3;
    double Tl[12];
    for (int q = 0; q < 12; ++q) Tl[q] = T[q];
    auto block_sum = [&](double v[], int cnt) {
        for (int q = 0; q < cnt; ++q) v[q] = wave_sum_f64(v[q]);
        __syncthreads();
        if (lane == 0)
            for (int q = 0; q < cnt; ++q) red[wv][q] = v[q];
        __syncthreads();
        for (int q = 0; q < cnt; ++q) v[q] = ((red[0][q] + red[1][q]) + red[2][q]) + red[3][q];
        __syncthreads();
    };
    // pass 1: matches, sums of p and q, squared distances
    double m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < ns; i += blockDim.x) {
        const int j = C[i];
        if (j < 0) continue;
        const float4 s = SS[i];
        double px, py, pz;
        xform(Tl, s.x, s.y, s.z, px, py, pz);
        const double tx = P[j * 3], ty = P[j * 3 + 1], tz = P[j * 3 + 2];
        m[0] += 1.0;
        m[1] += px; m[2] += py; m[3] += pz;
        m[4] += tx; m[5] += ty; m[6] += tz;
        const double dx = px - tx, dy = py - ty, dz = pz - tz;
        m[7] += dx * dx + dy * dy + dz * dz;
    }
    block_sum(m, 8);
    const double cnt = m[0];
    const double fit = cnt / (double)ns;
    const double rmse = cnt > 0 ? sqrt(m[7] / cnt) : 0.0;
    const int it = (int)T[S_IT];
    bool done = it >= max_iter;
    if (it >= 1 && fabs(T[S_PF] - fit) < rel_fit && fabs(T[S_PR] - rmse) < rel_rmse) done = true;
    if (done) {
        if (threadIdx.x == 0) {
            T[S_F] = fit; T[S_R] = rmse; T[S_CNT] = cnt; T[S_DONE] = 1.0;
        }
        return;
    }
    double H[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    double ms[3] = {0, 0, 0}, mt[3] = {0, 0, 0};
    if (cnt > 0) {
        for (int d = 0; d < 3; ++d) { ms[d] = m[1 + d] / cnt; mt[d] = m[4 + d] / cnt; }
        double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = threadIdx.x; i < ns; i += blockDim.x) {
            const int j = C[i];
            if (j < 0) continue;
            const float4 s = SS[i];
            double p3[3];
            xform(Tl, s.x, s.y, s.z, p3[0], p3[1], p3[2]);
            const double a[3] = {p3[0] - ms[0], p3[1] - ms[1], p3[2] - ms[2]};
            const double c[3] = {P[j * 3] - mt[0], P[j * 3 + 1] - mt[1], P[j * 3 + 2] - mt[2]};
            for (int p = 0; p < 3; ++p)
                for (int q = 0; q < 3; ++q) h[p * 3 + q] += a[p] * c[q];
        }
        block_sum(h, 9);
        for (int p = 0; p < 3; ++p)
            for (int q = 0; q < 3; ++q) H[p][q] = h[p * 3 + q];
    }
    if (threadIdx.x != 0) return;
    double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, t[3] = {0, 0, 0};
    if (cnt > 0) {  // Kabsch (Eigen::umeyama without scaling): R = V diag(1,1,det) U^T
        double u[3][3], v[3][3], sig[3];
        const double d = svd3_usv(H, u, sig, v);
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
                R[a][b] = v[0][a] * u[0][b] + v[1][a] * u[1][b] + d * v[2][a] * u[2][b];
        for (int a = 0; a < 3; ++a) t[a] = mt[a] - (R[a][0] * ms[0] + R[a][1] * ms[1] + R[a][2] * ms[2]);
    }
    double Tn[12];
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b)
            Tn[a * 4 + b] = R[a][0] * Tl[b] + R[a][1] * Tl[4 + b] + R[a][2] * Tl[8 + b];
        Tn[a * 4 + 3] = R[a][0] * Tl[3] + R[a][1] * Tl[7] + R[a][2] * Tl[11] + t[a];
    }
    for (int q = 0; q < 12; ++q) T[q] = Tn[q];
    T[S_PF] = fit; T[S_PR] = rmse; T[S_F] = fit; T[S_R] = rmse; T[S_CNT] = cnt;
    T[S_IT] = (double)(it + 1);
}

__global__ void icp_init_kernel(double *state, const float *__restrict__ T0, int nb) {
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= nb) return;
    double *S = state + (size_t)pair * ST_DOUBLES;
    for (int q = 0; q < ST_DOUBLES; ++q) S[q] = 0.0;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 4; ++b) S[a * 4 + b] = T0 ? (double)T0[(size_t)pair * 16 + a * 4 + b] : (a == b ? 1.0 : 0.0);
}

__global__ void icp_result_kernel(const double *state, int nb, float *T_out, float *fitness,
                                  float *rmse, int32_t *iters, int32_t *done) {
    const int pair = blockIdx.x * blockDim.x + threadIdx.x;
    if (pair >= nb) return;
    const double *S = state + (size_t)pair * ST_DOUBLES;
    if (T_out) {
        float *o = T_out + (size_t)pair * 16;
        for (int q = 0; q < 12; ++q) o[q] = (float)S[q];
        o[12] = 0.f; o[13] = 0.f; o[14] = 0.f; o[15] = 1.f;
    }
    if (fitness) fitness[pair] = (float)S[S_F];
    if (rmse) rmse[pair] = (float)S[S_R];
    if (iters) iters[pair] = (int32_t)S[S_IT];
    if (done) done[pair] = S[S_DONE] != 0.0 ? 1 : 0;
}

}  // namespace

extern "C" size_t hreg_icp_ws_bytes(int nb, int n_src, int n_dst) {
    if (nb <= 0 || n_src <= 0 || n_dst <= 0) return 0;
    const size_t nps = np_of(n_src), npt = np_of(n_dst);
    return (size_t)nb * (nps + nps / 64 * 2) * sizeof(float4) +
           (size_t)nb * (npt + npt / 64 * 2) * sizeof(float4) +
           ((size_t)nb * nps * sizeof(int32_t) + 255) / 256 * 256 + (size_t)nb * ST_DOUBLES * sizeof(double);
}

// source [nb][n_src][3], target [nb][n_dst][3] fp32; T0 [nb][4][4] fp32 (null: identity)
extern "C" int hreg_icp_init(const float *src, const float *dst, int nb, int n_src, int n_dst,
                             const float *T0, void *ws, void *stream) {
    if (!src || !dst || !ws || nb < 0 || n_src <= 0 || n_dst <= 0) return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(ws) & 255)) return HREG_ERR_INVALID;
    if (nb == 0) return HREG_OK;
    Layout L = layout_of(ws, nb, n_src, n_dst);
    int rc = hreg_spatial_index(src, nb, n_src, const_cast<float4 *>(L.ss), stream);
    if (rc) return rc;
    rc = hreg_spatial_index(dst, nb, n_dst, const_cast<float4 *>(L.ts), stream);
    if (rc) return rc;
    hipLaunchKernelGGL(icp_init_kernel, dim3((nb + 63) / 64), dim3(64), 0, as_stream(stream), L.state, T0, nb);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// `iters` more ICP iterations (each: matches, then convergence test / Kabsch update) for
// every pair not done; all on the device, asynchronous
extern "C" int hreg_icp_iterate(const float *dst, int nb, int n_src, int n_dst, float max_corr_dist,
                                double rel_fitness, double rel_rmse, int max_iteration, int iters,
                                void *ws, void *stream) {
    if (!dst || !ws || nb < 0 || n_src <= 0 || n_dst <= 0 || iters < 0 || max_iteration < 0 ||
        !(max_corr_dist > 0.f))
        return HREG_ERR_INVALID;
    if (nb == 0 || iters == 0) return HREG_OK;
    Layout L = layout_of(ws, nb, n_src, n_dst);
    hipStream_t st = as_stream(stream);
    const float r2 = max_corr_dist * max_corr_dist;
    const int sblk = (n_src + 63) / 64;
    const dim3 grid((sblk + ICP_WAVES - 1) / ICP_WAVES, nb);
    for (int k = 0; k < iters; ++k) {
        hipLaunchKernelGGL(icp_nn_kernel, grid, dim3(ICP_WAVES * 64), 0, st, L, nb, n_src, n_dst, r2);
        hipLaunchKernelGGL(icp_update_kernel, dim3(nb), dim3(256), 0, st, L, dst, nb, n_src, n_dst,
                           rel_fitness, rel_rmse, max_iteration);
    }
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// T_out [nb][4][4], fitness / inlier_rmse [nb] (float), iterations applied and done flags
// [nb] (int32); any output may be null
extern "C" int hreg_icp_result(const void *ws, int nb, int n_src, int n_dst, float *T_out, float *fitness,
                               float *inlier_rmse, int32_t *iterations, int32_t *done, void *stream) {
    if (!ws || nb < 0 || n_src <= 0 || n_dst <= 0) return HREG_ERR_INVALID;
    if (nb == 0) return HREG_OK;
    Layout L = layout_of(const_cast<void *>(ws), nb, n_src, n_dst);
    hipLaunchKernelGGL(icp_result_kernel, dim3((nb + 63) / 64), dim3(64), 0, as_stream(stream), L.state, nb,
                       T_out, fitness, inlier_rmse, iterations, done);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
