// heads.hip -- attentive pooling, group max, output heads, similarity
// gathering, correspondence feature rows, weighted SVD and point transforms.
#include "common.h"
#include "svd3.h"

namespace {

constexpr int WAVES = 4;

// ------------------------------------------------------------------ attend
// One wave per group of k (<= 64) rows (layers.py:150-159, 329-337, 384-390,
// 446-450): a = softmax_k(max_c logits), att[c] = sum_j fl(V[j][c] * a_j),
// kp = sum_j a_j * xyz_j.  Sums over j run in order j = 0..k-1.
__global__ __launch_bounds__(256) void attend_kernel(
    const float *__restrict__ logits, int C, int ldl, int G, int k, float *__restrict__ attw,
    const float *__restrict__ vals, const int32_t *__restrict__ vgather, int Cv, int ldv,
    float *__restrict__ att, int ldatt, const float *__restrict__ xyz_rows, float *__restrict__ kp) {
    __shared__ float sa[WAVES][64];
    __shared__ int srow[WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = blockIdx.x * WAVES + w;
    if (g >= G) return;
    const size_t r = (size_t)g * k + lane;
    float x1 = -__builtin_huge_valf();
    if (lane < k) {
        const float *row = logits + r * ldl;
        int c = 0;
        if ((ldl & 3) == 0) {
            for (; c + 4 <= C; c += 4) {
                const float4 v = *reinterpret_cast<const float4 *>(row + c);
                x1 = fmaxf(fmaxf(x1, v.x), fmaxf(v.y, fmaxf(v.z, v.w)));
            }
        }
        for (; c < C; ++c) x1 = fmaxf(x1, row[c]);
    }
    const float mx = wave_max_f32(x1);
    const float e = lane < k ? expf(fsub_rn(x1, mx)) : 0.f;
    const float s = wave_sum_f32(e);
    const float a = lane < k ? e / s : 0.f;
    if (attw && lane < k) attw[r] = a;
    if (kp) {
        float px = 0.f, py = 0.f, pz = 0.f;
        if (lane < k) {
            px = fmul_rn(a, xyz_rows[r * 3 + 0]);
            py = fmul_rn(a, xyz_rows[r * 3 + 1]);
            pz = fmul_rn(a, xyz_rows[r * 3 + 2]);
        }
        px = wave_sum_f32(px);
        py = wave_sum_f32(py);
        pz = wave_sum_f32(pz);
        if (lane == 0) {
            kp[(size_t)g * 3 + 0] = px;
            kp[(size_t)g * 3 + 1] = py;
            kp[(size_t)g * 3 + 2] = pz;
        }
    }
    if (att) {
        sa[w][lane] = a;
        srow[w][lane] = lane < k ? (vgather ? vgather[r] : (int)r) : 0;
        wave_sync();
        for (int c = lane; c < Cv; c += 64) {
            float t = 0.f;
            for (int j = 0; j < k; ++j)
                t = fadd_rn(t, fmul_rn(vals[(size_t)srow[w][j] * ldv + c], sa[w][j]));
            att[(size_t)g * ldatt + c] = t;
        }
    }
}

// --------------------------------------------------------------- group max
__global__ void group_max_kernel(const float *__restrict__ x, int G, int k, int C, int ldx,
                                 float *__restrict__ out, int ldo) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (size_t)G * C) return;
    const size_t g = e / C;
    const int c = (int)(e % C);
    const float *p = x + g * k * ldx + c;
    float m = p[0];
    for (int j = 1; j < k; ++j) m = fmaxf(m, p[(size_t)j * ldx]);
    out[g * ldo + c] = m;
}

// ---------------------------------------------------------------- head out
// z = dot(x[r], w3) + b3 (mlp3 Conv1d(C,1), layers.py:130/268/431), then
// softplus(z) + 0.001 (layers.py:161-163) or sigmoid(z) (layers.py:393-394).
// One wave per row over the whole grid.
__global__ __launch_bounds__(256) void head_out_kernel(const float *__restrict__ x, int C, int ldx,
                                                       int R, const float *__restrict__ w3,
                                                       const float *__restrict__ b3, int mode,
                                                       float *__restrict__ out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * WAVES + w;
    if (r >= R) return;
    const float *row = x + (size_t)r * ldx;
    float t = 0.f;
    for (int c = lane; c < C; c += 64) t = fadd_rn(t, fmul_rn(row[c], w3[c]));
    t = wave_sum_f32(t);
    const float z = fadd_rn(t, b3[0]);
    float o;
    if (mode == HREG_HEAD_SOFTPLUS) {
        const float sp = z > 20.f ? z : log1pf(expf(z));
        o = fadd_rn(sp, 0.001f);
    } else {
        o = 1.0f / fadd_rn(1.0f, expf(-z));
    }
    if (lane == 0) out[r] = o;
}

// weights = (1/(sigma+1e-5)) / mean_cloud(1/(sigma+1e-5)) (models.py:30-32); block per cloud
__global__ __launch_bounds__(256) void sigma_weights_kernel(const float *__restrict__ sig, int rows,
                                                            float *__restrict__ wout) {
    __shared__ float red[WAVES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float *s = sig + (size_t)blockIdx.x * rows;
    float part = 0.f;
    for (int i = threadIdx.x; i < rows; i += blockDim.x)
        part = fadd_rn(part, 1.0f / fadd_rn(s[i], 1e-5f));
    part = wave_sum_f32(part);
    if (lane == 0) red[w] = part;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < WAVES; ++i) tot = fadd_rn(tot, red[i]);
    const float mean = tot / (float)rows;
    float *o = wout + (size_t)blockIdx.x * rows;
    for (int i = threadIdx.x; i < rows; i += blockDim.x) o[i] = (1.0f / fadd_rn(s[i], 1e-5f)) / mean;
}

// --------------------------------------------------------------- row norms
__global__ __launch_bounds__(256) void row_norms_kernel(const float *__restrict__ x, int R, int C,
                                                        int ldx, float *__restrict__ norms) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * WAVES + w;
    if (r >= R) return;
    float t = 0.f;
    for (int c = lane; c < C; c += 64) {
        const float v = x[(size_t)r * ldx + c];
        t = fadd_rn(t, fmul_rn(v, v));
    }
    t = wave_sum_f32(t);
    if (lane == 0) norms[r] = sqrtf(t);
}

// -------------------------------------------------------------- sim gather
// layers.py:296-313: per pair, row max over n and column max over i of S,
// then (S[i][n]/(rowmax_i+1e-6), S[i][n]/(colmax_n+1e-6)) at n = kidx[i][j].
// maxes [nb][N1 + N2] = (rowmax, colmax).
__global__ __launch_bounds__(256) void sim_rowmax_kernel(const float *__restrict__ S, int nb, int N1,
                                                         int N2, float *__restrict__ maxes) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * WAVES + w;  // global row b*N1 + i
    if (r >= nb * N1) return;
    const float *row = S + (size_t)r * N2;
    float m = -__builtin_huge_valf();
    for (int n = lane; n < N2; n += 64) m = fmaxf(m, row[n]);
    m = wave_max_f32(m);
    if (lane == 0) maxes[(size_t)(r / N1) * (N1 + N2) + (r % N1)] = m;
}

__global__ __launch_bounds__(256) void sim_colmax_kernel(const float *__restrict__ S, int N1, int N2,
                                                         float *__restrict__ maxes) {
    __shared__ float part[4][64];
    const int b = blockIdx.y;
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int g = threadIdx.x >> 6;
    const float *Sb = S + (size_t)b * N1 * N2;
    float m = -__builtin_huge_valf();
    // (unrolled: the loads of 16 rows issue together instead of one L2 round trip per row; the
    // maxima still run in row order)
    if (c < N2) {
#pragma unroll 16
        for (int i = g; i < N1; i += 4) m = fmaxf(m, Sb[(size_t)i * N2 + c]);
    }
    part[g][threadIdx.x & 63] = m;
    __syncthreads();
    if (g == 0 && c < N2) {
        const int l = threadIdx.x;
        maxes[(size_t)b * (N1 + N2) + N1 + c] =
            fmaxf(fmaxf(part[0][l], part[1][l]), fmaxf(part[2][l], part[3][l]));
    }
}

__global__ void sim_gather_kernel(const float *__restrict__ S, int nb, int N1, int N2,
                                  const int32_t *__restrict__ kidx, int k,
                                  const float *__restrict__ maxes, float *__restrict__ sims,
                                  int ld_sims) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (size_t)nb * N1 * k) return;
    const size_t bi = e / k;  // b*N1 + i
    const int b = (int)(bi / N1), i = (int)(bi % N1);
    const int n = kidx[e];
    const float s = S[bi * N2 + n];
    const float *mx = maxes + (size_t)b * (N1 + N2);
    float *o = sims + e * ld_sims;
    o[0] = s / fadd_rn(mx[i], 1e-6f);
    o[1] = s / fadd_rn(mx[N1 + n], 1e-6f);
}

// -------------------------------------------------------------- pair feats
// Correspondence feature rows with the reference's geometry/weight/similarity
// channels (layers.py:279-288, 364-370 coarse; :434-445 fine), packed first so
// the GEMM reads one 16-float segment: [p-q, |p-q|, q, p, w_q, w_p, sims(4)].
__global__ void pair_feats_kernel(const float *__restrict__ src_xyz,
                                  const float *__restrict__ dst_xyz,
                                  const float *__restrict__ src_w, const float *__restrict__ dst_w,
                                  const int32_t *__restrict__ kidx, int nb, int M, int N, int k,
                                  const float *__restrict__ sims_a,
                                  const float *__restrict__ sims_b, float *__restrict__ feats,
                                  int ldf, float *__restrict__ knn_xyz,
                                  int32_t *__restrict__ gidx) {
    const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)nb * M * k;
    if (r >= total) return;
    const size_t bi = r / k;  // b*M + i
    const int b = (int)(bi / M);
    const int n = kidx[r];
    const size_t pn = (size_t)b * N + n;
    const float qx = src_xyz[bi * 3], qy = src_xyz[bi * 3 + 1], qz = src_xyz[bi * 3 + 2];
    const float px = dst_xyz[pn * 3], py = dst_xyz[pn * 3 + 1], pz = dst_xyz[pn * 3 + 2];
    const float rx = fsub_rn(px, qx), ry = fsub_rn(py, qy), rz = fsub_rn(pz, qz);
    const float d = sqrtf(fadd_rn(fadd_rn(fmul_rn(rx, rx), fmul_rn(ry, ry)), fmul_rn(rz, rz)));
    float *f = feats + r * ldf;
    f[0] = rx; f[1] = ry; f[2] = rz; f[3] = d;
    f[4] = qx; f[5] = qy; f[6] = qz;
    f[7] = px; f[8] = py; f[9] = pz;
    f[10] = src_w[bi];
    f[11] = dst_w[pn];
    if (ldf >= 16) {
        f[12] = sims_a ? sims_a[r * 2 + 0] : 0.f;
        f[13] = sims_a ? sims_a[r * 2 + 1] : 0.f;
        f[14] = sims_b ? sims_b[r * 2 + 0] : 0.f;
        f[15] = sims_b ? sims_b[r * 2 + 1] : 0.f;
    }
    if (knn_xyz) { knn_xyz[r * 3] = px; knn_xyz[r * 3 + 1] = py; knn_xyz[r * 3 + 2] = pz; }
    if (gidx) gidx[r] = (int32_t)pn;
}

// -------------------------------------------------------------- weighted SVD
// layers.py:469-504 in fp64: w <- w/(sum w + 1e-4); mu = sum w x / (sum w + 1e-4);
// H = sum w (s - mu_s)(c - mu_c)^T; H = U S V^T; R = V diag(1,1,det(V U^T)) U^T;
// t = mu_c - R mu_s.  A non-finite H marks the pair (R_[0] = NaN) and the
// batch kernel below turns the whole batch into R = I, t = 0 (layers.py:485-493).
__device__ void svd_rotation(const double H[3][3], double R[3][3]) {
    double u[3][3], v[3][3], sig[3];
    const double d = svd3_usv(H, u, sig, v);
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b)
            R[a][b] = v[0][a] * u[0][b] + v[1][a] * u[1][b] + d * v[2][a] * u[2][b];
}

__global__ __launch_bounds__(256) void svd_pair_kernel(const float *__restrict__ src,
                                                       const float *__restrict__ cor,
                                                       const float *__restrict__ w, int n,
                                                       float *__restrict__ R_out,
                                                       float *__restrict__ t_out) {
    __shared__ double red[WAVES][16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const float *S = src + (size_t)b * n * 3;
    const float *Cc = cor + (size_t)b * n * 3;
    const float *W = w + (size_t)b * n;
    auto block_sum = [&](double v[], int cnt) {
        for (int q = 0; q < cnt; ++q) v[q] = wave_sum_f64(v[q]);
        __syncthreads();
        if (lane == 0)
            for (int q = 0; q < cnt; ++q) red[wv][q] = v[q];
        __syncthreads();
        for (int q = 0; q < cnt; ++q) v[q] = red[0][q] + red[1][q] + red[2][q] + red[3][q];
        __syncthreads();
    };
    double v1[1] = {0.0};
    for (int i = threadIdx.x; i < n; i += blockDim.x) v1[0] += (double)W[i];
    block_sum(v1, 1);
    const double sw = v1[0] + 1e-4;
    double m[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double wi = (double)W[i] / sw;
        m[0] += wi;
        for (int d = 0; d < 3; ++d) {
            m[1 + d] += wi * (double)S[i * 3 + d];
            m[4 + d] += wi * (double)Cc[i * 3 + d];
        }
    }
    block_sum(m, 7);
    const double den = m[0] + 1e-4;
    const double ms[3] = {m[1] / den, m[2] / den, m[3] / den};
    const double mc[3] = {m[4] / den, m[5] / den, m[6] / den};
    double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double wi = (double)W[i] / sw;
        double a[3], c[3];
        for (int d = 0; d < 3; ++d) {
            a[d] = (double)S[i * 3 + d] - ms[d];
            c[d] = (double)Cc[i * 3 + d] - mc[d];
        }
        for (int p = 0; p < 3; ++p)
            for (int q = 0; q < 3; ++q) h[p * 3 + q] += a[p] * wi * c[q];
    }
    block_sum(h, 9);
    if (threadIdx.x != 0) return;
    bool finite = true;
    for (int q = 0; q < 9; ++q) finite = finite && isfinite(h[q]);
    for (int q = 0; q < 3; ++q) finite = finite && isfinite(ms[q]) && isfinite(mc[q]);
    float *Ro = R_out + (size_t)b * 9;
    float *to = t_out + (size_t)b * 3;
    if (!finite) {
        Ro[0] = __builtin_nanf("");
        return;
    }
    double H[3][3], R[3][3];
    for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) H[p][q] = h[p * 3 + q];
    svd_rotation(H, R);
    for (int p = 0; p < 3; ++p) {
        for (int q = 0; q < 3; ++q) Ro[p * 3 + q] = (float)R[p][q];
        to[p] = (float)(mc[p] - (R[p][0] * ms[0] + R[p][1] * ms[1] + R[p][2] * ms[2]));
    }
}

// one workgroup per group of `group` consecutive pairs (the reference's batch: its identity
// fallback resets the whole batch it ran, layers.py:485-493; a forward of several batches
// merged into one launch set keeps each batch's own fallback)
// tr_xyz (hreg_weighted_svd_tr): then the group's point sets [b][tr_n][3] are moved by the pair's
// final R, t into tr_out, with transform_kernel's arithmetic (one launch less per FineReg stage)
__device__ __forceinline__ void transform_point(const float *Rb, const float *tb, const float *p, float *o) {
    const float x = p[0], y = p[1], z = p[2];
    for (int i = 0; i < 3; ++i) {
        const float s = fadd_rn(fadd_rn(fmul_rn(Rb[i * 3], x), fmul_rn(Rb[i * 3 + 1], y)), fmul_rn(Rb[i * 3 + 2], z));
        o[i] = fadd_rn(s, tb[i]);
    }
}

__global__ void svd_batch_kernel(int nb, int group, float *__restrict__ R_, float *__restrict__ t_,
                                 const float *__restrict__ pR, const float *__restrict__ pt,
                                 float *__restrict__ R, float *__restrict__ t,
                                 const float *__restrict__ tr_xyz = nullptr, int tr_n = 0,
                                 float *__restrict__ tr_out = nullptr) {
    __shared__ int bad;
    const int b0 = blockIdx.x * group, b1 = min(b0 + group, nb);
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    for (int b = b0 + threadIdx.x; b < b1; b += blockDim.x)
        if (!(R_[(size_t)b * 9] == R_[(size_t)b * 9])) atomicOr(&bad, 1);
    __syncthreads();
    for (int b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
        float *Rb = R_ + (size_t)b * 9, *tb = t_ + (size_t)b * 3;
        if (bad) {
            for (int q = 0; q < 9; ++q) Rb[q] = (q % 4 == 0) ? 1.f : 0.f;
            tb[0] = tb[1] = tb[2] = 0.f;
        }
        if (pR && R) {  // T = T_ @ T_prev (models.py:108-110, 125-127)
            const float *P = pR + (size_t)b * 9, *pv = pt + (size_t)b * 3;
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) {
                    float s = 0.f;
                    for (int q = 0; q < 3; ++q) s = fadd_rn(s, fmul_rn(Rb[i * 3 + q], P[q * 3 + j]));
                    R[(size_t)b * 9 + i * 3 + j] = s;
                }
                float s = 0.f;
                for (int q = 0; q < 3; ++q) s = fadd_rn(s, fmul_rn(Rb[i * 3 + q], pv[q]));
                t[(size_t)b * 3 + i] = fadd_rn(s, tb[i]);
            }
        } else if (R) {
            for (int q = 0; q < 9; ++q) R[(size_t)b * 9 + q] = Rb[q];
            for (int q = 0; q < 3; ++q) t[(size_t)b * 3 + q] = tb[q];
        }
    }
    if (!tr_xyz) return;
    __syncthreads();  // the group's final R, t (written above by other threads) are visible
    const float *Rf = R ? R : R_, *tf = R ? t : t_;
    for (size_t e = (size_t)b0 * tr_n + threadIdx.x; e < (size_t)b1 * tr_n; e += blockDim.x) {
        const size_t b = e / tr_n;
        transform_point(Rf + b * 9, tf + b * 3, tr_xyz + e * 3, tr_out + e * 3);
    }
}

// ---------------------------------------------------------------- transform
__global__ void transform_kernel(const float *__restrict__ xyz, const float *__restrict__ R,
                                 const float *__restrict__ t, int n, size_t total,
                                 float *__restrict__ out) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const size_t b = e / n;
    const float *Rb = R + b * 9, *tb = t + b * 3;
    transform_point(Rb, tb, xyz + e * 3, out + e * 3);
}

// ------------------------------------------------------- gather (point_utils)
// gather_points_kernel_fast (.cu:7-21) / gather_points_grad_kernel_fast (.cu:41-55)
__global__ void gather_points_kernel(int c, int n, int m, const float *__restrict__ pts,
                                     const int32_t *__restrict__ idx, float *__restrict__ out) {
    const int b = blockIdx.z, ch = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    out[((size_t)b * c + ch) * m + j] = pts[((size_t)b * c + ch) * n + idx[(size_t)b * m + j]];
}

__global__ void gather_points_grad_kernel(int c, int n, int m, const float *__restrict__ go,
                                          const int32_t *__restrict__ idx, float *__restrict__ gp) {
    const int b = blockIdx.z, ch = blockIdx.y;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    atomicAdd(gp + ((size_t)b * c + ch) * n + idx[(size_t)b * m + j], go[((size_t)b * c + ch) * m + j]);
}

}  // namespace

extern "C" int hreg_attend(const float *logits_src, int C, int ldl, int G, int k, float *attw,
                           const float *vals, const int32_t *vgather, int Cv, int ldv, float *att,
                           int ldatt, const float *xyz_rows, float *kp, void *stream) {
    if (!logits_src || C <= 0 || ldl < C || G < 0 || k <= 0) return HREG_ERR_INVALID;
    if (k > 64) return HREG_ERR_UNSUPPORTED;
    if (att && (!vals || Cv <= 0 || ldv < Cv || ldatt < Cv)) return HREG_ERR_INVALID;
    if (kp && !xyz_rows) return HREG_ERR_INVALID;
    if (G == 0) return HREG_OK;
    hipLaunchKernelGGL(attend_kernel, dim3((G + WAVES - 1) / WAVES), dim3(256), 0,
                       as_stream(stream), logits_src, C, ldl, G, k, attw, vals, vgather, Cv, ldv,
                       att, ldatt, xyz_rows, kp);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_max(const float *x, int G, int k, int C, int ldx, float *out, int ldo,
                              void *stream) {
    if (!x || !out || G < 0 || k <= 0 || C <= 0 || ldx < C || ldo < C) return HREG_ERR_INVALID;
    const size_t total = (size_t)G * C;
    if (!total) return HREG_OK;
    hipLaunchKernelGGL(group_max_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       as_stream(stream), x, G, k, C, ldx, out, ldo);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_head_out(const float *x, int C, int ldx, int nclouds, int rows_per_cloud,
                             const float *w3, const float *b3, int mode, float *out,
                             float *weights_out, void *stream) {
    if (!x || !w3 || !b3 || !out || C <= 0 || ldx < C || nclouds < 0 || rows_per_cloud <= 0)
        return HREG_ERR_INVALID;
    if (mode != HREG_HEAD_SOFTPLUS && mode != HREG_HEAD_SIGMOID) return HREG_ERR_INVALID;
    if (weights_out && mode != HREG_HEAD_SOFTPLUS) return HREG_ERR_INVALID;
    if (!nclouds) return HREG_OK;
    const int R = nclouds * rows_per_cloud;
    hipLaunchKernelGGL(head_out_kernel, dim3((R + WAVES - 1) / WAVES), dim3(256), 0,
                       as_stream(stream), x, C, ldx, R, w3, b3, mode, out);
    HREG_CHECK_LAUNCH();
    if (weights_out) {
        hipLaunchKernelGGL(sigma_weights_kernel, dim3(nclouds), dim3(256), 0, as_stream(stream),
                           out, rows_per_cloud, weights_out);
        HREG_CHECK_LAUNCH();
    }
    return HREG_OK;
}

extern "C" int hreg_sigma_weights(const float *sigma, int nclouds, int rows_per_cloud, float *weights,
                                  void *stream) {
    if (!sigma || !weights || nclouds < 0 || rows_per_cloud <= 0) return HREG_ERR_INVALID;
    if (!nclouds) return HREG_OK;
    hipLaunchKernelGGL(sigma_weights_kernel, dim3(nclouds), dim3(256), 0, as_stream(stream), sigma,
                       rows_per_cloud, weights);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_row_norms(const float *x, int R, int C, int ldx, float *norms, void *stream) {
    if (!x || !norms || R < 0 || C <= 0 || ldx < C) return HREG_ERR_INVALID;
    if (!R) return HREG_OK;
    hipLaunchKernelGGL(row_norms_kernel, dim3((R + WAVES - 1) / WAVES), dim3(256), 0,
                       as_stream(stream), x, R, C, ldx, norms);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_sim_gather(const float *S, int nb, int N1, int N2, const int32_t *kidx, int k,
                               float *maxes, float *sims, int ld_sims, void *stream) {
    if (!S || !kidx || !sims || !maxes || nb < 0 || N1 <= 0 || N2 <= 0 || k <= 0 || ld_sims < 2)
        return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(sim_rowmax_kernel, dim3((nb * N1 + WAVES - 1) / WAVES), dim3(256), 0, st, S,
                       nb, N1, N2, maxes);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sim_colmax_kernel, dim3((N2 + 63) / 64, nb), dim3(256), 0, st, S, N1, N2,
                       maxes);
    HREG_CHECK_LAUNCH();
    const size_t total = (size_t)nb * N1 * k;
    hipLaunchKernelGGL(sim_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, S,
                       nb, N1, N2, kidx, k, maxes, sims, ld_sims);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_pair_feats(const float *src_xyz, const float *dst_xyz, const float *src_w,
                               const float *dst_w, const int32_t *kidx, int nb, int M, int N, int k,
                               const float *sims_a, const float *sims_b, float *feats, int ldf,
                               float *knn_xyz, int32_t *gidx, void *stream) {
    if (!src_xyz || !dst_xyz || !src_w || !dst_w || !kidx || !feats || nb < 0 || M < 0 || N <= 0 ||
        k <= 0 || ldf < 12)
        return HREG_ERR_INVALID;
    const size_t total = (size_t)nb * M * k;
    if (!total) return HREG_OK;
    hipLaunchKernelGGL(pair_feats_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       as_stream(stream), src_xyz, dst_xyz, src_w, dst_w, kidx, nb, M, N, k,
                       sims_a, sims_b, feats, ldf, knn_xyz, gidx);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_weighted_svd_grouped(const float *src, const float *corres, const float *w, int nb,
                                         int group, int n, const float *prev_R, const float *prev_t, float *R_,
                                         float *t_, float *R, float *t, void *stream) {
    if (!src || !corres || !w || !R_ || !t_ || nb < 0 || n <= 0 || group <= 0) return HREG_ERR_INVALID;
    if ((prev_R == nullptr) != (prev_t == nullptr)) return HREG_ERR_INVALID;
    if ((R == nullptr) != (t == nullptr)) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(svd_pair_kernel, dim3(nb), dim3(256), 0, st, src, corres, w, n, R_, t_);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(svd_batch_kernel, dim3((nb + group - 1) / group), dim3(256), 0, st, nb, group, R_, t_,
                       prev_R, prev_t, R, t);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_weighted_svd_tr(const float *src, const float *corres, const float *w, int nb, int group,
                                    int n, const float *prev_R, const float *prev_t, float *R_, float *t_,
                                    float *R, float *t, const float *tr_xyz, int tr_n, float *tr_out,
                                    void *stream) {
    if (!src || !corres || !w || !R_ || !t_ || nb < 0 || n <= 0 || group <= 0) return HREG_ERR_INVALID;
    if ((prev_R == nullptr) != (prev_t == nullptr)) return HREG_ERR_INVALID;
    if ((R == nullptr) != (t == nullptr)) return HREG_ERR_INVALID;
    if (!tr_xyz || !tr_out || tr_n <= 0) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(svd_pair_kernel, dim3(nb), dim3(256), 0, st, src, corres, w, n, R_, t_);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(svd_batch_kernel, dim3((nb + group - 1) / group), dim3(256), 0, st, nb, group, R_, t_,
                       prev_R, prev_t, R, t, tr_xyz, tr_n, tr_out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_weighted_svd(const float *src, const float *corres, const float *w, int nb,
                                 int n, const float *prev_R, const float *prev_t, float *R_,
                                 float *t_, float *R, float *t, void *stream) {
    return hreg_weighted_svd_grouped(src, corres, w, nb, nb > 0 ? nb : 1, n, prev_R, prev_t, R_, t_, R, t,
                                     stream);
}

extern "C" int hreg_transform_points(const float *xyz, const float *R, const float *t, int nb,
                                     int n, float *out, void *stream) {
    if (!xyz || !R || !t || !out || nb < 0 || n < 0) return HREG_ERR_INVALID;
    const size_t total = (size_t)nb * n;
    if (!total) return HREG_OK;
    hipLaunchKernelGGL(transform_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       as_stream(stream), xyz, R, t, n, total, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_gather_points(int b, int c, int n, int npoints, const float *points,
                                  const int32_t *idx, float *out, void *stream) {
    if (!points || !idx || !out || b < 0 || c < 0 || n <= 0 || npoints < 0) return HREG_ERR_INVALID;
    if (!b || !c || !npoints) return HREG_OK;
    dim3 grid((npoints + 255) / 256, c, b);
    hipLaunchKernelGGL(gather_points_kernel, grid, dim3(256), 0, as_stream(stream), c, n, npoints,
                       points, idx, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_gather_points_grad(int b, int c, int n, int npoints, const float *grad_out,
                                       const int32_t *idx, float *grad_points, void *stream) {
    if (!grad_out || !idx || !grad_points || b < 0 || c < 0 || n <= 0 || npoints < 0)
        return HREG_ERR_INVALID;
    if (!b || !c || !npoints) return HREG_OK;
    dim3 grid((npoints + 255) / 256, c, b);
    hipLaunchKernelGGL(gather_points_grad_kernel, grid, dim3(256), 0, as_stream(stream), c, n,
                       npoints, grad_out, idx, grad_points);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" const char *hreg_version(void) { return "hregnet_amd gfx950 r1"; }
