// train_ops.hip -- forward/backward kernels of the HRegNet training step
// (BASELINE configs[3]: train_reg_v0.py:241-296).
//
// The training graph keeps the reference's layer structure (train-mode BatchNorm
// needs batch statistics between every conv, so the eval-mode fused kernels do not
// apply) and runs every op of it here; pcd_reg_hregnet_amd/train_graph.py wires
// them into torch.autograd.Function objects.  Layout: activations are point-major
// rows [rows][channels]; the rows of a group of k neighbours are consecutive.
//
//   copy_rows / group_sum        cat / split, repeat over k and its backward
//   gather_rows, csr + scatter   knn_gather / gather_operation (layers.py:20-26,
//                                139-143) and their backward, deterministic: the
//                                backward sums each source row's contributions in
//                                ascending destination order (the reference's
//                                gather_points_grad_kernel uses atomicAdd, .cu:41-73)
//   geom_rows                    [knn_xyz - q, |knn_xyz - q|] (layers.py:21-23, 284-285)
//   attention                    max over channels -> softmax over k -> attentive sums
//                                (layers.py:151-159, 384-388, 447-450, 340-343)
//   group_max_arg                torch.max over k (layers.py:202, 208) with its argmax
//   head_out_bwd                 mlp3 + softplus(+0.001) / sigmoid backward
//   sim_*                        max-normalised cosine similarity gathered at the
//                                descriptor kNN (layers.py:290-313, 345-362), backward
//                                through the row/column maxima and the norms
//   weighted_svd_bwd             WeightedSVDHead (layers.py:469-504) backward, fp64,
//                                torch.svd's backward formula + det() of the reflection fix
//   transform / compose          R x + t (models.py:91-92, 113-114) and T_ @ T_prev
//                                (models.py:100-110, 120-127)
//   transformation_loss_bwd      losses.py:117-160 (alpha * mean |R^T R_gt - I|_F + mean |dt|)
#include "common.h"
#include "svd3.h"

namespace {

constexpr int TB = 256;

inline unsigned g1d(size_t n) {
    size_t b = (n + TB - 1) / TB;
    if (b > (1u << 20)) b = (1u << 20);
    return (unsigned)(b ? b : 1);
}

#define GRID_STRIDE(i, total) \
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (total); \
         i += (size_t)gridDim.x * blockDim.x)

// ------------------------------------------------------------ copies / sums
__global__ void copy_rows_kernel(const float *__restrict__ src, int lds, int row_div, int R, int C,
                                 float *__restrict__ dst, int ldd, int acc) {
    GRID_STRIDE(i, (size_t)R * C) {
        const int r = (int)(i / C), c = (int)(i % C);
        const float v = src[(size_t)(r / row_div) * lds + c];
        float *o = dst + (size_t)r * ldd + c;
        *o = acc ? fadd_rn(*o, v) : v;
    }
}

// float4 form (C, lds, ldd multiples of 4, 16-byte aligned rows, R * C / 4 < 2^31): four
// channels per thread, 32-bit index arithmetic; the same per-element operations
template <bool ACC>
__global__ __launch_bounds__(TB) void copy_rows4_kernel(const float4 *__restrict__ src, int lds4,
                                                        int row_div, int R, int C4,
                                                        float4 *__restrict__ dst, int ldd4) {
    const uint32_t total = (uint32_t)R * (uint32_t)C4;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const uint32_t r = i / (uint32_t)C4, c = i - r * (uint32_t)C4;
        const float4 v = src[(size_t)(r / (uint32_t)row_div) * lds4 + c];
        float4 *o = dst + (size_t)r * ldd4 + c;
        if (ACC) {
            const float4 a = *o;
            *o = make_float4(fadd_rn(a.x, v.x), fadd_rn(a.y, v.y), fadd_rn(a.z, v.z), fadd_rn(a.w, v.w));
        } else {
            *o = v;
        }
    }
}

__global__ void group_sum_kernel(const float *__restrict__ x, int ldx, int G, int k, int C,
                                 float *__restrict__ out, int ldo, int acc) {
    GRID_STRIDE(i, (size_t)G * C) {
        const int g = (int)(i / C), c = (int)(i % C);
        const float *p = x + (size_t)g * k * ldx + c;
        float s = 0.f;
        for (int j = 0; j < k; ++j) s = fadd_rn(s, p[(size_t)j * ldx]);
        float *o = out + (size_t)g * ldo + c;
        *o = acc ? fadd_rn(*o, s) : s;
    }
}

__global__ void gather_rows_kernel(const float *__restrict__ x, int ldx,
                                   const int32_t *__restrict__ idx, int M, int C,
                                   float *__restrict__ out, int ldo) {
    GRID_STRIDE(i, (size_t)M * C) {
        const int m = (int)(i / C), c = (int)(i % C);
        out[(size_t)m * ldo + c] = x[(size_t)idx[m] * ldx + c];
    }
}

// out[b*m + j] = idx[b*m + j] + b*n: per-cloud indices -> rows of the [nb*n] stack
__global__ void index_offset_kernel(const int32_t *__restrict__ idx, int nb, int m, int n,
                                    int32_t *__restrict__ out) {
    GRID_STRIDE(i, (size_t)nb * m) out[i] = idx[i] + (int32_t)(i / m) * n;
}

// ---------------------------------------------------------- CSR of an index
// ws: offsets [n+1] | entries [M] | cursor [n]  (int32)
struct Csr {
    int32_t *off, *ent, *cur;
};
__host__ __device__ inline Csr csr_view(void *ws, int M, int n) {
    int32_t *p = (int32_t *)ws;
    return Csr{p, p + (n + 1), p + (n + 1) + M};
}

__global__ void csr_count_kernel(const int32_t *__restrict__ idx, int M, int n,
                                 int32_t *__restrict__ cur) {
    GRID_STRIDE(i, (size_t)M) {
        const int v = idx[i];
        if (v >= 0 && v < n) atomicAdd(&cur[v], 1);
    }
}

// exclusive scan of cur[0..n) -> off[0..n], single workgroup of 1024 threads
__global__ __launch_bounds__(1024) void csr_scan_kernel(const int32_t *__restrict__ cnt, int n,
                                                        int32_t *__restrict__ off) {
    __shared__ int32_t part[1024];
    const int t = threadIdx.x;
    const int chunk = (n + 1023) / 1024;
    const int a = min(n, t * chunk), b = min(n, a + chunk);
    int32_t s = 0;
    for (int i = a; i < b; ++i) s += cnt[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int32_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int32_t run = part[t] - s;  // exclusive prefix of this chunk
    for (int i = a; i < b; ++i) {
        off[i] = run;
        run += cnt[i];
    }
    if (t == 1023) off[n] = part[1023];
}

__global__ void csr_fill_kernel(const int32_t *__restrict__ idx, int M, int n,
                                const int32_t *__restrict__ off, int32_t *__restrict__ cur,
                                int32_t *__restrict__ ent) {
    GRID_STRIDE(i, (size_t)M) {
        const int v = idx[i];
        if (v >= 0 && v < n) ent[off[v] + atomicAdd(&cur[v], 1)] = (int32_t)i;
    }
}

// each segment sorted ascending: the scatter then sums in destination order.
// One thread per segment; segments of up to CSR_REG entries (nearly all: ~4 on average
// at level 1) are loaded with independent loads and sorted in registers by an unrolled
// odd-even transposition network.  Longer ones are taken by the whole wave, one at a
// time (ballot): each lane holds up to CSR_LR of the segment's entries and ranks them
// against the full segment (independent broadcast loads), then writes each entry to its
// rank -- every read precedes every write in each lane.  Segments beyond 64 x CSR_LR
// fall back to an insertion sort by one lane.  Entries are distinct row ids, so every
// path gives the one ascending order.  (A thread-serial insertion sort in memory for
// every segment took 59 us per call, set by the longest segments.)
constexpr int CSR_REG = 16;
constexpr int CSR_LR = 8;
__global__ __launch_bounds__(TB) void csr_sort_kernel(int n, const int32_t *__restrict__ off,
                                                      int32_t *__restrict__ ent) {
    const int lane = threadIdx.x & 63;
    // whole waves iterate together (the ballot below needs every lane)
    for (size_t s0 = (size_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); s0 < (size_t)n;
         s0 += (size_t)gridDim.x * blockDim.x) {
        const size_t s = s0 + lane;
        const int a = s < (size_t)n ? off[s] : 0, b = s < (size_t)n ? off[s + 1] : 0;
        const int len = b - a;
        if (len > 1 && len <= CSR_REG) {
            int32_t v[CSR_REG];
#pragma unroll
            for (int i = 0; i < CSR_REG; ++i) v[i] = i < len ? ent[a + i] : INT32_MAX;
#pragma unroll
            for (int r = 0; r < CSR_REG; ++r)
#pragma unroll
                for (int i = r & 1; i + 1 < CSR_REG; i += 2) {
                    const int32_t lo = min(v[i], v[i + 1]), hi = max(v[i], v[i + 1]);
                    v[i] = lo;
                    v[i + 1] = hi;
                }
#pragma unroll
            for (int i = 0; i < CSR_REG; ++i)
                if (i < len) ent[a + i] = v[i];
        }
        uint64_t longs = __ballot(len > CSR_REG);
        while (longs) {  // wave-uniform
            const int l = (int)__builtin_ctzll(longs);
            longs &= longs - 1;
            const int la = __builtin_amdgcn_readlane(a, l), lb = __builtin_amdgcn_readlane(b, l);
            if (lb - la <= 64 * CSR_LR) {
                int32_t v[CSR_LR];
                int rk[CSR_LR];
#pragma unroll
                for (int r = 0; r < CSR_LR; ++r) {
                    const int i = la + r * 64 + lane;
                    v[r] = i < lb ? ent[i] : INT32_MAX;
                    rk[r] = 0;
                }
                for (int q = la; q < lb; ++q) {
                    const int32_t e = ent[q];
#pragma unroll
                    for (int r = 0; r < CSR_LR; ++r) rk[r] += e < v[r] ? 1 : 0;
                }
#pragma unroll
                for (int r = 0; r < CSR_LR; ++r)
                    if (la + r * 64 + lane < lb) ent[la + rk[r]] = v[r];
            } else if (lane == 0) {
                for (int i = la + 1; i < lb; ++i) {
                    const int32_t x = ent[i];
                    int j = i - 1;
                    while (j >= la && ent[j] > x) {
                        ent[j + 1] = ent[j];
                        --j;
                    }
                    ent[j + 1] = x;
                }
            }
        }
    }
}

// float4 forms of gather_rows / scatter_rows (same conditions as copy_rows4_kernel): four
// channels per thread, 32-bit index arithmetic, the same per-element operations and order
__global__ __launch_bounds__(TB) void gather_rows4_kernel(const float4 *__restrict__ x, int ldx4,
                                                          const int32_t *__restrict__ idx, int M,
                                                          int C4, float4 *__restrict__ out, int ldo4) {
    const uint32_t total = (uint32_t)M * (uint32_t)C4;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const uint32_t m = i / (uint32_t)C4, c = i - m * (uint32_t)C4;
        out[(size_t)m * ldo4 + c] = x[(size_t)idx[m] * ldx4 + c];
    }
}

__global__ __launch_bounds__(TB) void scatter_rows4_kernel(const float4 *__restrict__ dy, int ldy4,
                                                           const int32_t *__restrict__ off,
                                                           const int32_t *__restrict__ ent, int n,
                                                           int C4, float4 *__restrict__ dx, int ldx4,
                                                           int acc) {
    const uint32_t total = (uint32_t)n * (uint32_t)C4;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const uint32_t s = i / (uint32_t)C4, c = i - s * (uint32_t)C4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int e = off[s]; e < off[s + 1]; ++e) {
            const float4 d = dy[(size_t)ent[e] * ldy4 + c];
            v = make_float4(fadd_rn(v.x, d.x), fadd_rn(v.y, d.y), fadd_rn(v.z, d.z), fadd_rn(v.w, d.w));
        }
        float4 *o = dx + (size_t)s * ldx4 + c;
        if (acc) {
            const float4 a = *o;
            v = make_float4(fadd_rn(a.x, v.x), fadd_rn(a.y, v.y), fadd_rn(a.z, v.z), fadd_rn(a.w, v.w));
        }
        *o = v;
    }
}

inline bool rows_v4(int C, int ld0, int ld1, const void *p0, const void *p1, size_t rows) {
    return !(C & 3) && !(ld0 & 3) && !(ld1 & 3) &&
           !((reinterpret_cast<uintptr_t>(p0) | reinterpret_cast<uintptr_t>(p1)) & 15) &&
           rows * (size_t)C / 4 < (1u << 31);
}

__global__ void scatter_rows_kernel(const float *__restrict__ dy, int ldy,
                                    const int32_t *__restrict__ off,
                                    const int32_t *__restrict__ ent, int n, int C,
                                    float *__restrict__ dx, int ldx, int acc) {
    GRID_STRIDE(i, (size_t)n * C) {
        const int s = (int)(i / C), c = (int)(i % C);
        float v = 0.f;
        for (int e = off[s]; e < off[s + 1]; ++e) v = fadd_rn(v, dy[(size_t)ent[e] * ldy + c]);
        float *o = dx + (size_t)s * ldx + c;
        *o = acc ? fadd_rn(*o, v) : v;
    }
}

// ------------------------------------------------------------- geometry rows
__global__ void geom_rows_kernel(const float *__restrict__ q, const float *__restrict__ kx, int G,
                                 int k, float *__restrict__ out, int ldo) {
    GRID_STRIDE(r, (size_t)G * k) {
        const size_t g = r / k;
        const float dx = fsub_rn(kx[r * 3], q[g * 3]);
        const float dy = fsub_rn(kx[r * 3 + 1], q[g * 3 + 1]);
        const float dz = fsub_rn(kx[r * 3 + 2], q[g * 3 + 2]);
        float *o = out + r * ldo;
        o[0] = dx;
        o[1] = dy;
        o[2] = dz;
        o[3] = sqrtf(fadd_rn(fadd_rn(fmul_rn(dx, dx), fmul_rn(dy, dy)), fmul_rn(dz, dz)));
    }
}

// geom = [rela(3), dist(1)]: drela = dgeom[0:3] + ddist * rela / dist (0 at dist 0, as
// torch.norm's backward); dkx = drela (+ dkx_extra); dq = -sum_k drela
__global__ void geom_rows_bwd_kernel(const float *__restrict__ geom, int ldg,
                                     const float *__restrict__ dgeom, int lddg,
                                     const float *__restrict__ dkx_extra, int G, int k,
                                     float *__restrict__ dq, float *__restrict__ dkx) {
    GRID_STRIDE(g, (size_t)G) {
        float sx = 0.f, sy = 0.f, sz = 0.f;
        for (int j = 0; j < k; ++j) {
            const size_t r = g * k + j;
            const float *gr = geom + r * ldg;
            const float *dg = dgeom + r * lddg;
            float d0 = dg[0], d1 = dg[1], d2 = dg[2];
            const float dist = gr[3];
            if (dist > 0.f) {
                const float f = dg[3] / dist;
                d0 = fadd_rn(d0, fmul_rn(f, gr[0]));
                d1 = fadd_rn(d1, fmul_rn(f, gr[1]));
                d2 = fadd_rn(d2, fmul_rn(f, gr[2]));
            }
            if (dkx) {
                float e0 = d0, e1 = d1, e2 = d2;
                if (dkx_extra) {
                    e0 = fadd_rn(e0, dkx_extra[r * 3]);
                    e1 = fadd_rn(e1, dkx_extra[r * 3 + 1]);
                    e2 = fadd_rn(e2, dkx_extra[r * 3 + 2]);
                }
                dkx[r * 3] = e0;
                dkx[r * 3 + 1] = e1;
                dkx[r * 3 + 2] = e2;
            }
            sx = fadd_rn(sx, d0);
            sy = fadd_rn(sy, d1);
            sz = fadd_rn(sz, d2);
        }
        if (dq) {
            dq[g * 3] = -sx;
            dq[g * 3 + 1] = -sy;
            dq[g * 3 + 2] = -sz;
        }
    }
}

// ----------------------------------------------------------------- attention
// One workgroup per group of k <= 64 rows.  x1 = max_c logits (first index),
// a = softmax_k(x1), kp = sum a*kx, vmap = vals*a, vsum = sum_k vmap.
// (PRE, r6) BatchNorm parameters of a pre-BN input: every logits / vals value enters as
// bn_act(x, mean[c], invstd[c], gamma[c], beta[c], ReLU) (hreg_bn_apply's values; the detector's
// last conv activation, never written: train.py _BNActAttention)
struct AttPre {
    const float *mean, *invstd, *gamma, *beta;
};
template <bool PRE>
__device__ __forceinline__ float att_in(const float *p, size_t i, int c, const AttPre &pp) {
    return PRE ? bn_act(p[i], pp.mean[c], pp.invstd[c], pp.gamma[c], pp.beta[c], 1) : p[i];
}

template <bool PRE = false>
__global__ __launch_bounds__(TB) void attention_fwd_kernel(
    const float *__restrict__ logits, int ldl, int C, const float *__restrict__ vals, int ldv,
    int Cv, const float *__restrict__ kx, int k, float *__restrict__ a_out,
    int32_t *__restrict__ amax, float *__restrict__ kp, float *__restrict__ vmap, int ldm,
    float *__restrict__ vsum, int lds, AttPre pp = {}) {
    __shared__ float x1[64], aw[64];
    const int g = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int j = w; j < k; j += TB / 64) {
        const float *row = logits + ((size_t)g * k + j) * ldl;
        float best = -INFINITY;
        int bi = 0x7fffffff;
        for (int c = lane; c < C; c += 64) {
            const float v = att_in<PRE>(row, c, c, pp);
            if (v > best) { best = v; bi = c; }
        }
        for (int m = 32; m >= 1; m >>= 1) {
            const float ob = __shfl_xor(best, m);
            const int oi = __shfl_xor(bi, m);
            if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        }
        if (lane == 0) {
            x1[j] = best;
            if (amax) amax[(size_t)g * k + j] = bi;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float m = -INFINITY;
        for (int j = 0; j < k; ++j) m = fmaxf(m, x1[j]);
        float s = 0.f;
        for (int j = 0; j < k; ++j) {
            aw[j] = expf(fsub_rn(x1[j], m));
            s = fadd_rn(s, aw[j]);
        }
        for (int j = 0; j < k; ++j) aw[j] = aw[j] / s;
    }
    __syncthreads();
    if (threadIdx.x < k && a_out) a_out[(size_t)g * k + threadIdx.x] = aw[threadIdx.x];
    if (kp && threadIdx.x < 3) {
        float s = 0.f;
        for (int j = 0; j < k; ++j)
            s = fadd_rn(s, fmul_rn(aw[j], kx[((size_t)g * k + j) * 3 + threadIdx.x]));
        kp[(size_t)g * 3 + threadIdx.x] = s;
    }
    if (vals)
        for (int c = threadIdx.x; c < Cv; c += TB) {
            float s = 0.f;
            for (int j = 0; j < k; ++j) {
                const float v = fmul_rn(att_in<PRE>(vals, ((size_t)g * k + j) * ldv + c, c, pp), aw[j]);
                if (vmap) vmap[((size_t)g * k + j) * ldm + c] = v;
                s = fadd_rn(s, v);
            }
            if (vsum) vsum[(size_t)g * lds + c] = s;
        }
}

// dve = dvmap + dvsum[g]; dvals = a*dve; da = sum_c vals*dve + kx.dkp;
// dx1 = a*(da - sum a da); dlogits = onehot(amax)*dx1 (+ dvals when vals == logits)
template <bool PRE = false>
__global__ __launch_bounds__(TB) void attention_bwd_kernel(
    const float *__restrict__ logits, int ldl, int C, const float *__restrict__ vals, int ldv,
    int Cv, const float *__restrict__ kx, int k, const float *__restrict__ a_in,
    const int32_t *__restrict__ amax, const float *__restrict__ dkp,
    const float *__restrict__ dvmap, int lddm, const float *__restrict__ dvsum, int ldds,
    int same, float *__restrict__ dlogits, int lddl, float *__restrict__ dvals, int lddv,
    float *__restrict__ dkx, AttPre pp = {}) {
    __shared__ float aw[64], da[64], dx1[64];
    const int g = blockIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < k) aw[threadIdx.x] = a_in[(size_t)g * k + threadIdx.x];
    __syncthreads();
    for (int j = w; j < k; j += TB / 64) {
        const size_t r = (size_t)g * k + j;
        float part = 0.f;
        if (vals && (dvmap || dvsum))
            for (int c = lane; c < Cv; c += 64) {
                float d = 0.f;
                if (dvmap) d = dvmap[r * lddm + c];
                if (dvsum) d = fadd_rn(d, dvsum[(size_t)g * ldds + c]);
                part = fadd_rn(part, fmul_rn(att_in<PRE>(vals, r * ldv + c, c, pp), d));
                if (dvals && !same) dvals[r * lddv + c] = fmul_rn(aw[j], d);
            }
        part = wave_sum_f32(part);
        if (lane == 0) {
            float s = part;
            if (dkp)
                for (int d = 0; d < 3; ++d) s = fadd_rn(s, fmul_rn(kx[r * 3 + d], dkp[(size_t)g * 3 + d]));
            da[j] = s;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int j = 0; j < k; ++j) s = fadd_rn(s, fmul_rn(aw[j], da[j]));
        for (int j = 0; j < k; ++j) dx1[j] = fmul_rn(aw[j], fsub_rn(da[j], s));
    }
    __syncthreads();
    if (dkx && dkp && threadIdx.x < 3 * k) {
        const int j = threadIdx.x / 3, d = threadIdx.x % 3;
        dkx[((size_t)g * k + j) * 3 + d] = fmul_rn(aw[j], dkp[(size_t)g * 3 + d]);
    }
    if (dlogits)
        for (int j = w; j < k; j += TB / 64) {
            const size_t r = (size_t)g * k + j;
            const int am = amax[r];
            for (int c = lane; c < C; c += 64) {
                float v = c == am ? dx1[j] : 0.f;
                if (same) {
                    float d = 0.f;
                    if (dvmap) d = dvmap[r * lddm + c];
                    if (dvsum) d = fadd_rn(d, dvsum[(size_t)g * ldds + c]);
                    v = fadd_rn(v, fmul_rn(aw[j], d));
                }
                dlogits[r * lddl + c] = v;
            }
        }
}

// --------------------------------------------------------------- group max
// PRE (r6): x is a pre-BatchNorm output and every value enters as bn_act(x, mean[c], invstd[c],
// gamma[c], beta[c], ReLU) -- hreg_bn_apply's values, so the same maxima and arguments as over the
// materialised activation
template <bool PRE = false>
__global__ void group_max_arg_kernel(const float *__restrict__ x, int ldx, int G, int k, int C,
                                     float *__restrict__ out, int ldo, int32_t *__restrict__ arg,
                                     const float *__restrict__ mean = nullptr, const float *__restrict__ invstd = nullptr,
                                     const float *__restrict__ gamma = nullptr,
                                     const float *__restrict__ beta = nullptr) {
    GRID_STRIDE(i, (size_t)G * C) {
        const int g = (int)(i / C), c = (int)(i % C);
        const float *p = x + (size_t)g * k * ldx + c;
        float mu = 0.f, is = 0.f, ga = 0.f, be = 0.f;
        if constexpr (PRE) {
            mu = mean[c];
            is = invstd[c];
            ga = gamma[c];
            be = beta[c];
        }
        auto val = [&](float v) { return PRE ? bn_act(v, mu, is, ga, be, 1) : v; };
        float b = val(p[0]);
        int bi = 0;
        for (int j = 1; j < k; ++j) {
            const float v = val(p[(size_t)j * ldx]);
            if (v > b) { b = v; bi = j; }
        }
        out[(size_t)g * ldo + c] = b;
        arg[i] = bi;
    }
}

__global__ void group_max_bwd_kernel(const float *__restrict__ dout, int ldd,
                                     const int32_t *__restrict__ arg, int G, int k, int C,
                                     float *__restrict__ dx, int ldx, int acc) {
    GRID_STRIDE(i, (size_t)G * C) {
        const int g = (int)(i / C), c = (int)(i % C);
        const int a = arg[i];
        const float d = dout[(size_t)g * ldd + c];
        float *p = dx + (size_t)g * k * ldx + c;
        if (acc) {
            p[(size_t)a * ldx] = fadd_rn(p[(size_t)a * ldx], d);
        } else {
            for (int j = 0; j < k; ++j) p[(size_t)j * ldx] = j == a ? d : 0.f;
        }
    }
}

// ---------------------------------------------------------- head output bwd
// y = softplus(z) + 0.001 (mode HREG_HEAD_SOFTPLUS) or sigmoid(z), z = x.w3 + b3:
// dz = dy * act'(z) (torch softplus_backward: threshold 20), dx = dz * w3
__global__ __launch_bounds__(TB) void head_out_bwd_kernel(const float *__restrict__ x, int ldx,
                                                          int C, const float *__restrict__ w3,
                                                          const float *__restrict__ b3,
                                                          const float *__restrict__ dy, int mode,
                                                          int G, float *__restrict__ dz,
                                                          float *__restrict__ dx, int lddx) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = blockIdx.x * (TB / 64) + w;
    if (g >= G) return;
    const float *row = x + (size_t)g * ldx;
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s = fadd_rn(s, fmul_rn(row[c], w3[c]));
    s = wave_sum_f32(s);
    const float z = fadd_rn(s, b3[0]);
    float d;
    if (mode == HREG_HEAD_SOFTPLUS) {
        if (z > 20.f) {
            d = dy[g];
        } else {
            const float e = expf(z);
            d = dy[g] * e / (e + 1.f);
        }
    } else {
        const float y = 1.f / (1.f + expf(-z));
        d = fmul_rn(dy[g], fmul_rn(y, fsub_rn(1.f, y)));
    }
    if (lane == 0) dz[g] = d;
    for (int c = lane; c < C; c += 64) dx[(size_t)g * lddx + c] = fmul_rn(d, w3[c]);
}

// --------------------------------------------------------- cosine similarity
// S [nb][N1][N2]: row maxima (over N2) and column maxima (over N1), first index
__global__ void sim_stats_kernel(const float *__restrict__ S, int nb, int N1, int N2,
                                 float *__restrict__ rmax, int32_t *__restrict__ rarg,
                                 float *__restrict__ cmax, int32_t *__restrict__ carg) {
    GRID_STRIDE(t, (size_t)nb * (N1 + N2)) {
        const int b = (int)(t / (N1 + N2)), u = (int)(t % (N1 + N2));
        const float *Sb = S + (size_t)b * N1 * N2;
        if (u < N1) {
            const float *row = Sb + (size_t)u * N2;
            float m = row[0];
            int a = 0;
            for (int j = 1; j < N2; ++j)
                if (row[j] > m) { m = row[j]; a = j; }
            rmax[(size_t)b * N1 + u] = m;
            rarg[(size_t)b * N1 + u] = a;
        } else {
            const int j = u - N1;
            float m = Sb[j];
            int a = 0;
            for (int i = 1; i < N1; ++i)
                if (Sb[(size_t)i * N2 + j] > m) { m = Sb[(size_t)i * N2 + j]; a = i; }
            cmax[(size_t)b * N2 + j] = m;
            carg[(size_t)b * N2 + j] = a;
        }
    }
}

// out[r][0] = S[i][n] / (rmax_i + 1e-6)   (src_dst_cos, layers.py:300-313)
// out[r][1] = S[i][n] / (cmax_n + 1e-6)   (dst_src_cos, layers.py:296-307), n = kidx[b][i][j]
__global__ void sim_feats_kernel(const float *__restrict__ S, int nb, int N1, int N2,
                                 const int32_t *__restrict__ kidx, int k,
                                 const float *__restrict__ rmax, const float *__restrict__ cmax,
                                 float *__restrict__ out, int ldo) {
    GRID_STRIDE(r, (size_t)nb * N1 * k) {
        const size_t bi = r / k;
        const int b = (int)(bi / N1);
        const int n = kidx[r];
        const float s = S[bi * N2 + n];
        out[r * ldo] = s / fadd_rn(rmax[bi], 1e-6f);
        out[r * ldo + 1] = s / fadd_rn(cmax[(size_t)b * N2 + n], 1e-6f);
    }
}

// dS rows (dS zeroed before): the gathered entries and the row-max term
__global__ void sim_bwd_rows_kernel(const float *__restrict__ S, int nb, int N1, int N2,
                                    const int32_t *__restrict__ kidx, int k,
                                    const float *__restrict__ rmax, const int32_t *__restrict__ rarg,
                                    const float *__restrict__ cmax, const float *__restrict__ dout,
                                    int ldd, float *__restrict__ dS) {
    GRID_STRIDE(bi, (size_t)nb * N1) {
        const int b = (int)(bi / N1);
        const float rm = fadd_rn(rmax[bi], 1e-6f);
        float drm = 0.f;
        float *dr = dS + bi * N2;
        for (int j = 0; j < k; ++j) {
            const size_t r = bi * k + j;
            const int n = kidx[r];
            const float s = S[bi * N2 + n];
            const float g1 = dout[r * ldd], g2 = dout[r * ldd + 1];
            const float cm = fadd_rn(cmax[(size_t)b * N2 + n], 1e-6f);
            dr[n] = fadd_rn(dr[n], fadd_rn(g1 / rm, g2 / cm));
            drm = fsub_rn(drm, g1 * s / fmul_rn(rm, rm));
        }
        const int a = rarg[bi];
        dr[a] = fadd_rn(dr[a], drm);
    }
}

// column-max term: dcm_n = -sum_{(i,j): kidx = n} g2 S[i][n] / (cmax_n+1e-6)^2 -> dS[carg_n][n]
// One wave per column (b, n): the N1*k index entries are scanned 64 per step (one
// coalesced load + ballot) and the matches applied in ascending e, i.e. the same
// sequential sum as a one-thread serial scan, at 1/64 of its dependent steps (one
// thread per column scanned 2048 entries: 293 us at B = 8, r2 training profile).
__global__ __launch_bounds__(TB) void sim_bwd_cols_kernel(
    const float *__restrict__ S, int nb, int N1, int N2, const int32_t *__restrict__ kidx, int k,
    const float *__restrict__ cmax, const int32_t *__restrict__ carg,
    const float *__restrict__ dout, int ldd, float *__restrict__ dS) {
    constexpr int WPB = TB / 64;
    const int lane = threadIdx.x & 63;
    const int E = N1 * k;
    for (size_t bn = (size_t)blockIdx.x * WPB + threadIdx.x / 64; bn < (size_t)nb * N2;
         bn += (size_t)gridDim.x * WPB) {
        const int b = (int)(bn / N2), n = (int)(bn % N2);
        const float cm = fadd_rn(cmax[bn], 1e-6f);
        const float cm2 = fmul_rn(cm, cm);
        float dcm = 0.f;
        const int32_t *ki = kidx + (size_t)b * E;
        for (int e0 = 0; e0 < E; e0 += 64) {
            const int e = e0 + lane;
            uint64_t hit = __ballot(e < E && ki[e] == n);
            while (hit) {  // wave-uniform: every lane computes the same terms
                const int ee = e0 + (int)__builtin_ctzll(hit);
                hit &= hit - 1;
                const int i = ee / k;
                const float s = S[((size_t)b * N1 + i) * N2 + n];
                dcm = fsub_rn(dcm, dout[((size_t)b * E + ee) * ldd + 1] * s / cm2);
            }
        }
        if (lane == 0) {
            float *p = dS + ((size_t)b * N1 + carg[bn]) * N2 + n;
            *p = fadd_rn(*p, dcm);
        }
    }
}

// cosine backward, S = P / (na nb^T + 1e-6): dP = dS / den;
// dna_i = -sum_j dS_ij S_ij nb_j / den_ij, dnb_j = -sum_i dS_ij S_ij na_i / den_ij
// Rows (dP and dna): one wave per row, lanes along j (coalesced), per-lane partial sums
// in ascending j then a fixed-order wave sum.  (One thread per row walked its row with a
// 1 KB stride between the lanes of a wave: 143 us per call at B = 8.)
__global__ __launch_bounds__(TB) void sim_bwd_cos_rows_kernel(
    const float *__restrict__ S, const float *__restrict__ dS, int nb, int N1, int N2,
    const float *__restrict__ na, const float *__restrict__ nbv, float *__restrict__ dP,
    float *__restrict__ dna) {
    constexpr int WPB = TB / 64;
    const int lane = threadIdx.x & 63;
    for (size_t row = (size_t)blockIdx.x * WPB + threadIdx.x / 64; row < (size_t)nb * N1;
         row += (size_t)gridDim.x * WPB) {
        const int b = (int)(row / N1);
        const float au = na[row];
        const float *c = nbv + (size_t)b * N2;
        const float *Sr = S + row * N2, *dSr = dS + row * N2;
        float acc = 0.f;
        for (int j = lane; j < N2; j += 64) {
            const float den = fadd_rn(fmul_rn(au, c[j]), 1e-6f);
            dP[row * N2 + j] = dSr[j] / den;
            acc = fsub_rn(acc, dSr[j] * Sr[j] / den * c[j]);
        }
        acc = wave_sum_f32(acc);
        if (lane == 0) dna[row] = acc;
    }
}

// Columns (dnb): a 1024-thread workgroup per 64 columns of one batch, lanes along j
// (coalesced), the 16 waves over 16 contiguous slices of i (ascending), the slice sums
// added in slice order.  (One thread per column over all N1 rows: 82 us at B = 8.)
constexpr int COS_SL = 16;
__global__ __launch_bounds__(64 * COS_SL) void sim_bwd_cos_cols_kernel(
    const float *__restrict__ S, const float *__restrict__ dS, int nb, int N1, int N2,
    const float *__restrict__ na, const float *__restrict__ nbv, float *__restrict__ dnb) {
    __shared__ float part[COS_SL][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int groups = (N2 + 63) / 64;
    const int b = blockIdx.x / groups, j = (blockIdx.x % groups) * 64 + lane;
    const int per = (N1 + COS_SL - 1) / COS_SL;
    const int i0 = w * per, i1 = min(N1, i0 + per);
    float acc = 0.f;
    if (j < N2) {
        const float *Sb = S + (size_t)b * N1 * N2, *dSb = dS + (size_t)b * N1 * N2;
        const float *a = na + (size_t)b * N1;
        const float cj = nbv[(size_t)b * N2 + j];
        for (int i = i0; i < i1; ++i) {
            const size_t e = (size_t)i * N2 + j;
            const float den = fadd_rn(fmul_rn(a[i], cj), 1e-6f);
            acc = fsub_rn(acc, dSb[e] * Sb[e] / den * a[i]);
        }
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0 && j < N2) {
        float t = part[0][lane];
        for (int q = 1; q < COS_SL; ++q) t = fadd_rn(t, part[q][lane]);
        dnb[(size_t)b * N2 + j] = t;
    }
}

// out[b][i][c] = sum_j M[b][i][j] X[b][j][c] + (dn_i / n_i) Y[b][i][c]   (TRANS: M^T)
// 64x64 output tile per 256-thread workgroup, 4x4 per thread, j staged through LDS.
template <bool TRANS>
__global__ __launch_bounds__(TB) void sim_bwd_mm_kernel(const float *__restrict__ M, int N1,
                                                        int N2, const float *__restrict__ X,
                                                        const float *__restrict__ Y,
                                                        const float *__restrict__ dn,
                                                        const float *__restrict__ nrm, int C,
                                                        float *__restrict__ out) {
    // rows of out: TRANS ? N2 : N1; reduction length: TRANS ? N1 : N2
    const int Ro = TRANS ? N2 : N1, Kr = TRANS ? N1 : N2;
    const int b = blockIdx.z;
    const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
    __shared__ float Ms[16][65], Xs[16][65];
    const int tr = threadIdx.x / 16, tc = threadIdx.x % 16;
    float acc[4][4] = {};
    const float *Mb = M + (size_t)b * N1 * N2;
    const float *Xb = X + (size_t)b * Kr * C;
    for (int j0 = 0; j0 < Kr; j0 += 16) {
        for (int e = threadIdx.x; e < 16 * 64; e += TB) {
            const int jj = e / 64, rr = e % 64;
            const int j = j0 + jj, r = r0 + rr, c = c0 + rr;
            float mv = 0.f;
            if (j < Kr && r < Ro) mv = TRANS ? Mb[(size_t)j * N2 + r] : Mb[(size_t)r * N2 + j];
            Ms[jj][rr] = mv;
            Xs[jj][rr] = (j < Kr && c < C) ? Xb[(size_t)j * C + c] : 0.f;
        }
        __syncthreads();
        for (int jj = 0; jj < 16; ++jj)
            for (int p = 0; p < 4; ++p)
                for (int q = 0; q < 4; ++q)
                    acc[p][q] = fmaf(Ms[jj][tr * 4 + p], Xs[jj][tc * 4 + q], acc[p][q]);
        __syncthreads();
    }
    for (int p = 0; p < 4; ++p) {
        const int r = r0 + tr * 4 + p;
        if (r >= Ro) continue;
        const float nv = nrm[(size_t)b * Ro + r];
        const float f = nv > 0.f ? dn[(size_t)b * Ro + r] / nv : 0.f;
        for (int q = 0; q < 4; ++q) {
            const int c = c0 + tc * 4 + q;
            if (c >= C) continue;
            out[((size_t)b * Ro + r) * C + c] =
                fadd_rn(acc[p][q], fmul_rn(f, Y[((size_t)b * Ro + r) * C + c]));
        }
    }
}

// ------------------------------------------------------- weighted SVD backward
// Forward (layers.py:469-504): sw = sum w + 1e-4; wn = w / sw; den = sum wn + 1e-4;
// mu_s = sum wn s / den; mu_c likewise; H = sum wn (s-mu_s)(c-mu_c)^T = U S V^T;
// d = det(V^T U^T); R = V diag(1,1,d) U^T; t = mu_c - R mu_s.
__global__ __launch_bounds__(TB) void svd_bwd_kernel(const float *__restrict__ src,
                                                     const float *__restrict__ cor,
                                                     const float *__restrict__ w, int n,
                                                     const float *__restrict__ dR_in,
                                                     const float *__restrict__ dt_in,
                                                     float *__restrict__ dsrc,
                                                     float *__restrict__ dcor,
                                                     float *__restrict__ dw) {
    __shared__ double red[TB / 64][16];
    __shared__ double sh[32];  // gH 9 | ms 3 | mc 3 | dPs 3 | dPc 3 | dden | sw | ok | red
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const float *S = src + (size_t)b * n * 3, *Cc = cor + (size_t)b * n * 3, *W = w + (size_t)b * n;
    auto block_sum = [&](double v[], int cnt) {
        for (int q = 0; q < cnt; ++q) v[q] = wave_sum_f64(v[q]);
        __syncthreads();
        if (lane == 0)
            for (int q = 0; q < cnt; ++q) red[wv][q] = v[q];
        __syncthreads();
        for (int q = 0; q < cnt; ++q) v[q] = ((red[0][q] + red[1][q]) + red[2][q]) + red[3][q];
        __syncthreads();
    };
    double v1[1] = {0.0};
    for (int i = threadIdx.x; i < n; i += TB) v1[0] += (double)W[i];
    block_sum(v1, 1);
    const double sw = v1[0] + 1e-4;
    double m[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += TB) {
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
    for (int i = threadIdx.x; i < n; i += TB) {
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
    if (threadIdx.x == 0) {
        bool ok = true;
        for (int q = 0; q < 9; ++q) ok = ok && isfinite(h[q]);
        double H[3][3], u[3][3], v[3][3], sg[3];
        for (int p = 0; p < 3; ++p)
            for (int q = 0; q < 3; ++q) H[p][q] = h[p * 3 + q];
        double gH[3][3] = {};
        double dms[3] = {0, 0, 0}, dmc[3] = {0, 0, 0};
        if (ok) {
            const double d = svd3_usv(H, u, sg, v);
            // U[:, i] = u[i], V[:, i] = v[i]
            double U[3][3], V[3][3], R[3][3], dR[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) { U[i][j] = u[j][i]; V[i][j] = v[j][i]; }
            const double D[3] = {1.0, 1.0, d};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int q = 0; q < 3; ++q) s += V[i][q] * D[q] * U[j][q];
                    R[i][j] = s;
                }
            const float *dRb = dR_in + (size_t)b * 9, *dtb = dt_in + (size_t)b * 3;
            // t = mu_c - R mu_s
            for (int i = 0; i < 3; ++i) {
                dmc[i] = (double)dtb[i];
                for (int j = 0; j < 3; ++j) dR[i][j] = (double)dRb[i * 3 + j] - (double)dtb[i] * ms[j];
            }
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int i = 0; i < 3; ++i) s += R[i][j] * (double)dtb[i];
                dms[j] = -s;
            }
            // R = V D U^T: gV = dR U D, gU = dR^T V D, gdet = (V^T dR U)[2][2]
            double gV[3][3], gU[3][3], M[3][3];
            double gdet = 0;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double sv = 0, su = 0;
                    for (int q = 0; q < 3; ++q) {
                        sv += dR[i][q] * U[q][j];
                        su += dR[q][i] * V[q][j];
                    }
                    gV[i][j] = sv * D[j];
                    gU[i][j] = su * D[j];
                }
            for (int p = 0; p < 3; ++p)
                for (int q = 0; q < 3; ++q) gdet += V[p][2] * dR[p][q] * U[q][2];
            // d = det(M), M = V^T U^T orthogonal: gM = gdet * d * M^{-T} = gdet * d * M
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int q = 0; q < 3; ++q) s += V[q][i] * U[j][q];
                    M[i][j] = s;
                }
            double gM[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) gM[i][j] = gdet * d * M[i][j];
            // dM = dV^T U^T + V^T dU^T: gV += U^T gM^T, gU += gM^T V^T
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double a = 0, c = 0;
                    for (int q = 0; q < 3; ++q) {
                        a += U[q][i] * gM[j][q];
                        c += gM[q][i] * V[j][q];
                    }
                    gV[i][j] += a;
                    gU[i][j] += c;
                }
            // torch svd_backward (gS = 0): skew(X) = X - X^T,
            // ret = (skew(U^T gU) * S_j + S_i * skew(V^T gV)) / (S_j^2 - S_i^2), gH = U ret V^T
            double UgU[3][3], VgV[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double a = 0, c = 0;
                    for (int q = 0; q < 3; ++q) {
                        a += U[q][i] * gU[q][j];
                        c += V[q][i] * gV[q][j];
                    }
                    UgU[i][j] = a;
                    VgV[i][j] = c;
                }
            double ret[3][3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    if (i == j) { ret[i][j] = 0; continue; }
                    const double ku = UgU[i][j] - UgU[j][i], kv = VgV[i][j] - VgV[j][i];
                    const double E = sg[j] * sg[j] - sg[i] * sg[i];
                    ret[i][j] = (ku * sg[j] + sg[i] * kv) / E;
                }
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int p = 0; p < 3; ++p)
                        for (int q = 0; q < 3; ++q) s += U[i][p] * ret[p][q] * V[j][q];
                    gH[i][j] = s;
                }
            for (int i = 0; i < 9; ++i) ok = ok && isfinite(gH[i / 3][i % 3]);
        }
        for (int i = 0; i < 9; ++i) sh[i] = ok ? gH[i / 3][i % 3] : 0.0;
        for (int d = 0; d < 3; ++d) {
            sh[9 + d] = ms[d];
            sh[12 + d] = mc[d];
            sh[15 + d] = ok ? dms[d] : 0.0;
            sh[18 + d] = ok ? dmc[d] : 0.0;
        }
        sh[21] = ok ? 1.0 : 0.0;
    }
    __syncthreads();
    double gH[9];
    for (int i = 0; i < 9; ++i) gH[i] = sh[i];
    const bool ok = sh[21] != 0.0;
    // pass A: sum of dsc, dcc (the means' share)
    double acc6[6] = {0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < n; i += TB) {
        const double wi = (double)W[i] / sw;
        double a[3], c[3];
        for (int d = 0; d < 3; ++d) {
            a[d] = (double)S[i * 3 + d] - ms[d];
            c[d] = (double)Cc[i * 3 + d] - mc[d];
        }
        for (int p = 0; p < 3; ++p) {
            double s1 = 0, s2 = 0;
            for (int q = 0; q < 3; ++q) {
                s1 += gH[p * 3 + q] * c[q];
                s2 += gH[q * 3 + p] * a[q];
            }
            acc6[p] += wi * s1;
            acc6[3 + p] += wi * s2;
        }
    }
    block_sum(acc6, 6);
    double dPs[3], dPc[3];
    for (int d = 0; d < 3; ++d) {
        dPs[d] = (sh[15 + d] - acc6[d]) / den;
        dPc[d] = (sh[18 + d] - acc6[3 + d]) / den;
    }
    const double dden = -((ms[0] * dPs[0] + ms[1] * dPs[1] + ms[2] * dPs[2]) +
                          (mc[0] * dPc[0] + mc[1] * dPc[1] + mc[2] * dPc[2]));
    // pass B: ds, dc; dwn_i; reduce sum dwn_i w_i
    double acc1[1] = {0.0};
    for (int i = threadIdx.x; i < n; i += TB) {
        const double wi = (double)W[i] / sw;
        double a[3], c[3], s[3], cc[3];
        for (int d = 0; d < 3; ++d) {
            s[d] = (double)S[i * 3 + d];
            cc[d] = (double)Cc[i * 3 + d];
            a[d] = s[d] - ms[d];
            c[d] = cc[d] - mc[d];
        }
        double dwn = dden;
        for (int p = 0; p < 3; ++p) {
            double s1 = 0, s2 = 0;
            for (int q = 0; q < 3; ++q) {
                s1 += gH[p * 3 + q] * c[q];
                s2 += gH[q * 3 + p] * a[q];
            }
            dwn += a[p] * s1 + s[p] * dPs[p] + cc[p] * dPc[p];
            dsrc[((size_t)b * n + i) * 3 + p] = ok ? (float)(wi * s1 + wi * dPs[p]) : 0.f;
            dcor[((size_t)b * n + i) * 3 + p] = ok ? (float)(wi * s2 + wi * dPc[p]) : 0.f;
        }
        acc1[0] += dwn * (double)W[i];
    }
    block_sum(acc1, 1);
    const double corr = acc1[0] / (sw * sw);
    for (int i = threadIdx.x; i < n; i += TB) {
        double a[3], c[3], s[3], cc[3];
        for (int d = 0; d < 3; ++d) {
            s[d] = (double)S[i * 3 + d];
            cc[d] = (double)Cc[i * 3 + d];
            a[d] = s[d] - ms[d];
            c[d] = cc[d] - mc[d];
        }
        double dwn = dden;
        for (int p = 0; p < 3; ++p) {
            double s1 = 0;
            for (int q = 0; q < 3; ++q) s1 += gH[p * 3 + q] * c[q];
            dwn += a[p] * s1 + s[p] * dPs[p] + cc[p] * dPc[p];
        }
        dw[(size_t)b * n + i] = ok ? (float)(dwn / sw - corr) : 0.f;
    }
}

// ------------------------------------------------------- transform / compose
// y = R x + t per point: dx = R^T dy; dR = sum dy x^T; dt = sum dy (fp64, one block per pair)
__global__ __launch_bounds__(TB) void transform_bwd_kernel(const float *__restrict__ xyz,
                                                           const float *__restrict__ R, int n,
                                                           const float *__restrict__ dy,
                                                           float *__restrict__ dx,
                                                           float *__restrict__ dR,
                                                           float *__restrict__ dt) {
    __shared__ double red[TB / 64][12];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const float *Rb = R + (size_t)b * 9;
    double acc[12] = {};
    for (int i = threadIdx.x; i < n; i += TB) {
        const size_t e = ((size_t)b * n + i) * 3;
        const float g[3] = {dy[e], dy[e + 1], dy[e + 2]};
        if (dx)
            for (int j = 0; j < 3; ++j)
                dx[e + j] = fadd_rn(fadd_rn(fmul_rn(Rb[j], g[0]), fmul_rn(Rb[3 + j], g[1])),
                                    fmul_rn(Rb[6 + j], g[2]));
        for (int p = 0; p < 3; ++p) {
            for (int q = 0; q < 3; ++q) acc[p * 3 + q] += (double)g[p] * (double)xyz[e + q];
            acc[9 + p] += (double)g[p];
        }
    }
    for (int q = 0; q < 12; ++q) acc[q] = wave_sum_f64(acc[q]);
    if (lane == 0)
        for (int q = 0; q < 12; ++q) red[wv][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < 12) {
        const int q = threadIdx.x;
        const double v = ((red[0][q] + red[1][q]) + red[2][q]) + red[3][q];
        if (q < 9) {
            if (dR) dR[(size_t)b * 9 + q] = (float)v;
        } else if (dt) {
            dt[(size_t)b * 3 + q - 9] = (float)v;
        }
    }
}

// Ro = Ra Rb, to = Ra tb + ta  (T = T_a @ T_b in homogeneous form)
__global__ void compose_kernel(int nb, const float *__restrict__ Ra, const float *__restrict__ ta,
                               const float *__restrict__ Rb, const float *__restrict__ tb,
                               float *__restrict__ Ro, float *__restrict__ to) {
    GRID_STRIDE(b, (size_t)nb) {
        const float *A = Ra + b * 9, *B = Rb + b * 9;
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) {
                float s = 0.f;
                for (int q = 0; q < 3; ++q) s = fadd_rn(s, fmul_rn(A[i * 3 + q], B[q * 3 + j]));
                Ro[b * 9 + i * 3 + j] = s;
            }
            float s = 0.f;
            for (int q = 0; q < 3; ++q) s = fadd_rn(s, fmul_rn(A[i * 3 + q], tb[b * 3 + q]));
            to[b * 3 + i] = fadd_rn(s, ta[b * 3 + i]);
        }
    }
}

// dRa = dRo Rb^T + dto tb^T; dta = dto; dRb = Ra^T dRo; dtb = Ra^T dto
__global__ void compose_bwd_kernel(int nb, const float *__restrict__ Ra,
                                   const float *__restrict__ Rb, const float *__restrict__ tb,
                                   const float *__restrict__ dRo, const float *__restrict__ dto,
                                   float *__restrict__ dRa, float *__restrict__ dta,
                                   float *__restrict__ dRb, float *__restrict__ dtb) {
    GRID_STRIDE(b, (size_t)nb) {
        const float *A = Ra + b * 9, *B = Rb + b * 9, *G = dRo + b * 9, *g = dto + b * 3;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                float s = fmul_rn(g[i], tb[b * 3 + j]);
                float u = 0.f;
                for (int q = 0; q < 3; ++q) {
                    s = fadd_rn(s, fmul_rn(G[i * 3 + q], B[j * 3 + q]));
                    u = fadd_rn(u, fmul_rn(A[q * 3 + i], G[q * 3 + j]));
                }
                dRa[b * 9 + i * 3 + j] = s;
                dRb[b * 9 + i * 3 + j] = u;
            }
        for (int i = 0; i < 3; ++i) {
            dta[b * 3 + i] = g[i];
            float u = 0.f;
            for (int q = 0; q < 3; ++q) u = fadd_rn(u, fmul_rn(A[q * 3 + i], g[q]));
            dtb[b * 3 + i] = u;
        }
    }
}

// --------------------------------------------------------- loss backward
// L = scale * (alpha * mean_b |E_b - I|_F + mean_b |t_b - t_gt,b|), E = R^T R_gt
__global__ void loss_bwd_kernel(const float *__restrict__ pR, const float *__restrict__ pt,
                                const float *__restrict__ gR, const float *__restrict__ gt, int nb,
                                float alpha, float scale, const float *__restrict__ dloss,
                                float *__restrict__ dR, float *__restrict__ dt) {
    if (dloss) scale *= dloss[0];
    GRID_STRIDE(b, (size_t)nb) {
        const float *R = pR + b * 9, *G = gR + b * 9;
        float D[3][3];
        float fro = 0.f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                float s = 0.f;
                for (int q = 0; q < 3; ++q) s = fadd_rn(s, fmul_rn(R[q * 3 + i], G[q * 3 + j]));
                D[i][j] = fsub_rn(s, i == j ? 1.f : 0.f);
                fro = fadd_rn(fro, fmul_rn(D[i][j], D[i][j]));
            }
        fro = sqrtf(fro);
        const float fR = fro > 0.f ? alpha * scale / (float)nb / fro : 0.f;
        // dE = fR * D; dR = G dE^T
        for (int p = 0; p < 3; ++p)
            for (int q = 0; q < 3; ++q) {
                float s = 0.f;
                for (int j = 0; j < 3; ++j) s = fadd_rn(s, fmul_rn(G[p * 3 + j], D[q][j]));
                dR[b * 9 + p * 3 + q] = fmul_rn(fR, s);
            }
        float e[3], n2 = 0.f;
        for (int q = 0; q < 3; ++q) {
            e[q] = fsub_rn(pt[b * 3 + q], gt[b * 3 + q]);
            n2 = fadd_rn(n2, fmul_rn(e[q], e[q]));
        }
        const float nr = sqrtf(n2);
        const float ft = nr > 0.f ? scale / (float)nb / nr : 0.f;
        for (int q = 0; q < 3; ++q) dt[b * 3 + q] = fmul_rn(ft, e[q]);
    }
}

}  // namespace

// ======================================================================= C ABI

// up to COPY_MANY contiguous byte ranges in one launch (blockIdx.y = range): 16-byte words when
// both ends and the size allow, else 4-byte words (every range a multiple of 4 bytes)
constexpr int COPY_MANY = 16;
struct CopyMany {
    const void *src[COPY_MANY];
    void *dst[COPY_MANY];
    size_t nbytes[COPY_MANY];
};

__global__ __launch_bounds__(TB) void copy_many_kernel(CopyMany cm) {
    const int e = blockIdx.y;
    const size_t nb = cm.nbytes[e];
    const uintptr_t a = reinterpret_cast<uintptr_t>(cm.src[e]) | reinterpret_cast<uintptr_t>(cm.dst[e]);
    if (!((a | nb) & 15)) {
        const uint4 *s = static_cast<const uint4 *>(cm.src[e]);
        uint4 *d = static_cast<uint4 *>(cm.dst[e]);
        for (size_t i = (size_t)blockIdx.x * TB + threadIdx.x; i < nb / 16; i += (size_t)gridDim.x * TB) d[i] = s[i];
    } else {
        const uint32_t *s = static_cast<const uint32_t *>(cm.src[e]);
        uint32_t *d = static_cast<uint32_t *>(cm.dst[e]);
        for (size_t i = (size_t)blockIdx.x * TB + threadIdx.x; i < nb / 4; i += (size_t)gridDim.x * TB) d[i] = s[i];
    }
}

// count (<= 16) device-to-device copies of nbytes[i] (multiples of 4) in one launch: the graph
// executor's per-round copies of a lane's feature-extraction outputs (r6: 12 copy nodes -> 1)
extern "C" int hreg_copy_many(int count, const void *const *src, void *const *dst, const size_t *nbytes,
                              void *stream) {
    if (count < 0 || count > COPY_MANY || (count && (!src || !dst || !nbytes))) return HREG_ERR_INVALID;
    CopyMany cm{};
    size_t most = 0;
    for (int i = 0; i < count; ++i) {
        if (!src[i] || !dst[i] || (nbytes[i] & 3)) return HREG_ERR_INVALID;
        cm.src[i] = src[i];
        cm.dst[i] = dst[i];
        cm.nbytes[i] = nbytes[i];
        most = nbytes[i] > most ? nbytes[i] : most;
    }
    if (!count || !most) return HREG_OK;
    hipLaunchKernelGGL(copy_many_kernel, dim3(g1d((most + 15) / 16), count), dim3(TB), 0, as_stream(stream), cm);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_copy_rows(const float *src, int lds, int row_div, int R, int C, float *dst,
                              int ldd, int accumulate, void *stream) {
    if (!src || !dst || R < 0 || C < 0 || row_div < 1 || lds < C || ldd < C) return HREG_ERR_INVALID;
    if (!R || !C) return HREG_OK;
    const bool v4 = !(C & 3) && !(lds & 3) && !(ldd & 3) &&
                    !((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) &&
                    (size_t)R * C / 4 < (1u << 31);
    if (v4) {
        const dim3 g(g1d((size_t)R * C / 4));
        if (accumulate)
            hipLaunchKernelGGL(copy_rows4_kernel<true>, g, dim3(TB), 0, as_stream(stream),
                               reinterpret_cast<const float4 *>(src), lds / 4, row_div, R, C / 4,
                               reinterpret_cast<float4 *>(dst), ldd / 4);
        else
            hipLaunchKernelGGL(copy_rows4_kernel<false>, g, dim3(TB), 0, as_stream(stream),
                               reinterpret_cast<const float4 *>(src), lds / 4, row_div, R, C / 4,
                               reinterpret_cast<float4 *>(dst), ldd / 4);
    } else {
        hipLaunchKernelGGL(copy_rows_kernel, dim3(g1d((size_t)R * C)), dim3(TB), 0, as_stream(stream),
                           src, lds, row_div, R, C, dst, ldd, accumulate);
    }
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_sum(const float *x, int ldx, int G, int k, int C, float *out, int ldo,
                              int accumulate, void *stream) {
    if (!x || !out || G < 0 || k < 1 || C < 0 || ldx < C || ldo < C) return HREG_ERR_INVALID;
    if (!G || !C) return HREG_OK;
    hipLaunchKernelGGL(group_sum_kernel, dim3(g1d((size_t)G * C)), dim3(TB), 0, as_stream(stream),
                       x, ldx, G, k, C, out, ldo, accumulate);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_gather_rows(const float *x, int ldx, const int32_t *idx, int M, int C,
                                float *out, int ldo, void *stream) {
    if (!x || !idx || !out || M < 0 || C < 0 || ldx < C || ldo < C) return HREG_ERR_INVALID;
    if (!M || !C) return HREG_OK;
    if (rows_v4(C, ldx, ldo, x, out, (size_t)M))
        hipLaunchKernelGGL(gather_rows4_kernel, dim3(g1d((size_t)M * C / 4)), dim3(TB), 0,
                           as_stream(stream), reinterpret_cast<const float4 *>(x), ldx / 4, idx, M,
                           C / 4, reinterpret_cast<float4 *>(out), ldo / 4);
    else
        hipLaunchKernelGGL(gather_rows_kernel, dim3(g1d((size_t)M * C)), dim3(TB), 0,
                           as_stream(stream), x, ldx, idx, M, C, out, ldo);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_index_offset(const int32_t *idx, int nb, int m, int n, int32_t *out,
                                 void *stream) {
    if (!idx || !out || nb < 0 || m < 0 || n < 0) return HREG_ERR_INVALID;
    if (!nb || !m) return HREG_OK;
    hipLaunchKernelGGL(index_offset_kernel, dim3(g1d((size_t)nb * m)), dim3(TB), 0,
                       as_stream(stream), idx, nb, m, n, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" size_t hreg_csr_ws_bytes(int M, int n) {
    if (M < 0 || n < 0) return 0;
    return ((size_t)(n + 1) + (size_t)M + (size_t)n) * sizeof(int32_t);
}

extern "C" int hreg_csr_build(const int32_t *idx, int M, int n, void *ws, void *stream) {
    if (!idx || !ws || M < 0 || n < 1) return HREG_ERR_INVALID;
    hipStream_t st = as_stream(stream);
    Csr c = csr_view(ws, M, n);
    if (hipMemsetAsync(c.cur, 0, (size_t)n * sizeof(int32_t), st) != hipSuccess) return HREG_ERR_LAUNCH;
    if (M) {
        hipLaunchKernelGGL(csr_count_kernel, dim3(g1d(M)), dim3(TB), 0, st, idx, M, n, c.cur);
        HREG_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(csr_scan_kernel, dim3(1), dim3(1024), 0, st, c.cur, n, c.off);
    HREG_CHECK_LAUNCH();
    if (hipMemsetAsync(c.cur, 0, (size_t)n * sizeof(int32_t), st) != hipSuccess) return HREG_ERR_LAUNCH;
    if (M) {
        hipLaunchKernelGGL(csr_fill_kernel, dim3(g1d(M)), dim3(TB), 0, st, idx, M, n, c.off, c.cur,
                           c.ent);
        HREG_CHECK_LAUNCH();
        hipLaunchKernelGGL(csr_sort_kernel, dim3(g1d(n)), dim3(TB), 0, st, n, c.off, c.ent);
        HREG_CHECK_LAUNCH();
    }
    return HREG_OK;
}

extern "C" int hreg_scatter_rows(const float *dy, int ldy, const void *ws, int M, int n, int C,
                                 float *dx, int ldx, int accumulate, void *stream) {
    if (!dy || !ws || !dx || M < 0 || n < 1 || C < 0 || ldy < C || ldx < C) return HREG_ERR_INVALID;
    if (!C) return HREG_OK;
    Csr c = csr_view(const_cast<void *>(ws), M, n);
    if (rows_v4(C, ldy, ldx, dy, dx, (size_t)n))
        hipLaunchKernelGGL(scatter_rows4_kernel, dim3(g1d((size_t)n * C / 4)), dim3(TB), 0,
                           as_stream(stream), reinterpret_cast<const float4 *>(dy), ldy / 4, c.off,
                           c.ent, n, C / 4, reinterpret_cast<float4 *>(dx), ldx / 4, accumulate);
    else
        hipLaunchKernelGGL(scatter_rows_kernel, dim3(g1d((size_t)n * C)), dim3(TB), 0,
                           as_stream(stream), dy, ldy, c.off, c.ent, n, C, dx, ldx, accumulate);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_geom_rows(const float *q, const float *knn_xyz, int G, int k, float *out,
                              int ldo, void *stream) {
    if (!q || !knn_xyz || !out || G < 0 || k < 1 || ldo < 4) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(geom_rows_kernel, dim3(g1d((size_t)G * k)), dim3(TB), 0, as_stream(stream),
                       q, knn_xyz, G, k, out, ldo);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_geom_rows_bwd(const float *geom, int ldg, const float *dgeom, int lddg,
                                  const float *dknn_extra, int G, int k, float *dq, float *dknn,
                                  void *stream) {
    if (!geom || !dgeom || G < 0 || k < 1 || ldg < 4 || lddg < 4) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(geom_rows_bwd_kernel, dim3(g1d(G)), dim3(TB), 0, as_stream(stream), geom, ldg,
                       dgeom, lddg, dknn_extra, G, k, dq, dknn);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_attention_fwd(const float *logits, int ldl, int C, const float *vals, int ldv,
                                  int Cv, const float *knn_xyz, int G, int k, float *a,
                                  int32_t *amax, float *kp, float *vmap, int ldm, float *vsum,
                                  int lds, void *stream) {
    if (!logits || G < 0 || k < 1 || k > 64 || C < 1 || ldl < C) return HREG_ERR_INVALID;
    if (vals && (ldv < Cv || Cv < 1)) return HREG_ERR_INVALID;
    if (kp && !knn_xyz) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(attention_fwd_kernel<false>, dim3(G), dim3(TB), 0, as_stream(stream), logits, ldl,
                       C, vals, ldv, Cv, knn_xyz, k, a, amax, kp, vmap, ldm, vsum, lds);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_attention_bwd(const float *logits, int ldl, int C, const float *vals, int ldv,
                                  int Cv, const float *knn_xyz, int G, int k, const float *a,
                                  const int32_t *amax, const float *dkp, const float *dvmap,
                                  int lddm, const float *dvsum, int ldds, int same,
                                  float *dlogits, int lddl, float *dvals, int lddv, float *dknn,
                                  void *stream) {
    if (!logits || !a || !amax || G < 0 || k < 1 || k > 64 || C < 1) return HREG_ERR_INVALID;
    if (dkp && !knn_xyz) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(attention_bwd_kernel<false>, dim3(G), dim3(TB), 0, as_stream(stream), logits, ldl,
                       C, vals, ldv, Cv, knn_xyz, k, a, amax, dkp, dvmap, lddm, dvsum, ldds, same,
                       dlogits, lddl, dvals, lddv, dknn);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// hreg_attention_fwd / _bwd over logits = vals = ReLU(BN(y)) of a pre-BN y [G*k][C] (the
// detector's last conv activation, never written; r6): every value of y enters as bn_act
// (hreg_bn_apply's arithmetic), so the outputs are those over the materialised activation; the
// backward's dlogits is d/d(activation) (the BN backward follows, train.py _BNActAttention)
extern "C" int hreg_attention_fwd_pre(const float *y, int ldy, int C, const float *mean, const float *invstd,
                                      const float *gamma, const float *beta, const float *knn_xyz, int G, int k,
                                      float *a, int32_t *amax, float *kp, float *vmap, int ldm, float *vsum,
                                      int lds, void *stream) {
    if (!y || !mean || !invstd || !gamma || !beta || G < 0 || k < 1 || k > 64 || C < 1 || ldy < C)
        return HREG_ERR_INVALID;
    if (kp && !knn_xyz) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(attention_fwd_kernel<true>, dim3(G), dim3(TB), 0, as_stream(stream), y, ldy, C, y, ldy, C,
                       knn_xyz, k, a, amax, kp, vmap, ldm, vsum, lds, AttPre{mean, invstd, gamma, beta});
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_attention_bwd_pre(const float *y, int ldy, int C, const float *mean, const float *invstd,
                                      const float *gamma, const float *beta, const float *knn_xyz, int G, int k,
                                      const float *a, const int32_t *amax, const float *dkp, const float *dvmap,
                                      int lddm, const float *dvsum, int ldds, float *dact, int ldda, float *dknn,
                                      void *stream) {
    if (!y || !mean || !invstd || !gamma || !beta || !a || !amax || !dact || G < 0 || k < 1 || k > 64 || C < 1)
        return HREG_ERR_INVALID;
    if (dkp && !knn_xyz) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(attention_bwd_kernel<true>, dim3(G), dim3(TB), 0, as_stream(stream), y, ldy, C, y, ldy, C,
                       knn_xyz, k, a, amax, dkp, dvmap, lddm, dvsum, ldds, 1, dact, ldda, nullptr, 0, dknn,
                       AttPre{mean, invstd, gamma, beta});
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_max_arg(const float *x, int ldx, int G, int k, int C, float *out,
                                  int ldo, int32_t *arg, void *stream) {
    if (!x || !out || !arg || G < 0 || k < 1 || C < 0 || ldx < C || ldo < C) return HREG_ERR_INVALID;
    if (!G || !C) return HREG_OK;
    hipLaunchKernelGGL(group_max_arg_kernel<false>, dim3(g1d((size_t)G * C)), dim3(TB), 0,
                       as_stream(stream), x, ldx, G, k, C, out, ldo, arg, nullptr, nullptr, nullptr, nullptr);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_max_arg_pre(const float *x, int ldx, int G, int k, int C, float *out, int ldo,
                                      int32_t *arg, const float *mean, const float *invstd, const float *gamma,
                                      const float *beta, void *stream) {
    if (!x || !out || !arg || !mean || !invstd || !gamma || !beta || G < 0 || k < 1 || C < 0 || ldx < C ||
        ldo < C)
        return HREG_ERR_INVALID;
    if (!G || !C) return HREG_OK;
    hipLaunchKernelGGL(group_max_arg_kernel<true>, dim3(g1d((size_t)G * C)), dim3(TB), 0,
                       as_stream(stream), x, ldx, G, k, C, out, ldo, arg, mean, invstd, gamma, beta);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_max_bwd(const float *dout, int ldd, const int32_t *arg, int G, int k,
                                  int C, float *dx, int ldx, int accumulate, void *stream) {
    if (!dout || !arg || !dx || G < 0 || k < 1 || C < 0 || ldd < C || ldx < C) return HREG_ERR_INVALID;
    if (!G || !C) return HREG_OK;
    hipLaunchKernelGGL(group_max_bwd_kernel, dim3(g1d((size_t)G * C)), dim3(TB), 0,
                       as_stream(stream), dout, ldd, arg, G, k, C, dx, ldx, accumulate);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_head_out_bwd(const float *x, int ldx, int C, const float *w3, const float *b3,
                                 const float *dy, int mode, int G, float *dz, float *dx, int lddx,
                                 void *stream) {
    if (!x || !w3 || !b3 || !dy || !dz || !dx || G < 0 || C < 1 || ldx < C || lddx < C)
        return HREG_ERR_INVALID;
    if (mode != HREG_HEAD_SOFTPLUS && mode != HREG_HEAD_SIGMOID) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    hipLaunchKernelGGL(head_out_bwd_kernel, dim3((G + 3) / 4), dim3(TB), 0, as_stream(stream), x,
                       ldx, C, w3, b3, dy, mode, G, dz, dx, lddx);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_sim_stats(const float *S, int nb, int N1, int N2, float *rmax, int32_t *rarg,
                              float *cmax, int32_t *carg, void *stream) {
    if (!S || !rmax || !rarg || !cmax || !carg || nb < 0 || N1 < 1 || N2 < 1) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(sim_stats_kernel, dim3(g1d((size_t)nb * (N1 + N2))), dim3(TB), 0,
                       as_stream(stream), S, nb, N1, N2, rmax, rarg, cmax, carg);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_sim_feats(const float *S, int nb, int N1, int N2, const int32_t *kidx, int k,
                              const float *rmax, const float *cmax, float *out, int ldo,
                              void *stream) {
    if (!S || !kidx || !rmax || !cmax || !out || nb < 0 || N1 < 1 || N2 < 1 || k < 1 || ldo < 2)
        return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(sim_feats_kernel, dim3(g1d((size_t)nb * N1 * k)), dim3(TB), 0,
                       as_stream(stream), S, nb, N1, N2, kidx, k, rmax, cmax, out, ldo);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" size_t hreg_sim_feats_bwd_ws_bytes(int nb, int N1, int N2) {
    return ((size_t)2 * nb * N1 * N2 + (size_t)nb * (N1 + N2)) * sizeof(float);
}

// a [nb][N1][C], b [nb][N2][C] (descriptors), na / nb_ their norms, S the cosine matrix;
// dout [nb*N1*k][ldd] the gradient of the two sim_feats columns -> da, db (written)
extern "C" int hreg_sim_feats_bwd(const float *S, const float *a, const float *b, const float *na,
                                  const float *nb_, int nb, int N1, int N2, int C,
                                  const int32_t *kidx, int k, const float *rmax,
                                  const int32_t *rarg, const float *cmax, const int32_t *carg,
                                  const float *dout, int ldd, void *ws, float *da, float *db,
                                  void *stream) {
    if (!S || !a || !b || !na || !nb_ || !kidx || !rmax || !rarg || !cmax || !carg || !dout ||
        !ws || !da || !db || nb < 0 || N1 < 1 || N2 < 1 || C < 1 || k < 1 || ldd < 2)
        return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipStream_t st = as_stream(stream);
    float *dS = (float *)ws;
    float *dP = dS + (size_t)nb * N1 * N2;
    float *dna = dP + (size_t)nb * N1 * N2;
    float *dnb = dna + (size_t)nb * N1;
    if (hipMemsetAsync(dS, 0, (size_t)nb * N1 * N2 * sizeof(float), st) != hipSuccess)
        return HREG_ERR_LAUNCH;
    hipLaunchKernelGGL(sim_bwd_rows_kernel, dim3(g1d((size_t)nb * N1)), dim3(TB), 0, st, S, nb, N1,
                       N2, kidx, k, rmax, rarg, cmax, dout, ldd, dS);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sim_bwd_cols_kernel, dim3(g1d((size_t)nb * N2 * 64)), dim3(TB), 0, st, S, nb, N1,
                       N2, kidx, k, cmax, carg, dout, ldd, dS);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sim_bwd_cos_rows_kernel, dim3(g1d((size_t)nb * N1 * 64)), dim3(TB), 0, st, S,
                       dS, nb, N1, N2, na, nb_, dP, dna);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sim_bwd_cos_cols_kernel, dim3(nb * ((N2 + 63) / 64)), dim3(64 * COS_SL), 0,
                       st, S, dS, nb, N1, N2, na, nb_, dnb);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sim_bwd_mm_kernel<false>, dim3((C + 63) / 64, (N1 + 63) / 64, nb), dim3(TB),
                       0, st, dP, N1, N2, b, a, dna, na, C, da);
    HREG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sim_bwd_mm_kernel<true>, dim3((C + 63) / 64, (N2 + 63) / 64, nb), dim3(TB),
                       0, st, dP, N1, N2, a, b, dnb, nb_, C, db);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_weighted_svd_bwd(const float *src, const float *corres, const float *w, int nb,
                                     int n, const float *dR, const float *dt, float *dsrc,
                                     float *dcorres, float *dw, void *stream) {
    if (!src || !corres || !w || !dR || !dt || !dsrc || !dcorres || !dw || nb < 0 || n < 1)
        return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(svd_bwd_kernel, dim3(nb), dim3(TB), 0, as_stream(stream), src, corres, w, n,
                       dR, dt, dsrc, dcorres, dw);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_transform_points_bwd(const float *xyz, const float *R, int nb, int n,
                                         const float *dy, float *dxyz, float *dR, float *dt,
                                         void *stream) {
    if (!xyz || !R || !dy || nb < 0 || n < 1) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(transform_bwd_kernel, dim3(nb), dim3(TB), 0, as_stream(stream), xyz, R, n, dy,
                       dxyz, dR, dt);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_compose_se3(int nb, const float *Ra, const float *ta, const float *Rb,
                                const float *tb, float *Ro, float *to, void *stream) {
    if (!Ra || !ta || !Rb || !tb || !Ro || !to || nb < 0) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(compose_kernel, dim3(g1d(nb)), dim3(TB), 0, as_stream(stream), nb, Ra, ta, Rb,
                       tb, Ro, to);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_compose_se3_bwd(int nb, const float *Ra, const float *Rb, const float *tb,
                                    const float *dRo, const float *dto, float *dRa, float *dta,
                                    float *dRb, float *dtb, void *stream) {
    if (!Ra || !Rb || !tb || !dRo || !dto || !dRa || !dta || !dRb || !dtb || nb < 0)
        return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(compose_bwd_kernel, dim3(g1d(nb)), dim3(TB), 0, as_stream(stream), nb, Ra, Rb,
                       tb, dRo, dto, dRa, dta, dRb, dtb);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_transformation_loss_bwd(const float *pred_R, const float *pred_t,
                                            const float *gt_R, const float *gt_t, int nb,
                                            float alpha, float scale, const float *dloss,
                                            float *dR, float *dt, void *stream) {
    if (!pred_R || !pred_t || !gt_R || !gt_t || !dR || !dt || nb < 0) return HREG_ERR_INVALID;
    if (!nb) return HREG_OK;
    hipLaunchKernelGGL(loss_bwd_kernel, dim3(g1d(nb)), dim3(TB), 0, as_stream(stream), pred_R, pred_t,
                       gt_R, gt_t, nb, alpha, scale, dloss, dR, dt);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
