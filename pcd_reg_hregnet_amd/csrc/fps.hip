// fps.hip -- farthest point sampling (plain and weighted) for gfx950.
//
// Replaces furthest_point_sampling_kernel / weighted_furthest_point_sampling_kernel
// (reference models/PointUtils/src/furthest_point_sampling_gpu.cu:84-206, :254-375).
// Not a translation: one workgroup per cloud keeps every point, its running
// minimum distance ("temp") and its weight in VGPRs for all m-1 dependent
// iterations (no HBM traffic inside the loop), and the per-iteration argmax
// is one 64-bit max over a packed key
//     key = orderable(d2) << 32 | ~rank,   rank = r' * Q + i
// which is tree-independent and reproduces the reference winner exactly.
//
// The reference winner ("FPS tie rule"): with bs =
// opt_n_threads(n) "threads" (cuda_utils.h:22-26), reference thread r scans
// k = r, r+bs, ... keeping the first strictly larger d2 (.cu:132-133); the
// shared-memory tree keeps the lower slot on ties (.cu:75-80), so among equal
// maxima the thread with the smallest bit-reversed id wins, then the smallest
// k.  Here reference thread r = bitrev_L(r') is handled by our thread r'/G
// (slot g = r' % G), and its points k = r + i*bs are scanned in order i, so
// "first strictly larger" inside our thread plus "smallest rank" across
// threads is the same order.  Initial best = -1 at k = 0 (rank 0) reproduces
// the reference's (best=-1, besti=0) start (.cu:115-116).
//
// The winner's coordinates come back through one broadcast global load
// (L2-resident cloud); the LDS slot is double-buffered by iteration parity so
// there is exactly one barrier per iteration (the reference re-reads
// dists_i[0] without a barrier: SURVEY.md 5, latent WAR race).
#include "common.h"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}

// max over each 16-lane row (quad_perm 1032, 2301, row_half_mirror, row_mirror)
__device__ __forceinline__ float row_max16(float v, float inf) {
    v = fmax_nc(v, dppf<0xb1>(v), inf);
    v = fmax_nc(v, dppf<0x4e>(v), inf);
    v = fmax_nc(v, dppf<0x141>(v), inf);
    v = fmax_nc(v, dppf<0x140>(v), inf);
    return v;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ float wave_max_uniform(float v, float inf) {
    v = row_max16(v, inf);
    return fmax_nc(fmax_nc(readlane_f(v, 0), readlane_f(v, 16), inf),
                   fmax_nc(readlane_f(v, 32), readlane_f(v, 48), inf), inf);
}

// Per iteration: packed (v_pk_*) distance update of S register-resident points,
// running max via max3; the wave's winner = max value, lowest lane (= lowest
// rank), first slot; DPP row reductions + ballot instead of a shuffle tree.
// Each wave publishes (x, y, z, d2, rank) of its winner in LDS (double
// buffered), one barrier, then a 16-lane DPP reduction picks the block winner.
template <int T, int S, bool WEIGHTED>
__global__ __launch_bounds__(T) void fps_reg_kernel(const float *__restrict__ xyz,
                                                    const float *__restrict__ wts,
                                                    float *__restrict__ temp_out,
                                                    int32_t *__restrict__ idx_out,
                                                    float *__restrict__ sampled_out, int n,
                                                    int m, int bs, int L, int G, int Q,
                                                    float inf) {
    constexpr int NW = T / HREG_WAVE;
    constexpr int S2 = (S + 1) / 2;
    static_assert(NW <= 16, "block winner reduction uses one 16-lane row");
    __shared__ float4 s_cand[2][NW];
    __shared__ int s_rank[2][NW];

    const int cloud = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const float *P = xyz + (size_t)cloud * n * 3;
    const float *W = WEIGHTED ? wts + (size_t)cloud * n : nullptr;

    f2 PX[S2], PY[S2], PZ[S2], PT[S2], PW[S2];
#pragma unroll
    for (int s = 0; s < 2 * S2; ++s) {
        const int g = s / Q, i = s % Q;
        const int rp = tid * G + g;  // position in bit-reversed thread order
        const int k = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
        const bool ok = (s < S) && (s < G * Q) && (rp < bs) && (k < n);
        const int kk = ok ? k : 0;
        PX[s / 2][s % 2] = P[kk * 3 + 0];
        PY[s / 2][s % 2] = P[kk * 3 + 1];
        PZ[s / 2][s % 2] = P[kk * 3 + 2];
        PW[s / 2][s % 2] = WEIGHTED ? W[kk] : 1.0f;
        // invalid slots can never be selected: d2 = -inf never reaches the max
        PT[s / 2][s % 2] = ok ? 1e10f : -__builtin_huge_valf();
    }

    float x1 = P[0], y1 = P[1], z1 = P[2];
    if (tid == 0) {
        idx_out[(size_t)cloud * m] = 0;
        if (sampled_out) {
            float *o = sampled_out + (size_t)cloud * m * 3;
            o[0] = x1; o[1] = y1; o[2] = z1;
        }
    }

    for (int j = 1; j < m; ++j) {
        const f2 X1 = {x1, x1}, Y1 = {y1, y1}, Z1 = {z1, z1};
        float best = -1.0f;
#pragma unroll
        for (int s = 0; s < S2; ++s) {
            const f2 dx = PX[s] - X1, dy = PY[s] - Y1, dz = PZ[s] - Z1;
            f2 d = (dx * dx + dy * dy) + dz * dz;
            if (WEIGHTED) d = PW[s] * d;
            f2 t;
            t.x = fmin_nc(d.x, PT[s].x, inf);
            t.y = fmin_nc(d.y, PT[s].y, inf);
            PT[s] = t;
            best = fmax_nc(best, fmax_nc(t.x, t.y, inf), inf);
        }
        const float wmax = wave_max_uniform(best, inf);
        // first slot holding the wave max, in this lane
        int myslot = 2 * S2;
#pragma unroll
        for (int s = 2 * S2 - 1; s >= 0; --s)
            myslot = (PT[s / 2][s % 2] == wmax) ? s : myslot;
        const uint64_t hit = __ballot(best == wmax);
        const int wl = (int)__builtin_ctzll(hit);  // lowest lane = lowest rank
        const int sl = __builtin_amdgcn_readlane(myslot, wl);
        const int rp = (wv * 64 + wl) * G + sl / Q;
        const int rank = rp * Q + sl % Q;
        const int kw = (int)bitrev_bits((uint32_t)rp, L) + (sl % Q) * bs;
        const int buf = j & 1;
        if (lane == 0) {
            const float *pw = P + (size_t)kw * 3;
            s_cand[buf][wv] = make_float4(pw[0], pw[1], pw[2], wmax);
            s_rank[buf][wv] = rank;
        }
        __syncthreads();
        const float4 c = lane < NW ? s_cand[buf][lane] : make_float4(0.f, 0.f, 0.f, -__builtin_huge_valf());
        const float gmax = readlane_f(row_max16(c.w, inf), 0);
        const uint64_t ghit = __ballot(lane < NW && c.w == gmax);
        const int gw = (int)__builtin_ctzll(ghit);
        int old;
        if (gmax > -1.0f) {
            const int grank = __builtin_amdgcn_readlane(s_rank[buf][lane < NW ? lane : 0], gw);
            old = (int)bitrev_bits((uint32_t)(grank / Q), L) + (grank % Q) * bs;
            x1 = readlane_f(c.x, gw);
            y1 = readlane_f(c.y, gw);
            z1 = readlane_f(c.z, gw);
        } else {  // no d2 > -1 anywhere: the reference keeps (best=-1, besti=0)
            old = 0;
            x1 = P[0]; y1 = P[1]; z1 = P[2];
        }
        if (tid == 0) {
            idx_out[(size_t)cloud * m + j] = old;
            if (sampled_out) {
                float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
    }

    if (temp_out) {
        float *tp = temp_out + (size_t)cloud * n;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int g = s / Q, i = s % Q;
            const int rp = tid * G + g;
            const int k = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
            if ((s < G * Q) && (rp < bs) && (k < n)) tp[k] = PT[s / 2][s % 2];
        }
    }
}

// Fallback for clouds too large for the register-resident path (S > 16):
// temp lives in the caller's buffer; same key, same winner.
template <bool WEIGHTED>
__global__ __launch_bounds__(1024) void fps_mem_kernel(const float *__restrict__ xyz,
                                                      const float *__restrict__ wts,
                                                      float *__restrict__ temp,
                                                      int32_t *__restrict__ idx_out,
                                                      float *__restrict__ sampled_out, int n,
                                                      int m, int bs, int L, int Q) {
    constexpr int T = 1024, NW = T / HREG_WAVE;
    __shared__ uint64_t red[2][NW];
    const int cloud = blockIdx.x;
    const int tid = threadIdx.x;
    const float *P = xyz + (size_t)cloud * n * 3;
    const float *W = WEIGHTED ? wts + (size_t)cloud * n : nullptr;
    float *tp = temp + (size_t)cloud * n;
    const int G = bs / T > 0 ? bs / T : 1;
    for (int k = tid; k < n; k += T) tp[k] = 1e10f;
    __syncthreads();
    float x1 = P[0], y1 = P[1], z1 = P[2];
    if (tid == 0) {
        idx_out[(size_t)cloud * m] = 0;
        if (sampled_out) {
            float *o = sampled_out + (size_t)cloud * m * 3;
            o[0] = x1; o[1] = y1; o[2] = z1;
        }
    }
    for (int j = 1; j < m; ++j) {
        float best = -1.0f;
        uint32_t brank = 0;
        bool have = false;
        for (int g = 0; g < G; ++g) {
            const int rp = tid * G + g;
            if (rp >= bs) break;
            const int r = (int)bitrev_bits((uint32_t)rp, L);
            for (int i = 0; i < Q; ++i) {
                const int k = r + i * bs;
                if (k >= n) break;
                float d = sqdist3(P[k * 3], P[k * 3 + 1], P[k * 3 + 2], x1, y1, z1);
                if (WEIGHTED) d = fmul_rn(W[k], d);
                const float d2 = fminf(d, tp[k]);
                tp[k] = d2;
                if (d2 > best) { best = d2; brank = (uint32_t)(rp * Q + i); have = true; }
            }
        }
        if (!have) brank = 0;
        uint64_t key = ((uint64_t)float_orderable(best) << 32) | (uint64_t)(0xffffffffu - brank);
        key = wave_max_u64(key);
        const int buf = j & 1;
        if ((tid & (HREG_WAVE - 1)) == 0) red[buf][tid / HREG_WAVE] = key;
        __syncthreads();
        uint64_t k2 = red[buf][0];
        for (int w = 1; w < NW; ++w) { const uint64_t o = red[buf][w]; k2 = o > k2 ? o : k2; }
        const uint32_t wr = 0xffffffffu - (uint32_t)(k2 & 0xffffffffu);
        const int old = (int)bitrev_bits(wr / (uint32_t)Q, L) + (int)(wr % (uint32_t)Q) * bs;
        x1 = P[old * 3 + 0];
        y1 = P[old * 3 + 1];
        z1 = P[old * 3 + 2];
        if (tid == 0) {
            idx_out[(size_t)cloud * m + j] = old;
            if (sampled_out) {
                float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
    }
}

template <bool WEIGHTED>
int launch_fps(int b, int n, int m, const float *xyz, const float *w, float *temp, int32_t *idx,
               float *sampled, hipStream_t st) {
    if (b < 0 || n <= 0 || xyz == nullptr || idx == nullptr) return HREG_ERR_INVALID;
    if (WEIGHTED && w == nullptr) return HREG_ERR_INVALID;
    if (b == 0 || m <= 0) return HREG_OK;  // .cu:92: if (m <= 0) return;
    const int bs = hreg_opt_n_threads(n);
    const int L = hreg_ilog2(bs);
    const int Q = (n + bs - 1) / bs;
    // choose our thread count T and slots per thread S = G * Q (T * G == bs)
    int T, G;
    if (Q == 1 && bs >= 256) { T = bs / 4; G = 4; }
    else if (bs >= 64) { T = bs; G = 1; }
    else { T = 64; G = 1; }
    // keep the per-slot registers (x, y, z, temp[, w]) inside the VGPR budget
    const int smax1024 = WEIGHTED ? 8 : 16;
    if (T == 1024 && G * Q > smax1024) { T = 512; G = 2; }
    const int S = G * Q;
#define HREG_FPS_CASE(TT, SS)                                                                 \
    if (T == TT && S <= SS) {                                                                 \
        hipLaunchKernelGGL((fps_reg_kernel<TT, SS, WEIGHTED>), dim3(b), dim3(TT), 0, st, xyz, \
                           w, temp, idx, sampled, n, m, bs, L, G, Q, __builtin_huge_valf());  \
        HREG_CHECK_LAUNCH();                                                                  \
        return HREG_OK;                                                                       \
    }
    HREG_FPS_CASE(1024, 1) HREG_FPS_CASE(1024, 2) HREG_FPS_CASE(1024, 4)
    HREG_FPS_CASE(1024, 8)
    if constexpr (!WEIGHTED) { HREG_FPS_CASE(1024, 16) }
    HREG_FPS_CASE(512, 2) HREG_FPS_CASE(512, 4) HREG_FPS_CASE(512, 8) HREG_FPS_CASE(512, 16)
    HREG_FPS_CASE(512, 32)
    HREG_FPS_CASE(256, 4) HREG_FPS_CASE(256, 8) HREG_FPS_CASE(256, 16)
    HREG_FPS_CASE(128, 4) HREG_FPS_CASE(128, 8) HREG_FPS_CASE(128, 16)
    HREG_FPS_CASE(64, 1) HREG_FPS_CASE(64, 2) HREG_FPS_CASE(64, 4) HREG_FPS_CASE(64, 8)
    HREG_FPS_CASE(64, 16)
#undef HREG_FPS_CASE
    // large clouds: temp through memory (caller's temp buffer is required)
    if (temp == nullptr) return HREG_ERR_INVALID;
    hipLaunchKernelGGL((fps_mem_kernel<WEIGHTED>), dim3(b), dim3(1024), 0, st, xyz, w, temp, idx,
                       sampled, n, m, bs, L, Q);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_furthest_point_sampling(int b, int n, int m, const float *points,
                                            float *temp, int32_t *idx, float *sampled_xyz,
                                            void *stream) {
    return launch_fps<false>(b, n, m, points, nullptr, temp, idx, sampled_xyz, as_stream(stream));
}

extern "C" int hreg_weighted_furthest_point_sampling(int b, int n, int m, const float *points,
                                                     const float *weights, float *temp,
                                                     int32_t *idx, float *sampled_xyz,
                                                     void *stream) {
    return launch_fps<true>(b, n, m, points, weights, temp, idx, sampled_xyz, as_stream(stream));
}
