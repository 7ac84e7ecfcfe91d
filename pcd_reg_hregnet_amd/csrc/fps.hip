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

template <int T, int S, bool WEIGHTED>
__global__ __launch_bounds__(T) void fps_reg_kernel(const float *__restrict__ xyz,
                                                    const float *__restrict__ wts,
                                                    float *__restrict__ temp_out,
                                                    int32_t *__restrict__ idx_out,
                                                    float *__restrict__ sampled_out, int n,
                                                    int m, int bs, int L, int G, int Q) {
    constexpr int NW = T / HREG_WAVE;
    __shared__ uint64_t red[2][NW];

    const int cloud = blockIdx.x;
    const int tid = threadIdx.x;
    const float *P = xyz + (size_t)cloud * n * 3;
    const float *W = WEIGHTED ? wts + (size_t)cloud * n : nullptr;

    float px[S], py[S], pz[S], pt[S], pw[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int g = s / Q, i = s % Q;
        const int rp = tid * G + g;  // position in bit-reversed thread order
        const int k = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
        const bool ok = (s < G * Q) && (rp < bs) && (k < n);
        const int kk = ok ? k : 0;
        px[s] = P[kk * 3 + 0];
        py[s] = P[kk * 3 + 1];
        pz[s] = P[kk * 3 + 2];
        pw[s] = WEIGHTED ? W[kk] : 1.0f;
        // invalid slots can never be selected: d2 = -inf is never > best
        pt[s] = ok ? 1e10f : -__builtin_huge_valf();
    }

    int old = 0;
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
        int bslot = -1;  // -1 == the reference's (best=-1, besti=0) start
#pragma unroll
        for (int s = 0; s < S; ++s) {
            float d = sqdist3(px[s], py[s], pz[s], x1, y1, z1);
            if (WEIGHTED) d = fmul_rn(pw[s], d);
            const float d2 = fminf(d, pt[s]);
            pt[s] = d2;
            const bool gt = d2 > best;
            best = gt ? d2 : best;
            bslot = gt ? s : bslot;
        }
        uint32_t rank = 0;
        if (bslot >= 0) {
            const int g = bslot / Q, i = bslot % Q;
            rank = (uint32_t)((tid * G + g) * Q + i);
        }
        uint64_t key = ((uint64_t)float_orderable(best) << 32) | (uint64_t)(0xffffffffu - rank);
        key = wave_max_u64(key);
        const int buf = j & 1;
        if ((tid & (HREG_WAVE - 1)) == 0) red[buf][tid / HREG_WAVE] = key;
        __syncthreads();
        uint64_t k2 = red[buf][0];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
            const uint64_t o = red[buf][w];
            k2 = o > k2 ? o : k2;
        }
        const uint32_t wr = 0xffffffffu - (uint32_t)(k2 & 0xffffffffu);
        const int rp = (int)(wr / (uint32_t)Q), i = (int)(wr % (uint32_t)Q);
        old = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
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

    if (temp_out) {
        float *tp = temp_out + (size_t)cloud * n;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int g = s / Q, i = s % Q;
            const int rp = tid * G + g;
            const int k = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
            if ((s < G * Q) && (rp < bs) && (k < n)) tp[k] = pt[s];
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
                           w, temp, idx, sampled, n, m, bs, L, G, Q);                         \
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
