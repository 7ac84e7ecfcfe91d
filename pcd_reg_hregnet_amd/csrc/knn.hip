// knn.hip -- exact K-nearest-neighbour selection for gfx950 (K <= 64).
//
// Replaces pytorch3d.ops.knn_points / knn_gather (pinned pytorch3d 0.7.8,
// Dockerfile:44-46; call sites models/HRegNet/layers.py:20,278,316,322,434)
// and fuses knn_group (layers.py:9-27).
//
// One wave per query.  The wave keeps the current best 64 candidates as a
// sorted list of packed keys (dist_bits << 32 | idx), one per lane; keys order
// exactly as (dist, idx) ascending (dist >= 0), which is the canonical tie
// order (pytorch3d's own tie order is an unstable sort: parity unpinned,
// SURVEY.md 8c).  The database is scanned 64 points per step; a point is a
// candidate only if its key beats the current K-th key (exact filter: a
// later index with an equal distance can never enter).  Candidates are
// compacted (ballot + mbcnt) into a per-wave LDS buffer; every 64 buffered
// candidates are bitonic-sorted across lanes and merged into the list
// (min(A[j], B[63-j]) + bitonic merge).  Distances use the reference order
// sum_d (q_d - p_d)^2, non-contracted, sequential in d.
#include "common.h"

namespace {

constexpr int WAVES = 4;
constexpr uint64_t KEY_INF = ~0ull;

__device__ __forceinline__ uint64_t u64min(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t u64max(uint64_t a, uint64_t b) { return a < b ? b : a; }

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const uint32_t lo = __shfl((unsigned)(v & 0xffffffffu), src);
    const uint32_t hi = __shfl((unsigned)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void wave_fence() { wave_sync(); }

// ascending bitonic sort of one key per lane
__device__ __forceinline__ uint64_t bitonic_sort64(uint64_t v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = shfl_xor_u64(v, j);
            const bool up = (lane & k) == 0;
            const bool lower = (lane & j) == 0;
            v = (lower == up) ? u64min(v, o) : u64max(v, o);
        }
    }
    return v;
}

// merge two ascending 64-lists, keep the 64 smallest, ascending
__device__ __forceinline__ uint64_t merge64(uint64_t a, uint64_t b_sorted, int lane) {
    const uint64_t br = shfl_u64(b_sorted, 63 - lane);
    uint64_t v = u64min(a, br);
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        const uint64_t o = shfl_xor_u64(v, j);
        v = ((lane & j) == 0) ? u64min(v, o) : u64max(v, o);
    }
    return v;
}

struct WaveList {
    uint64_t key;  // lane j: j-th best
    uint64_t tau;  // key of the K-th best (broadcast)
    int cnt;       // buffered candidates
};

template <int K>
__device__ __forceinline__ void flush64(WaveList &L, uint64_t *buf, int lane) {
    wave_fence();
    const uint64_t c = lane < L.cnt ? buf[lane] : KEY_INF;
    const uint64_t s = bitonic_sort64(c, lane);
    L.key = merge64(L.key, s, lane);
    wave_fence();
    const int rest = L.cnt - 64;
    if (rest > 0 && lane < rest) buf[lane] = buf[64 + lane];
    wave_fence();
    L.cnt = rest > 0 ? rest : 0;
    L.tau = shfl_u64(L.key, K - 1);
}

template <int K>
__device__ __forceinline__ void offer(WaveList &L, uint64_t *buf, uint64_t key, int lane) {
    const bool take = key < L.tau;
    const uint64_t mask = __ballot(take);
    if (mask) {
        const int pos = L.cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
        if (take) buf[pos] = key;
        L.cnt += __popcll(mask);
        if (L.cnt >= 64) flush64<K>(L, buf, lane);
    }
}

// ---- dim == 3 ----------------------------------------------------------
template <int K>
__device__ void knn3_query(const float *__restrict__ P, int n2, float qx, float qy, float qz,
                           uint64_t *buf, int lane, WaveList &L) {
    L.key = KEY_INF; L.tau = KEY_INF; L.cnt = 0;
    for (int base = 0; base < n2; base += 64) {
        const int p = base + lane;
        uint64_t key = KEY_INF;
        if (p < n2) {
            const float d = sqdist3(qx, qy, qz, P[p * 3 + 0], P[p * 3 + 1], P[p * 3 + 2]);
            key = ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)p;
        }
        offer<K>(L, buf, key, lane);
    }
    if (L.cnt > 0) flush64<K>(L, buf, lane);
}

template <int K>
__global__ __launch_bounds__(256) void knn3_kernel(const float *__restrict__ q,
                                                   const float *__restrict__ p, int nb, int n1,
                                                   int n2, float *__restrict__ dists,
                                                   int64_t *__restrict__ idx64,
                                                   int32_t *__restrict__ idx32,
                                                   float *__restrict__ nn, int k) {
    __shared__ uint64_t sbuf[WAVES][128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qi = blockIdx.x * WAVES + w;
    if (qi >= nb * n1) return;
    const int cloud = qi / n1;
    const float *P = p + (size_t)cloud * n2 * 3;
    const float qx = q[(size_t)qi * 3], qy = q[(size_t)qi * 3 + 1], qz = q[(size_t)qi * 3 + 2];
    WaveList L;
    knn3_query<K>(P, n2, qx, qy, qz, sbuf[w], lane, L);
    if (lane < k) {
        const bool valid = L.key != KEY_INF;
        const int id = valid ? (int)(uint32_t)(L.key & 0xffffffffu) : -1;
        const size_t o = (size_t)qi * k + lane;
        if (dists) dists[o] = valid ? __uint_as_float((uint32_t)(L.key >> 32)) : 0.f;
        if (idx64) idx64[o] = id;
        if (idx32) idx32[o] = id;
        if (nn) {
            nn[o * 3 + 0] = valid ? P[id * 3 + 0] : 0.f;
            nn[o * 3 + 1] = valid ? P[id * 3 + 1] : 0.f;
            nn[o * 3 + 2] = valid ? P[id * 3 + 2] : 0.f;
        }
    }
}

// knn_group: global neighbour rows + (p - q, |p - q|) + neighbour xyz
template <int K>
__global__ __launch_bounds__(256) void knn_group_kernel(const float *__restrict__ q,
                                                        const float *__restrict__ p, int nb, int m,
                                                        int n, int k, int32_t *__restrict__ gidx,
                                                        float *__restrict__ geom,
                                                        float *__restrict__ knn_xyz) {
    __shared__ uint64_t sbuf[WAVES][128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qi = blockIdx.x * WAVES + w;
    if (qi >= nb * m) return;
    const int cloud = qi / m;
    const float *P = p + (size_t)cloud * n * 3;
    const float qx = q[(size_t)qi * 3], qy = q[(size_t)qi * 3 + 1], qz = q[(size_t)qi * 3 + 2];
    WaveList L;
    knn3_query<K>(P, n, qx, qy, qz, sbuf[w], lane, L);
    if (lane < k) {
        const size_t r = (size_t)qi * k + lane;
        const bool valid = L.key != KEY_INF;
        const int id = valid ? (int)(uint32_t)(L.key & 0xffffffffu) : 0;
        const float px = P[id * 3], py = P[id * 3 + 1], pz = P[id * 3 + 2];
        const float rx = fsub_rn(px, qx), ry = fsub_rn(py, qy), rz = fsub_rn(pz, qz);
        const float d2 = fadd_rn(fadd_rn(fmul_rn(rx, rx), fmul_rn(ry, ry)), fmul_rn(rz, rz));
        gidx[r] = cloud * n + id;
        float4 gv = make_float4(rx, ry, rz, sqrtf(d2));
        *reinterpret_cast<float4 *>(geom + r * 4) = gv;
        if (knn_xyz) {
            knn_xyz[r * 3 + 0] = px;
            knn_xyz[r * 3 + 1] = py;
            knn_xyz[r * 3 + 2] = pz;
        }
    }
}

// ---- general dim (descriptor space) ------------------------------------
// A block takes 16 queries (4 per wave) against 64 database rows at a time:
// the 64 rows x 64 dims and the 16 queries x 64 dims are staged in LDS
// (padded stride 65), lane = database row, so each wave ends a chunk with the
// 64 distances of its 4 queries in registers, one per lane, and offers them to
// the queries' lists.  Dims accumulate in order (canonical distance).
constexpr int QPW = 4;  // queries per wave

template <int K>
__global__ __launch_bounds__(256) void knnd_kernel(const float *__restrict__ q,
                                                   const float *__restrict__ p, int nb, int n1,
                                                   int n2, int dim, float *__restrict__ dists,
                                                   int64_t *__restrict__ idx64,
                                                   int32_t *__restrict__ idx32,
                                                   float *__restrict__ nn, int k) {
    constexpr int QB = WAVES * QPW;
    __shared__ uint64_t sbuf[WAVES][QPW][128];
    __shared__ float tile[64 * 65];
    __shared__ float qt[QB * 65];
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int nq = nb * n1;
    const int q0 = blockIdx.x * QB;  // queries of one block never straddle clouds: n1 % QB == 0
    const int cloud = q0 / n1;
    const float *P = p + (size_t)cloud * n2 * dim;
    WaveList L[QPW];
#pragma unroll
    for (int u = 0; u < QPW; ++u) { L[u].key = KEY_INF; L[u].tau = KEY_INF; L[u].cnt = 0; }
    for (int base = 0; base < n2; base += 64) {
        float acc[QPW];
#pragma unroll
        for (int u = 0; u < QPW; ++u) acc[u] = 0.f;
        for (int d0 = 0; d0 < dim; d0 += 64) {
            const int dc = min(64, dim - d0);
            __syncthreads();
            for (int e = tid; e < 64 * 64; e += 256) {
                const int rr = e >> 6, cc = e & 63;
                const int row = base + rr;
                tile[rr * 65 + cc] = (row < n2 && cc < dc) ? P[(size_t)row * dim + d0 + cc] : 0.f;
            }
            for (int e = tid; e < QB * 64; e += 256) {
                const int rr = e >> 6, cc = e & 63;
                const int qi = q0 + rr;
                qt[rr * 65 + cc] = (qi < nq && cc < dc) ? q[(size_t)qi * dim + d0 + cc] : 0.f;
            }
            __syncthreads();
            for (int e = 0; e < dc; ++e) {
                const float pv = tile[lane * 65 + e];
#pragma unroll
                for (int u = 0; u < QPW; ++u) {
                    const float diff = fsub_rn(qt[(w * QPW + u) * 65 + e], pv);
                    acc[u] = fadd_rn(acc[u], fmul_rn(diff, diff));
                }
            }
        }
        const int pi = base + lane;
#pragma unroll
        for (int u = 0; u < QPW; ++u) {
            const uint64_t key =
                pi < n2 ? (((uint64_t)__float_as_uint(acc[u]) << 32) | (uint32_t)pi) : KEY_INF;
            offer<K>(L[u], sbuf[w][u], key, lane);
        }
    }
#pragma unroll
    for (int u = 0; u < QPW; ++u) {
        if (L[u].cnt > 0) flush64<K>(L[u], sbuf[w][u], lane);
        const int qi = q0 + w * QPW + u;
        if (qi < nq && lane < k) {
            const bool valid = L[u].key != KEY_INF;
            const int id = valid ? (int)(uint32_t)(L[u].key & 0xffffffffu) : -1;
            const size_t o = (size_t)qi * k + lane;
            if (dists) dists[o] = valid ? __uint_as_float((uint32_t)(L[u].key >> 32)) : 0.f;
            if (idx64) idx64[o] = id;
            if (idx32) idx32[o] = id;
            if (nn)
                for (int e = 0; e < dim; ++e) nn[o * dim + e] = valid ? P[(size_t)id * dim + e] : 0.f;
        }
    }
}

template <int K>
int launch_knn(const float *p1, const float *p2, int b, int n1, int n2, int dim, int k,
               float *dists, int64_t *idx64, int32_t *idx32, float *nn, hipStream_t st) {
    const int nq = b * n1;
    if (dim == 3) {
        hipLaunchKernelGGL((knn3_kernel<K>), dim3((nq + WAVES - 1) / WAVES), dim3(256), 0, st, p1,
                           p2, b, n1, n2, dists, idx64, idx32, nn, k);
    } else {
        constexpr int QB = WAVES * QPW;
        if (b > 1 && n1 % QB) {  // a block's queries must belong to one cloud
            for (int c = 0; c < b; ++c) {
                const int rc = launch_knn<K>(p1 + (size_t)c * n1 * dim, p2 + (size_t)c * n2 * dim, 1,
                                             n1, n2, dim, k, dists ? dists + (size_t)c * n1 * k : nullptr,
                                             idx64 ? idx64 + (size_t)c * n1 * k : nullptr,
                                             idx32 ? idx32 + (size_t)c * n1 * k : nullptr,
                                             nn ? nn + (size_t)c * n1 * k * dim : nullptr, st);
                if (rc) return rc;
            }
            return HREG_OK;
        }
        hipLaunchKernelGGL((knnd_kernel<K>), dim3((nq + QB - 1) / QB), dim3(256), 0, st, p1, p2, b,
                           n1, n2, dim, dists, idx64, idx32, nn, k);
    }
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

__global__ void knn_gather_kernel(const float *__restrict__ x, const int64_t *__restrict__ idx,
                                  int n, int c, int m, int k, size_t total,
                                  float *__restrict__ out) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const size_t row = e / c;
    const int ch = (int)(e % c);
    const size_t bm = row / k;        // b*m + i
    const size_t bi = bm / m;         // batch
    const int64_t id = idx[row];
    out[e] = (id >= 0 && id < n) ? x[(bi * n + id) * c + ch] : 0.f;
}

}  // namespace

extern "C" int hreg_knn_points(const float *p1, const float *p2, int b, int n1, int n2, int dim,
                               int k, float *dists, int64_t *idx64, int32_t *idx32, float *nn,
                               void *stream) {
    if (!p1 || !p2 || b < 0 || n1 < 0 || n2 < 0 || dim <= 0 || k <= 0) return HREG_ERR_INVALID;
    if (k > 64) return HREG_ERR_UNSUPPORTED;
    if (b == 0 || n1 == 0) return HREG_OK;
    hipStream_t st = as_stream(stream);
    if (k <= 8) return launch_knn<8>(p1, p2, b, n1, n2, dim, k, dists, idx64, idx32, nn, st);
    if (k <= 16) return launch_knn<16>(p1, p2, b, n1, n2, dim, k, dists, idx64, idx32, nn, st);
    if (k <= 32) return launch_knn<32>(p1, p2, b, n1, n2, dim, k, dists, idx64, idx32, nn, st);
    return launch_knn<64>(p1, p2, b, n1, n2, dim, k, dists, idx64, idx32, nn, st);
}

extern "C" int hreg_knn_gather(const float *x, const int64_t *idx, int b, int n, int c, int m,
                               int k, float *out, void *stream) {
    if (!x || !idx || !out || b < 0 || n < 0 || c <= 0 || m < 0 || k <= 0) return HREG_ERR_INVALID;
    const size_t total = (size_t)b * m * k * c;
    if (total == 0) return HREG_OK;
    hipLaunchKernelGGL(knn_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       as_stream(stream), x, idx, n, c, m, k, total, out);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_knn_group(const float *q, const float *p, int nb, int m, int n, int k,
                              int32_t *gidx, float *geom, float *knn_xyz, void *stream) {
    if (!q || !p || !gidx || !geom || nb < 0 || m < 0 || n <= 0 || k <= 0) return HREG_ERR_INVALID;
    if (k > 64) return HREG_ERR_UNSUPPORTED;
    if (nb == 0 || m == 0) return HREG_OK;
    hipStream_t st = as_stream(stream);
    dim3 grid((nb * m + WAVES - 1) / WAVES);
#define HREG_KG(KK)                                                                       \
    hipLaunchKernelGGL((knn_group_kernel<KK>), grid, dim3(256), 0, st, q, p, nb, m, n, k, \
                       gidx, geom, knn_xyz)
    if (k <= 8) HREG_KG(8);
    else if (k <= 16) HREG_KG(16);
    else if (k <= 32) HREG_KG(32);
    else HREG_KG(64);
#undef HREG_KG
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
