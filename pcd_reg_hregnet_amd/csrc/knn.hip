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

// QW queries (of one cloud) per wave: every database point a lane loads feeds QW distances;
// each query keeps its own list, buffer and distance order (the lists of knn3_query).  The xyz
// kNNs run QW = 1: with 3 floats per point the load is not their cost (r5, bench lines 8392 /
// 8294 at QW 1 vs 8296 / 8024 at QW 4, gpurun_out/r5w); the descriptor kNN shares its rows
// (knnd_wave_kernel, KNND_QW).
template <int K, int QW>
__device__ void knn3_query_multi(const float *__restrict__ P, int n2, const float (&qx)[QW], const float (&qy)[QW],
                                 const float (&qz)[QW], uint64_t (*buf)[128], int lane, WaveList (&L)[QW]) {
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        L[t].key = KEY_INF; L[t].tau = KEY_INF; L[t].cnt = 0;
    }
    for (int base = 0; base < n2; base += 64) {
        const int p = base + lane;
        const bool ok = p < n2;
        const int pp = ok ? p : 0;
        const float px = P[pp * 3 + 0], py = P[pp * 3 + 1], pz = P[pp * 3 + 2];
#pragma unroll
        for (int t = 0; t < QW; ++t) {
            uint64_t key = KEY_INF;
            if (ok) {
                const float d = sqdist3(qx[t], qy[t], qz[t], px, py, pz);
                key = ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)p;
            }
            offer<K>(L[t], buf[t], key, lane);
        }
    }
#pragma unroll
    for (int t = 0; t < QW; ++t)
        if (L[t].cnt > 0) flush64<K>(L[t], buf[t], lane);
}

template <int K, int QW>
__global__ __launch_bounds__(256) void knn3_kernel(const float *__restrict__ q,
                                                   const float *__restrict__ p, int nb, int n1,
                                                   int n2, float *__restrict__ dists,
                                                   int64_t *__restrict__ idx64,
                                                   int32_t *__restrict__ idx32,
                                                   float *__restrict__ nn, int k) {
    __shared__ uint64_t sbuf[WAVES][QW][128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int q0 = (xcd_block(blockIdx.x, gridDim.x) * WAVES + w) * QW;
    if (q0 >= nb * n1) return;
    const int cloud = q0 / n1;
    const float *P = p + (size_t)cloud * n2 * 3;
    float qx[QW], qy[QW], qz[QW];
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        qx[t] = q[(size_t)(q0 + t) * 3]; qy[t] = q[(size_t)(q0 + t) * 3 + 1]; qz[t] = q[(size_t)(q0 + t) * 3 + 2];
    }
    WaveList L[QW];
    knn3_query_multi<K, QW>(P, n2, qx, qy, qz, sbuf[w], lane, L);
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        if (lane < k) {
            const bool valid = L[t].key != KEY_INF;
            const int id = valid ? (int)(uint32_t)(L[t].key & 0xffffffffu) : -1;
            const size_t o = (size_t)(q0 + t) * k + lane;
            if (dists) dists[o] = valid ? __uint_as_float((uint32_t)(L[t].key >> 32)) : 0.f;
            if (idx64) idx64[o] = id;
            if (idx32) idx32[o] = id;
            if (nn) {
                nn[o * 3 + 0] = valid ? P[id * 3 + 0] : 0.f;
                nn[o * 3 + 1] = valid ? P[id * 3 + 1] : 0.f;
                nn[o * 3 + 2] = valid ? P[id * 3 + 2] : 0.f;
            }
        }
    }
}

// knn_group: global neighbour rows + (p - q, |p - q|) + neighbour xyz
template <int K, int QW>
__global__ __launch_bounds__(256) void knn_group_kernel(const float *__restrict__ q,
                                                        const float *__restrict__ p, int nb, int m,
                                                        int n, int k, int32_t *__restrict__ gidx,
                                                        float *__restrict__ geom,
                                                        float *__restrict__ knn_xyz) {
    __shared__ uint64_t sbuf[WAVES][QW][128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int q0 = (xcd_block(blockIdx.x, gridDim.x) * WAVES + w) * QW;
    if (q0 >= nb * m) return;
    const int cloud = q0 / m;
    const float *P = p + (size_t)cloud * n * 3;
    float qx[QW], qy[QW], qz[QW];
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        qx[t] = q[(size_t)(q0 + t) * 3]; qy[t] = q[(size_t)(q0 + t) * 3 + 1]; qz[t] = q[(size_t)(q0 + t) * 3 + 2];
    }
    WaveList L[QW];
    knn3_query_multi<K, QW>(P, n, qx, qy, qz, sbuf[w], lane, L);
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        if (lane < k) {
            const size_t r = (size_t)(q0 + t) * k + lane;
            const bool valid = L[t].key != KEY_INF;
            const int id = valid ? (int)(uint32_t)(L[t].key & 0xffffffffu) : 0;
            const float px = P[id * 3], py = P[id * 3 + 1], pz = P[id * 3 + 2];
            const float rx = fsub_rn(px, qx[t]), ry = fsub_rn(py, qy[t]), rz = fsub_rn(pz, qz[t]);
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
    const int q0 = xcd_block(blockIdx.x, gridDim.x) * QB;  // queries of one block never straddle clouds: n1 % QB == 0
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

// Descriptor-space kNN, one wave per query, no LDS staging and no barriers (dim % 4
// == 0, 16-byte aligned rows): lane = database row of a 64-row chunk, the row read
// straight from L2 as float4s, the query's dims wave-uniform (scalar loads).  The
// CoarseReg desc kNN (layers.py:278: 256 queries x 256 rows x 256 dims per pair) as
// 16-query blocks gave one block per 16 queries -- 128 blocks at B=8, each a chain
// of 16 barrier-separated staging round trips; this is 2048 independent waves.
// Same distance order (q - p, squared, added in d order) and the same offer/merge:
// bit-identical lists.
// KNND_QW: queries per wave.  Every database row a lane loads (1 KB at 256 dims) feeds
// QW queries' distances, so the L2 -> CU row stream per query drops QW-fold; each query keeps
// its own candidate list (WaveList + LDS buffer) and its own accumulation order (bit-identical
// distances and lists).  The QW queries of a wave belong to one cloud (n1 % QW == 0, else 1).
// Measured (gpurun_out/r5r): CoarseReg's kNN over 32 pairs (256 x 256 x 256 dims) 0.274 ->
// 0.091 ms at QW = 4; bench lines at --steps 20 7990 -> 8178 pairs/s (paired, one box).
// QW = 8: 0.158 ms (more VGPRs, fewer waves).
constexpr int KNND_QW = 4;
template <int K, int QW>
__global__ __launch_bounds__(256) void knnd_wave_kernel(const float *__restrict__ q,
                                                        const float *__restrict__ p, int nb, int n1,
                                                        int n2, int dim, float *__restrict__ dists,
                                                        int64_t *__restrict__ idx64,
                                                        int32_t *__restrict__ idx32,
                                                        float *__restrict__ nn, int k) {
    __shared__ uint64_t sbuf[WAVES][QW][128];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q0 = (xcd_block(blockIdx.x, gridDim.x) * WAVES + w) * QW;
    if (q0 >= nb * n1) return;  // wave-uniform
    const int cloud = q0 / n1;
    const float *P = p + (size_t)cloud * n2 * dim;
    const float *Q = q + (size_t)q0 * dim;
    WaveList L[QW];
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        L[t].key = KEY_INF; L[t].tau = KEY_INF; L[t].cnt = 0;
    }
    for (int base = 0; base < n2; base += 64) {
        const int pi = base + lane;
        const float *pr = P + (size_t)(pi < n2 ? pi : n2 - 1) * dim;
        float acc[QW];
#pragma unroll
        for (int t = 0; t < QW; ++t) acc[t] = 0.f;
#pragma unroll 4
        for (int e = 0; e < dim; e += 4) {
            const float4 pv = *reinterpret_cast<const float4 *>(pr + e);
#pragma unroll
            for (int t = 0; t < QW; ++t) {
                const float4 qv = *reinterpret_cast<const float4 *>(Q + (size_t)t * dim + e);
                float d;
                d = fsub_rn(qv.x, pv.x); acc[t] = fadd_rn(acc[t], fmul_rn(d, d));
                d = fsub_rn(qv.y, pv.y); acc[t] = fadd_rn(acc[t], fmul_rn(d, d));
                d = fsub_rn(qv.z, pv.z); acc[t] = fadd_rn(acc[t], fmul_rn(d, d));
                d = fsub_rn(qv.w, pv.w); acc[t] = fadd_rn(acc[t], fmul_rn(d, d));
            }
        }
#pragma unroll
        for (int t = 0; t < QW; ++t) {
            const uint64_t key = pi < n2 ? (((uint64_t)__float_as_uint(acc[t]) << 32) | (uint32_t)pi) : KEY_INF;
            offer<K>(L[t], sbuf[w][t], key, lane);
        }
    }
#pragma unroll
    for (int t = 0; t < QW; ++t) {
        if (L[t].cnt > 0) flush64<K>(L[t], sbuf[w][t], lane);
        if (lane < k) {
            const bool valid = L[t].key != KEY_INF;
            const int id = valid ? (int)(uint32_t)(L[t].key & 0xffffffffu) : -1;
            const size_t o = (size_t)(q0 + t) * k + lane;
            if (dists) dists[o] = valid ? __uint_as_float((uint32_t)(L[t].key >> 32)) : 0.f;
            if (idx64) idx64[o] = id;
            if (idx32) idx32[o] = id;
            if (nn)
                for (int e = 0; e < dim; ++e) nn[o * dim + e] = valid ? P[(size_t)id * dim + e] : 0.f;
        }
    }
}

// ---- spatially indexed kNN grouping (xyz, n <= 65536) --------------------
// hreg_spatial_index orders each cloud's points by a 12-bit Morton cell (one
// workgroup per cloud, counting sort in LDS) and records the bounding box of
// every run of 64 ordered points.  A query then scans only the
// 64-point blocks whose box lower bound does not exceed its current K-th
// distance: exact, because the bound is computed with the same fp32 operation
// order as the point distances and fl() is monotone (for p in the box,
// |fl(q - p)| >= |fl(q - clamp(q, lo, hi))| per axis), and because every point
// with d <= tau is still offered, so ties order by index as in the full scan.
constexpr int SI_THREADS = 1024;
constexpr int SI_LDSN = 16384;  // clouds up to this size sort through an LDS index list
constexpr int SI_MAXN = 65536;  // larger ones (Model_V2's config 5) scatter straight to HBM

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// (NaN coordinates map to cell 0: !(t > 0) holds for NaN, so the float -> uint conversion only
// ever sees values in (0, 1023))
__device__ __forceinline__ uint32_t quant10(float x, float lo, float sc) {
    const float t = (x - lo) * sc;
    return !(t > 0.f) ? 0u : (t >= 1023.f ? 1023u : (uint32_t)t);
}

__device__ __forceinline__ float box_lb(float qx, float qy, float qz, float4 lo, float4 hi) {
    const float cx = fminf(fmaxf(qx, lo.x), hi.x);
    const float cy = fminf(fmaxf(qy, lo.y), hi.y);
    const float cz = fminf(fmaxf(qz, lo.z), hi.z);
    return sqdist3(qx, qy, qz, cx, cy, cz);
}

// Large clouds (SI_LDSN < n <= SI_MAXN, Model_V2): a counting sort by a 15-bit Morton prefix
// (32 cells per axis, 128 KB of LDS counters); inside a cell the order is the LDS atomics', so the
// cell size bounds a 64-point block's box.  On KITTI-shape 65536-point clouds (numpy model of the
// pruned FPS, fps.hip fps_blocks_kernel) 15-bit cells leave ~28 blocks to scan per FPS iteration
// against ~47 with the 12-bit cells of r1-r5 (a full 18-bit order: ~23).  The rank list does not
// fit LDS, so points are scattered to their sorted slot in HBM directly and the boxes read them
// back (this workgroup's own stores; fenced at agent scope).  The kNN and FPS results do not
// depend on the order inside a cell.
constexpr int SI_CELLS_BIG = 32768;

__global__ __launch_bounds__(SI_THREADS) void spatial_index_kernel(const float *__restrict__ p, int n,
                                                                   float4 *__restrict__ spts,
                                                                   float4 *__restrict__ boxes) {
    constexpr int CELLS = SI_CELLS_BIG;
    __shared__ uint32_t cnt[CELLS];
    __shared__ float red[6][SI_THREADS / 64];
    __shared__ uint32_t wsum[SI_THREADS / 64];
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float *P = p + (size_t)c * n * 3;
    for (int i = tid; i < CELLS; i += SI_THREADS) cnt[i] = 0;
    // cloud bounding box
    float mn[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
    float mx[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    for (int i = tid; i < n; i += SI_THREADS)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            mn[d] = fminf(mn[d], P[i * 3 + d]);
            mx[d] = fmaxf(mx[d], P[i * 3 + d]);
        }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        mn[d] = -wave_max_f32(-mn[d]);
        mx[d] = wave_max_f32(mx[d]);
        if (lane == 0) { red[d][w] = mn[d]; red[3 + d][w] = mx[d]; }
    }
    __syncthreads();
    float lo[3], sc[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float a = red[d][0], b = red[3 + d][0];
        for (int i = 1; i < SI_THREADS / 64; ++i) { a = fminf(a, red[d][i]); b = fmaxf(b, red[3 + d][i]); }
        lo[d] = a;
        sc[d] = b > a ? 1023.99f / (b - a) : 0.f;
    }
    auto cell_of = [&](int i) {
        const uint32_t code = spread10(quant10(P[i * 3], lo[0], sc[0])) |
                              (spread10(quant10(P[i * 3 + 1], lo[1], sc[1])) << 1) |
                              (spread10(quant10(P[i * 3 + 2], lo[2], sc[2])) << 2);
        return code >> 15;
    };
    for (int i = tid; i < n; i += SI_THREADS) atomicAdd(&cnt[cell_of(i)], 1u);
    __syncthreads();
    // exclusive prefix over the cells: CELLS / SI_THREADS per thread, wave scans, wave totals
    constexpr int PER = CELLS / SI_THREADS;
    uint32_t v[PER], tsum = 0;
#pragma unroll
    for (int e = 0; e < PER; ++e) { v[e] = cnt[tid * PER + e]; tsum += v[e]; }
    uint32_t incl = tsum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int i = 0; i < w; ++i) wbase += wsum[i];
    uint32_t run = wbase + incl - tsum;
#pragma unroll
    for (int e = 0; e < PER; ++e) { cnt[tid * PER + e] = run; run += v[e]; }
    __syncthreads();
    int np = 64;
    while (np < n) np <<= 1;
    float4 *S = spts + (size_t)c * np;
    for (int i = tid; i < n; i += SI_THREADS)
        S[atomicAdd(&cnt[cell_of(i)], 1u)] = make_float4(P[i * 3], P[i * 3 + 1], P[i * 3 + 2], __int_as_float(i));
    __threadfence();  // release: the scattered stores complete before the barrier
    __syncthreads();
    __threadfence();  // acquire: no stale L1 lines for the reads below
    const int nblk = (n + 63) / 64;
    float4 *B = boxes + (size_t)c * (np / 64) * 2;
    for (int b = w; b < nblk; b += SI_THREADS / 64) {
        const int i = b * 64 + lane;
        float v3[3], u3[3];
        if (i < n) {
            const float4 q = S[i];
            v3[0] = u3[0] = q.x; v3[1] = u3[1] = q.y; v3[2] = u3[2] = q.z;
        } else {
#pragma unroll
            for (int d = 0; d < 3; ++d) { v3[d] = __builtin_huge_valf(); u3[d] = -__builtin_huge_valf(); }
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) { v3[d] = -wave_max_f32(-v3[d]); u3[d] = wave_max_f32(u3[d]); }
        if (lane == 0) {
            B[b * 2] = make_float4(v3[0], v3[1], v3[2], 0.f);
            B[b * 2 + 1] = make_float4(u3[0], u3[1], u3[2], 0.f);
        }
    }
}

// Clouds of <= SI_LDSN points: the points ordered by an 18-bit Morton prefix
// (64 cells per axis; ties by index) instead of the 12-bit cell alone.  Inside a 12-bit cell
// (1/16 of the cloud's extent per axis) the counting sort leaves the points in atomic order,
// so a 64-point block spans most of its cell and a level-1 query (k = 64 of 16384 LiDAR
// points) scanned ~34 blocks; in 18-bit order ~13 (full 30-bit order ~11;
// tools/knn_block_sim.py).  The kNN result does not depend on the order (exact bounds, ties
// by index).  Sort: keys (prefix << 14 | index) packed in 32 bits, three stable LSD counting
// passes of 6-bit digits in LDS (ping-pong, 2 x 64 KB); each wave owns a contiguous range of
// the keys, so per-(digit, wave) offsets plus the in-chunk rank among lanes holding the same
// digit (6 ballots) keep every pass stable.
constexpr int SI_DIG = 6, SI_BUCKETS = 1 << SI_DIG, SI_WAVES = SI_THREADS / 64;

__global__ __launch_bounds__(SI_THREADS) void spatial_index_morton_kernel(const float *__restrict__ p, int n,
                                                                          float4 *__restrict__ spts,
                                                                          float4 *__restrict__ boxes) {
    __shared__ uint32_t keys[2][SI_LDSN];
    __shared__ uint32_t off[SI_BUCKETS][SI_WAVES];  // per-(digit, wave) running scatter offsets
    __shared__ float red[6][SI_WAVES];
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float *P = p + (size_t)c * n * 3;
    // cloud bounding box (as spatial_index_kernel)
    float mn[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
    float mx[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    for (int i = tid; i < n; i += SI_THREADS)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            mn[d] = fminf(mn[d], P[i * 3 + d]);
            mx[d] = fmaxf(mx[d], P[i * 3 + d]);
        }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        mn[d] = -wave_max_f32(-mn[d]);
        mx[d] = wave_max_f32(mx[d]);
        if (lane == 0) { red[d][w] = mn[d]; red[3 + d][w] = mx[d]; }
    }
    __syncthreads();
    float lo[3], sc[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        float a = red[d][0], b = red[3 + d][0];
        for (int i = 1; i < SI_WAVES; ++i) { a = fminf(a, red[d][i]); b = fmaxf(b, red[3 + d][i]); }
        lo[d] = a;
        sc[d] = b > a ? 1023.99f / (b - a) : 0.f;
    }
    int np = 64;
    while (np < n) np <<= 1;
    for (int e = tid; e < np; e += SI_THREADS) {
        uint32_t v = ~0u;  // padding sorts last (and stays after every real key of equal bits)
        if (e < n) {
            const uint32_t code = spread10(quant10(P[e * 3], lo[0], sc[0])) |
                                  (spread10(quant10(P[e * 3 + 1], lo[1], sc[1])) << 1) |
                                  (spread10(quant10(P[e * 3 + 2], lo[2], sc[2])) << 2);
            v = ((code >> 12) << 14) | (uint32_t)e;
        }
        keys[0][e] = v;
    }
    // wave w owns keys [w * per, (w + 1) * per), in 64-key chunks
    const int per = np / SI_WAVES >= 64 ? np / SI_WAVES : 64;
    const int e_lo = w * per, e_hi = min(np, e_lo + per);
    const uint64_t below = (1ull << lane) - 1ull;
    int src = 0;
    for (int pass = 0; pass < 3; ++pass, src ^= 1) {
        const int shift = 14 + SI_DIG * pass;
        for (int i = tid; i < SI_BUCKETS * SI_WAVES; i += SI_THREADS) (&off[0][0])[i] = 0;
        __syncthreads();
        for (int e0 = e_lo; e0 < e_hi; e0 += 64) {  // counts (lane order inside the wave's range)
            const uint32_t d = (keys[src][e0 + lane] >> shift) & (SI_BUCKETS - 1);
            atomicAdd(&off[d][w], 1u);
        }
        __syncthreads();
        if (tid < 64) {  // exclusive scan over (digit, wave) in that order: 64 digits x 16 waves
            uint32_t v[SI_WAVES], t = 0;
#pragma unroll
            for (int q = 0; q < SI_WAVES; ++q) { v[q] = off[tid][q]; t += v[q]; }
            uint32_t incl = t;
#pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t o = __shfl_up(incl, dd);
                if (lane >= dd) incl += o;
            }
            uint32_t run = incl - t;
#pragma unroll
            for (int q = 0; q < SI_WAVES; ++q) { off[tid][q] = run; run += v[q]; }
        }
        __syncthreads();
        for (int e0 = e_lo; e0 < e_hi; e0 += 64) {  // stable scatter
            const uint32_t v = keys[src][e0 + lane];
            const uint32_t d = (v >> shift) & (SI_BUCKETS - 1);
            uint64_t same = ~0ull;
#pragma unroll
            for (int b = 0; b < SI_DIG; ++b) {
                const uint64_t m = __ballot((d >> b) & 1u);
                same &= ((d >> b) & 1u) ? m : ~m;
            }
            const uint32_t base = off[d][w];
            keys[src ^ 1][base + (uint32_t)__popcll(same & below)] = v;
            wave_sync();  // every lane has read its digit's offset
            if ((same & below) == 0) off[d][w] = base + (uint32_t)__popcll(same);
            wave_sync();
        }
        __syncthreads();
    }
    const uint32_t *K = keys[src];
    float4 *S = spts + (size_t)c * np;
    for (int i = tid; i < n; i += SI_THREADS) {
        const int id = (int)(K[i] & 0x3fffu);
        S[i] = make_float4(P[id * 3], P[id * 3 + 1], P[id * 3 + 2], __int_as_float(id));
    }
    const int nblk = (n + 63) / 64;
    float4 *B = boxes + (size_t)c * (np / 64) * 2;
    for (int b = w; b < nblk; b += SI_WAVES) {
        const int i = b * 64 + lane;
        float v3[3], u3[3];
        if (i < n) {
            const int id = (int)(K[i] & 0x3fffu);
#pragma unroll
            for (int d = 0; d < 3; ++d) v3[d] = u3[d] = P[id * 3 + d];
        } else {
#pragma unroll
            for (int d = 0; d < 3; ++d) { v3[d] = __builtin_huge_valf(); u3[d] = -__builtin_huge_valf(); }
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) { v3[d] = -wave_max_f32(-v3[d]); u3[d] = wave_max_f32(u3[d]); }
        if (lane == 0) {
            B[b * 2] = make_float4(v3[0], v3[1], v3[2], 0.f);
            B[b * 2 + 1] = make_float4(u3[0], u3[1], u3[2], 0.f);
        }
    }
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    // DPP row minima, then the four row results
    v = min(v, (uint32_t)dpp_all_i<0xb1>((int)v));
    v = min(v, (uint32_t)dpp_all_i<0x4e>((int)v));
    v = min(v, (uint32_t)dpp_all_i<0x141>((int)v));
    v = min(v, (uint32_t)dpp_all_i<0x140>((int)v));
    const uint32_t a = min((uint32_t)__builtin_amdgcn_readlane((int)v, 0),
                           (uint32_t)__builtin_amdgcn_readlane((int)v, 16));
    const uint32_t c = min((uint32_t)__builtin_amdgcn_readlane((int)v, 32),
                           (uint32_t)__builtin_amdgcn_readlane((int)v, 48));
    return min(a, c);
}

// NBL point blocks of 64 per lane: 4 for n <= 16384, 16 for n <= 65536
template <int K, int NBL>
__global__ __launch_bounds__(256) void knn_group_indexed_kernel(
    const float *__restrict__ q, const float *__restrict__ p, const float4 *__restrict__ spts,
    const float4 *__restrict__ boxes, int nb, int m, int n, int k, int32_t *__restrict__ gidx,
    float *__restrict__ geom, float *__restrict__ knn_xyz) {
    constexpr int IDB = NBL * 64 <= 256 ? 8 : 10;  // low key bits carrying the block id
    constexpr uint32_t HI = ~((1u << IDB) - 1u);
    __shared__ uint64_t sbuf[WAVES][128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qi = xcd_block(blockIdx.x, gridDim.x) * WAVES + w;
    if (qi >= nb * m) return;
    const int cloud = qi / m;
    int np = 64;
    while (np < n) np <<= 1;
    const int nblk = (n + 63) / 64;
    const float4 *S = spts + (size_t)cloud * np;
    const float4 *B = boxes + (size_t)cloud * (np / 64) * 2;
    const float *P = p + (size_t)cloud * n * 3;
    const float qx = q[(size_t)qi * 3], qy = q[(size_t)qi * 3 + 1], qz = q[(size_t)qi * 3 + 2];

    // lower bounds of this lane's blocks (bit patterns: lb >= 0 orders as uint32)
    uint32_t lb[NBL];
#pragma unroll
    for (int t = 0; t < NBL; ++t) {
        const int b = t * 64 + lane;
        lb[t] = b < nblk ? __float_as_uint(box_lb(qx, qy, qz, B[b * 2], B[b * 2 + 1])) : 0xffffffffu;
    }

    WaveList L;
    L.key = KEY_INF; L.tau = KEY_INF; L.cnt = 0;
    // best-first: visit blocks in increasing lower bound until the smallest remaining
    // bound exceeds the K-th distance so far.  The visiting order only needs to be
    // approximate (bound bits truncated to make room for the block id), the stop
    // test is exact: stop when even the truncated bound exceeds tau; a block whose
    // exact bound exceeds tau is skipped, not visited.
    // the next block by (truncated) lower bound, removed from the candidates; returns the
    // block (or -1 when none is left or even the truncated bound exceeds tau_bits) and its
    // exact bound
    auto next_block = [&](uint32_t tau_bits, uint32_t &lbb) -> int {
        uint32_t kmin = 0xffffffffu;
#pragma unroll
        for (int t = 0; t < NBL; ++t) {
            const uint32_t kk = lb[t] == 0xffffffffu ? 0xffffffffu
                                                     : ((lb[t] & HI) | (uint32_t)(t * 64 + lane));
            kmin = kk < kmin ? kk : kmin;
        }
        kmin = wave_min_u32(kmin);
        if (kmin == 0xffffffffu || (kmin & HI) > tau_bits) return -1;
        const int b = (int)(kmin & ~HI);
        lbb = __builtin_amdgcn_readlane(lb[b >> 6], b & 63);
#pragma unroll
        for (int t = 0; t < NBL; ++t)
            if ((b >> 6) == t && lane == (b & 63)) lb[t] = 0xffffffffu;
        return b;
    };
    auto block_key = [&](const float4 v, int i) -> uint64_t {
        if (i >= n) return KEY_INF;
        const float d = sqdist3(qx, qy, qz, v.x, v.y, v.z);
        return ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)__float_as_int(v.w);
    };
    for (;;) {
        const uint32_t tau_bits = (uint32_t)(L.tau >> 32);  // >= 0x7f800000 while unset
        uint32_t lbb = 0;
        const int b = next_block(tau_bits, lbb);
        if (b < 0) break;
        // (r4: the next best blocks loaded in the same round trip, 2 or 4 per step, measured
        // neutral and removed)
        if (lbb > tau_bits) continue;
        const int i = b * 64 + lane;
        const float4 v = i < n ? S[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        offer<K>(L, sbuf[w], block_key(v, i), lane);
        if (L.tau == KEY_INF && L.cnt > 0) flush64<K>(L, sbuf[w], lane);  // first tau early
    }
    if (L.cnt > 0) flush64<K>(L, sbuf[w], lane);

    if (lane < k) {
        const size_t r = (size_t)qi * k + lane;
        const bool valid = L.key != KEY_INF;
        const int id = valid ? (int)(uint32_t)(L.key & 0xffffffffu) : 0;
        const float px = P[id * 3], py = P[id * 3 + 1], pz = P[id * 3 + 2];
        const float rx = fsub_rn(px, qx), ry = fsub_rn(py, qy), rz = fsub_rn(pz, qz);
        const float d2 = fadd_rn(fadd_rn(fmul_rn(rx, rx), fmul_rn(ry, ry)), fmul_rn(rz, rz));
        gidx[r] = cloud * n + id;
        *reinterpret_cast<float4 *>(geom + r * 4) = make_float4(rx, ry, rz, sqrtf(d2));
        if (knn_xyz) {
            knn_xyz[r * 3 + 0] = px;
            knn_xyz[r * 3 + 1] = py;
            knn_xyz[r * 3 + 2] = pz;
        }
    }
}


template <int K>
int launch_knn(const float *p1, const float *p2, int b, int n1, int n2, int dim, int k,
               float *dists, int64_t *idx64, int32_t *idx32, float *nn, hipStream_t st) {
    const int nq = b * n1;
    if (dim == 3) {
        hipLaunchKernelGGL((knn3_kernel<K, 1>), dim3((nq + WAVES - 1) / WAVES), dim3(256), 0, st, p1, p2, b,
                           n1, n2, dists, idx64, idx32, nn, k);
    } else if (dim % 4 == 0 && !((reinterpret_cast<uintptr_t>(p1) | reinterpret_cast<uintptr_t>(p2)) & 15)) {
        if (n1 % KNND_QW == 0) {
            constexpr int QW = KNND_QW;
            hipLaunchKernelGGL((knnd_wave_kernel<K, QW>), dim3((nq / QW + WAVES - 1) / WAVES), dim3(256), 0, st,
                               p1, p2, b, n1, n2, dim, dists, idx64, idx32, nn, k);
        } else {
            hipLaunchKernelGGL((knnd_wave_kernel<K, 1>), dim3((nq + WAVES - 1) / WAVES), dim3(256), 0, st, p1,
                               p2, b, n1, n2, dim, dists, idx64, idx32, nn, k);
        }
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

static size_t spatial_index_np(int n) {
    size_t np = 64;
    while (np < (size_t)n) np <<= 1;
    return np;
}

extern "C" size_t hreg_spatial_index_bytes(int nb, int n) {
    if (nb <= 0 || n <= 0 || n > SI_MAXN) return 0;
    const size_t np = spatial_index_np(n);
    return (size_t)nb * (np * sizeof(float4) + (np / 64) * 2 * sizeof(float4));
}

extern "C" int hreg_spatial_index(const float *p, int nb, int n, void *ws, void *stream) {
    if (!p || !ws || nb < 0 || n <= 0) return HREG_ERR_INVALID;
    if (n > SI_MAXN) return HREG_ERR_UNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(ws) & 15)) return HREG_ERR_INVALID;
    if (nb == 0) return HREG_OK;
    const size_t np = spatial_index_np(n);
    float4 *spts = static_cast<float4 *>(ws);
    float4 *boxes = spts + (size_t)nb * np;
    if (n > SI_LDSN)
        hipLaunchKernelGGL(spatial_index_kernel, dim3(nb), dim3(SI_THREADS), 0, as_stream(stream), p, n, spts,
                           boxes);
    else
        hipLaunchKernelGGL(spatial_index_morton_kernel, dim3(nb), dim3(SI_THREADS), 0, as_stream(stream), p, n,
                           spts, boxes);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_knn_group_indexed(const float *q, const float *p, const void *ws, int nb, int m,
                                      int n, int k, int32_t *gidx, float *geom, float *knn_xyz,
                                      void *stream) {
    if (!q || !p || !ws || !gidx || !geom || nb < 0 || m < 0 || n <= 0 || k <= 0)
        return HREG_ERR_INVALID;
    if (k > 64 || n > SI_MAXN) return HREG_ERR_UNSUPPORTED;
    if (nb == 0 || m == 0) return HREG_OK;
    const size_t np = spatial_index_np(n);
    const float4 *spts = static_cast<const float4 *>(ws);
    const float4 *boxes = spts + (size_t)nb * np;
    hipStream_t st = as_stream(stream);
    dim3 grid((nb * m + WAVES - 1) / WAVES);
#define KGI_CASE(KK)                                                                              \
    if (n > SI_LDSN)                                                                              \
        hipLaunchKernelGGL((knn_group_indexed_kernel<KK, SI_MAXN / 4096>), grid, dim3(256), 0, st, q, \
                           p, spts, boxes, nb, m, n, k, gidx, geom, knn_xyz);                      \
    else                                                                                          \
        hipLaunchKernelGGL((knn_group_indexed_kernel<KK, SI_LDSN / 4096>), grid, dim3(256), 0, st, q, \
                           p, spts, boxes, nb, m, n, k, gidx, geom, knn_xyz)
    if (k <= 8) { KGI_CASE(8); }
    else if (k <= 16) { KGI_CASE(16); }
    else if (k <= 32) { KGI_CASE(32); }
    else { KGI_CASE(64); }
#undef KGI_CASE
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
#define KG_CASE(KK) \
    hipLaunchKernelGGL((knn_group_kernel<KK, 1>), grid, dim3(256), 0, st, q, p, nb, m, n, k, gidx, geom, knn_xyz)
    if (k <= 8) KG_CASE(8);
    else if (k <= 16) KG_CASE(16);
    else if (k <= 32) KG_CASE(32);
    else KG_CASE(64);
#undef KG_CASE
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
