// mlp_head.hip -- the per-keypoint MLP heads as one launch each.
//
// KeypointDetector (layers.py:124-132, 161-163), CoarseReg (layers.py:262-268,
// 389-394) and FineReg (layers.py:425-431, 451-452) end in the same head over a
// per-keypoint feature row x [C]:
//   y1 = ReLU(BN(W1 x))  (mlp1: Conv1d C->C + BN + ReLU)
//   y2 = ReLU(BN(W2 y1)) (mlp2)
//   z  = w3 . y2 + b3    (mlp3: Conv1d C->1)
//   out = softplus(z) + 0.001 (sigma) or sigmoid(z) (correspondence weight)
// The layer-by-layer path runs this as two GEMM launches + hreg_head_out; with
// only 2k-16k rows per launch those GEMMs are latency-bound (~20 TF).  Here one
// workgroup owns a 32-row tile: the rows are staged into LDS, CW waves split each
// layer's output channels (P <= 2 tiles of 32 per wave, split_chain.h), y1 goes
// back through the same LDS buffer, y2 stays in registers and the mlp3 dot is
// reduced lane half -> waves in a fixed order.  hreg_mlp_head6: the same with bf16x6
// products (fp32-accurate, bf16 matrix cores).  BN is folded (eval) into the
// per-channel alpha/beta epilogue, as everywhere else (engine._bn_fold).
#include "split_chain.h"

namespace {

using namespace hreg_chain;
using namespace hreg_split;

// Table: [mlp1 fragments][mlp2 fragments] (engine.mlp_head_table: frag_layer order,
// 4 k-steps innermost per lane), then alpha1, beta1, alpha2, beta2 (C each), w3 (C),
// b3 (1) padded to 4.
template <int C_, int CW_, int RT_, int WMAX_ = SWIN>
struct HCfg {
    static constexpr int C = C_, CW = CW_, RT = RT_, WMAX = WMAX_;
    static constexpr int T = C / 32, P = T / CW, NS = T * 16;
    static_assert(P * CW == T && P >= 1 && P <= 2, "channel split");
    static constexpr int F_M1 = 0, F_M2 = T * NS * 64, F_END = 2 * F_M2;
    // epilogue section (offsets from its start): alpha1, beta1, alpha2, beta2, w3, b3 (+3)
    static constexpr int R_M1 = 0, R_M2 = 2 * C, R_W3 = 4 * C, R_B3 = 5 * C, NE = 5 * C + 4;
    static constexpr int E_M1 = F_END + R_M1, E_M2 = F_END + R_M2, E_W3 = F_END + R_W3, E_B3 = F_END + R_B3;
    static constexpr int TABLE = F_END + NE;
    // bf16x6 table (engine.mlp_head_table6): mlp1, mlp2 as bf16 piece chunk fragments
    // [tile][chunk] (units of 3 pieces x 64 lanes x 16 B), then the same epilogue section
    static constexpr int NCH = 2 * T, G_M1 = 0, G_M2 = T * NCH;
    static constexpr int F_END6 = 2 * T * NCH * 3 * 64 * 4, TABLE6 = F_END6 + NE;
    static constexpr int LDSW = C + 4;
    static constexpr int THREADS = CW * RT * 64;
};

using H64 = HCfg<64, 2, 2>;
using H128 = HCfg<128, 4, 1>;
using H256 = HCfg<256, 4, 1>;
using H512 = HCfg<512, 8, 1, 8>;  // 2 waves per SIMD: 128 VGPRs + AGPRs, short windows

// B6: the two layers on the bf16 matrix cores at fp32 accuracy (bf16x6, split_chain.h
// pipe_lds6: each wave splits the B chunks it reads from LDS into bf16 pieces)
template <class K, bool B6>
__global__ __launch_bounds__(K::THREADS) void mlp_head_kernel(const float *__restrict__ table,
                                                              const float *__restrict__ x, int ldx,
                                                              int G, int mode, float *__restrict__ out) {
    constexpr int C = K::C, P = K::P, CW = K::CW, RT = K::RT, LDSW = K::LDSW, NS = K::NS;
    constexpr int NE = K::NE, WIN = NS < K::WMAX ? NS : K::WMAX;
    constexpr int FE = B6 ? K::F_END6 : K::F_END;
    __shared__ float ep[NE];
    __shared__ __attribute__((aligned(16))) float sA[RT][32 * LDSW];
    __shared__ float sPart[RT][CW][32];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[FE + i];
    const float *eb = ep;
    // the wave index is uniform: in SGPRs, every fragment address is an SGPR base plus
    // the lane's offset (not a hoisted per-load 64-bit VGPR address)
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rt = w / CW, cw = w % CW;
    const int h = lane >> 5, j = lane & 31;
    const int NT = G / 32;
    float *A = sA[rt];
    const int c0 = cw * P;
    const FragSeq f1{K::F_M1 / 64 + c0 * NS, NS}, f2{K::F_M2 / 64 + c0 * NS, NS};
    const FragSeq g1{K::G_M1 + c0 * K::NCH, K::NCH}, g2{K::G_M2 + c0 * K::NCH, K::NCH};

    float carry[SCARRY];
    Carry6 carry6;
    if constexpr (B6) {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int i = 0; i < P; ++i) ld6(wt, g1.base + i * g1.stride, lane, carry6[i]);
    } else {
        const gfloat *tb = reinterpret_cast<const gfloat *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int s0 = 0; s0 < WIN; s0 += 4)
#pragma unroll
            for (int i = 0; i < P; ++i) {
                float v[4];
                ldgroup<4>(tb, f1.base + i * f1.stride + s0, lane, v);
#pragma unroll
                for (int q = 0; q < 4; ++q) carry[(s0 + q) * P + i] = v[q];
            }
    }
    for (int base = blockIdx.x * RT; base < NT; base += gridDim.x * RT) {
        // every wave runs the same trip count (barriers): a row tile past the end
        // recomputes the last tile (identical values, identical stores)
        const int t = min(base + rt, NT - 1);
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gfloat *tb = reinterpret_cast<const gfloat *>(tba);
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
        float ca[SCARRY];
        Carry6 ca6;

        tile_sync();  // the previous tile's readers of A are done (and ep is loaded)
        constexpr int F4 = C / 4;
#pragma unroll
        for (int i = cw * 64 + lane; i < 32 * F4; i += CW * 64) {
            const int r = i / F4, c4 = i - r * F4;
            *reinterpret_cast<float4 *>(A + r * LDSW + c4 * 4) =
                *reinterpret_cast<const float4 *>(x + ((size_t)t * 32 + r) * ldx + c4 * 4);
        }
        tile_sync();

        f32x16 y1[P];
        if constexpr (B6)
            beta_p<P, C>(eb + K::R_M1, c0, h, y1);  // folded BN (engine._fold_bn)
        else
            zero_tiles(y1);
        if constexpr (B6)
{ pipe_lds6<K::NCH, P, P>(wt, lane, g1, ChanB{A + j * LDSW, h}, y1, carry6, g2, ca6); }
        else
            pipe_lds<NS, P, P, WIN, WIN>(tb, lane, f1, ChanB{A + j * LDSW, h}, y1, carry, f2, ca);
        if constexpr (B6)
            relu_tiles(y1);
        else
            epi<P, C>(eb + K::R_M1, c0, h, y1);
        tile_sync();  // every wave has read x from A
#pragma unroll
        for (int i = 0; i < P; ++i) put_tile<LDSW>(A, c0 + i, j, h, y1[i]);
        tile_sync();

        f32x16 y2[P];
        if constexpr (B6)
            beta_p<P, C>(eb + K::R_M2, c0, h, y2);
        else
            zero_tiles(y2);
        if constexpr (B6)
{ pipe_lds6<K::NCH, P, P>(wt, lane, g2, ChanB{A + j * LDSW, h}, y2, ca6, g1, carry6); }
        else
            pipe_lds<NS, P, P, WIN, WIN>(tb, lane, f2, ChanB{A + j * LDSW, h}, y2, ca, f1, carry);
        if constexpr (B6)
            relu_tiles(y2);
        else
            epi<P, C>(eb + K::R_M2, c0, h, y2);

        // mlp3: this wave's channels, then the two lane halves, then the waves in order
        float p = 0.f;
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) p = fadd_rn(p, fmul_rn(y2[i][q], eb[K::R_W3 + chan(c0 + i, q, h)]));
        p = fadd_rn(p, __shfl_xor(p, 32));  // commutative: both halves hold the same bits
        if (h == 0) sPart[rt][cw][j] = p;
        tile_sync();
        if (cw == 0 && h == 0) {
            float z = sPart[rt][0][j];
#pragma unroll
            for (int c = 1; c < CW; ++c) z = fadd_rn(z, sPart[rt][c][j]);
            z = fadd_rn(z, eb[K::R_B3]);
            float o;
            if (mode == HREG_HEAD_SOFTPLUS) {
                const float sp = z > 20.f ? z : log1pf(expf(z));
                o = fadd_rn(sp, 0.001f);
            } else {
                o = 1.0f / fadd_rn(1.0f, expf(-z));
            }
            out[(size_t)t * 32 + j] = o;
        }
    }
}

// bf16x6 heads: one workgroup of CW waves owns JT row tiles at once and every
// wave multiplies each chunk of weight pieces it streams from L2 into all JT row tiles
// (split_chain.h pipe_lds6_jt), so a head moves JT x fewer weight bytes per MFMA -- the
// pieces of a C = 512 head are 3 MB per pass, and that stream, not the matrix cores, set
// the kernel's CU time.  Per row the arithmetic is the JT = 1 kernel's, in the same order,
// whatever row tiles share a workgroup (test_gpu_model.py: a pair alone and inside a batch,
// ragged row-tile counts).  CU time -16 %, bench +1 % (r4).

template <int C> struct HeadJT { static constexpr int v = C >= 256 ? 2 : 4; };

template <class K, int JT>
__global__ __launch_bounds__(K::CW * 64) void mlp_head6_jt_kernel(const float *__restrict__ table,
                                                                   const float *__restrict__ x, int ldx,
                                                                   int G, int mode, float *__restrict__ out) {
    constexpr int C = K::C, P = K::P, CW = K::CW, LDSW = K::LDSW, NE = K::NE, NCH = K::NCH;
    __shared__ float ep[NE];
    __shared__ __attribute__((aligned(16))) float sA[JT * 32 * LDSW];
    __shared__ float sPart[CW][JT][32];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END6 + i];
    const float *eb = ep;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G / 32;
    const int c0 = w * P;
    const FragSeq g1{K::G_M1 + c0 * NCH, NCH}, g2{K::G_M2 + c0 * NCH, NCH};
    const ChanBJ<LDSW> xb{sA + j * LDSW, h};

    Carry6 carry6;
    {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int i = 0; i < P; ++i) ld6(wt, g1.base + i * g1.stride, lane, carry6[i]);
    }
    for (int base = blockIdx.x * JT; base < NT; base += gridDim.x * JT) {
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
        Carry6 ca6;

        tile_sync();  // the previous group's readers of sA are done (and ep is loaded)
        // row tiles past the end restage the last tile (their outputs are not stored)
        constexpr int F4 = C / 4;
#pragma unroll
        for (int i = threadIdx.x; i < JT * 32 * F4; i += CW * 64) {
            const int r = i / F4, c4 = i - r * F4;
            const int t = min(base + (r >> 5), NT - 1);
            *reinterpret_cast<float4 *>(sA + r * LDSW + c4 * 4) =
                *reinterpret_cast<const float4 *>(x + ((size_t)t * 32 + (r & 31)) * ldx + c4 * 4);
        }
        tile_sync();

        f32x16 y[P][JT];
        {
            f32x16 b[P];
            beta_p<P, C>(eb + K::R_M1, c0, h, b);  // folded BN (engine._fold_bn)
#pragma unroll
            for (int i = 0; i < P; ++i)
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) y[i][jt] = b[i];
        }
        pipe_lds6_jt<NCH, P, P, JT, false>(wt, lane, g1, xb, y, carry6, g2, ca6);
#pragma unroll
        for (int i = 0; i < P; ++i) relu_tiles(y[i]);
        tile_sync();  // every wave has read x from sA
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) put_tile<LDSW>(sA + jt * 32 * LDSW, c0 + i, j, h, y[i][jt]);
        tile_sync();

        {
            f32x16 b[P];
            beta_p<P, C>(eb + K::R_M2, c0, h, b);
#pragma unroll
            for (int i = 0; i < P; ++i)
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) y[i][jt] = b[i];
        }
        pipe_lds6_jt<NCH, P, P, JT, false>(wt, lane, g2, xb, y, ca6, g1, carry6);
#pragma unroll
        for (int i = 0; i < P; ++i) relu_tiles(y[i]);

        // mlp3 as in mlp_head_kernel, per row tile
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            float p = 0.f;
#pragma unroll
            for (int i = 0; i < P; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    p = fadd_rn(p, fmul_rn(y[i][jt][q], eb[K::R_W3 + chan(c0 + i, q, h)]));
            p = fadd_rn(p, __shfl_xor(p, 32));
            if (h == 0) sPart[w][jt][j] = p;
        }
        tile_sync();
        if (threadIdx.x < JT * 32) {
            const int jt = threadIdx.x >> 5, r = threadIdx.x & 31, t = base + jt;
            float z = sPart[0][jt][r];
#pragma unroll
            for (int c = 1; c < CW; ++c) z = fadd_rn(z, sPart[c][jt][r]);
            z = fadd_rn(z, eb[K::R_B3]);
            float o;
            if (mode == HREG_HEAD_SOFTPLUS) {
                const float sp = z > 20.f ? z : log1pf(expf(z));
                o = fadd_rn(sp, 0.001f);
            } else {
                o = 1.0f / fadd_rn(1.0f, expf(-z));
            }
            if (t < NT) out[(size_t)t * 32 + r] = o;
        }
    }
}

// row_tiles (bf16x6 heads): 0 = HeadJT's tiles per workgroup (the weight pieces of a chunk feed
// 2-4 row tiles: fewer weight bytes per MFMA, for launches that share the chip); 1 = one row tile
// per workgroup, 2-4x the workgroups, for a forward alone on the GPU, where a batch-8 head is
// 32-128 workgroups on 256 CUs (engine.chain_fork).  Each row's sums are the same either way.
template <class K, bool B6>
int launch_head(const float *table, const float *x, int ldx, int G, int mode, float *out, void *stream,
                int row_tiles = 0) {
    const int NT = G / 32;
    if (B6 && (reinterpret_cast<uintptr_t>(table) & 15)) return HREG_ERR_INVALID;
    if constexpr (B6) {
        constexpr int JT = HeadJT<K::C>::v;
        const int jt = row_tiles == 1 ? 1 : JT;
        int grid = (NT + jt - 1) / jt;
        if (grid > 2048) grid = 2048;
        if (jt == 1)
            hipLaunchKernelGGL((mlp_head6_jt_kernel<K, 1>), dim3(grid), dim3(K::CW * 64), 0, as_stream(stream),
                               table, x, ldx, G, mode, out);
        else
            hipLaunchKernelGGL((mlp_head6_jt_kernel<K, JT>), dim3(grid), dim3(K::CW * 64), 0, as_stream(stream),
                               table, x, ldx, G, mode, out);
    } else {
        int grid = (NT + K::RT - 1) / K::RT;
        if (grid > 2048) grid = 2048;
        hipLaunchKernelGGL((mlp_head_kernel<K, B6>), dim3(grid), dim3(K::THREADS), 0, as_stream(stream), table,
                           x, ldx, G, mode, out);
    }
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_mlp_head_table_floats(int C) {
    switch (C) {
        case 64: return H64::TABLE;
        case 128: return H128::TABLE;
        case 256: return H256::TABLE;
        case 512: return H512::TABLE;
        default: return -1;
    }
}

extern "C" int hreg_mlp_head6_table_floats(int C) {
    switch (C) {
        case 64: return H64::TABLE6;
        case 128: return H128::TABLE6;
        case 256: return H256::TABLE6;
        case 512: return H512::TABLE6;
        default: return -1;
    }
}

template <bool B6>
static int mlp_head_entry(const float *table, int C, const float *x, int ldx, int nclouds, int rows_per_cloud,
                          int mode, float *out, float *weights_out, void *stream, int row_tiles = 0) {
    if (!table || !x || !out || nclouds < 0 || rows_per_cloud <= 0 || ldx < C || (ldx & 3) ||
        (mode != HREG_HEAD_SOFTPLUS && mode != HREG_HEAD_SIGMOID) || row_tiles < 0 || row_tiles > 1)
        return HREG_ERR_INVALID;
    if (reinterpret_cast<uintptr_t>(x) & 15) return HREG_ERR_INVALID;
    const int G = nclouds * rows_per_cloud;
    if (G % 32) return HREG_ERR_UNSUPPORTED;  // whole 32-row tiles
    if (hreg_mlp_head_table_floats(C) < 0) return HREG_ERR_UNSUPPORTED;
    if (!G) return HREG_OK;
    int rc;
    switch (C) {
        case 64: rc = launch_head<H64, B6>(table, x, ldx, G, mode, out, stream, row_tiles); break;
        case 128: rc = launch_head<H128, B6>(table, x, ldx, G, mode, out, stream, row_tiles); break;
        case 256: rc = launch_head<H256, B6>(table, x, ldx, G, mode, out, stream, row_tiles); break;
        default: rc = launch_head<H512, B6>(table, x, ldx, G, mode, out, stream, row_tiles); break;
    }
    if (rc != HREG_OK || !weights_out) return rc;
    return hreg_sigma_weights(out, nclouds, rows_per_cloud, weights_out, stream);
}

extern "C" int hreg_mlp_head(const float *table, int C, const float *x, int ldx, int nclouds,
                             int rows_per_cloud, int mode, float *out, float *weights_out, void *stream) {
    return mlp_head_entry<false>(table, C, x, ldx, nclouds, rows_per_cloud, mode, out, weights_out, stream);
}

extern "C" int hreg_mlp_head6(const float *table, int C, const float *x, int ldx, int nclouds,
                              int rows_per_cloud, int mode, float *out, float *weights_out, void *stream) {
    return mlp_head_entry<true>(table, C, x, ldx, nclouds, rows_per_cloud, mode, out, weights_out, stream);
}

extern "C" int hreg_mlp_head6x(const float *table, int C, const float *x, int ldx, int nclouds,
                               int rows_per_cloud, int mode, float *out, float *weights_out, int row_tiles,
                               void *stream) {
    return mlp_head_entry<true>(table, C, x, ldx, nclouds, rows_per_cloud, mode, out, weights_out, stream,
                                row_tiles);
}
