// group_split6.hip -- the channel-split level-2 / level-3 keypoint detector + descriptor
// of group_split.hip (same layers, same decomposition and LDS hand-offs, 11 workgroup
// barriers per 32-row tile; layers.py:115-121, 150-159, 183-208) with the products on
// the bf16 matrix cores at fp32 accuracy (bf16x6, mfma_chain.h / split_chain.h
// pipe_lds6): each 16-deep k-chunk is 6 v_mfma_f32_32x32x16_bf16 per output tile
// instead of 8 v_mfma_f32_32x32x2_f32.  The activations stay f32 in LDS (the buffers of
// group_split.hip, two workgroups per CU); each wave splits the B chunk it reads into its
// bf16 pieces in registers.  Weight pieces stream from the L2-resident table
// (engine.split_table6: group_fused6.hip's chunk fragments, then mlp1's x2 block f32
// row-major for the per-group matrix-vector product, then the f32 epilogues).  BN is
// folded (engine._fold_bn): alpha in the weights, the accumulators start from beta, the
// epilogue is the ReLU.
#include "split_chain.h"

namespace {

using namespace hreg_chain;
using namespace hreg_split;

template <int KN_, int CF_, int C1, int C3, int CM1, int CM2, int RT_, int CW_>
struct SCfg6 {
    static constexpr int KN = KN_, CF = CF_, RT = RT_, CW = CW_;
    static constexpr int TF = CF / 2, NF = TF / 8;
    static constexpr int T1 = C1 / 32, T3 = C3 / 32, TM1 = CM1 / 32, TM2 = CM2 / 32;
    static constexpr int P1 = T1 / CW, P3 = T3 / CW, PM1 = TM1 / CW, PM2 = TM2 / CW;
    static_assert(P1 * CW == T1 && P3 * CW == T3 && PM1 * CW == TM1 && PM2 * CW == TM2, "split");
    static_assert(RT * CW == 4, "4 waves");
    static constexpr int N1 = 2 * T1, N3 = 2 * T3, NM1 = 2 * TM1;  // chunks over C1 / C3 / CM1 inputs
    // chunk-fragment blocks (units of 3 pieces x 64 lanes x 16 B): group_fused6.hip Cfg6
    static constexpr int G_DG = 0, G_DF = G_DG + T1, G_D2 = G_DF + T1 * NF, G_D3 = G_D2 + T1 * N1;
    static constexpr int G_EG = G_D3 + T3 * N1, G_EF = G_EG + T1, G_E2 = G_EF + T1 * NF, G_E3 = G_E2 + T1 * N1;
    static constexpr int G_M1 = G_E3 + T3 * N1, G_M2 = G_M1 + TM1 * 3 * N3, G_END = G_M2 + TM2 * NM1;
    static constexpr int F_X2 = G_END * 3 * 64 * 4;  // floats: mlp1 x2 block [CM1][C3]
    static constexpr int F_END = F_X2 + CM1 * C3;
    static constexpr int E_D1 = F_END, E_D2 = E_D1 + 2 * C1, E_D3 = E_D2 + 2 * C1,
                         E_E1 = E_D3 + 2 * C3, E_E2 = E_E1 + 2 * C1, E_E3 = E_E2 + 2 * C1,
                         E_M1 = E_E3 + 2 * C3, E_M2 = E_M1 + 2 * CM1, TABLE = E_M2 + 2 * CM2;
    static constexpr int W0 = C3 > 4 + CF ? C3 : 4 + CF;
    static constexpr int LDSW = (W0 > CM1 ? W0 : CM1) + 4;
    static constexpr int GPT = 32 / KN;
    static constexpr int X2W = C3 + 4;
};

using S2x6 = SCfg6<32, 64, 64, 128, 64, 128, 2, 2>;
using S3x6 = SCfg6<16, 128, 128, 256, 128, 256, 1, 4>;

// stage [geom 4 | feats[gidx[row]] CF] of the tile's 32 rows into buf (group_split.hip)
template <class K, bool PRE>
__device__ __forceinline__ void stage_rows6(float *buf, const float *__restrict__ geom,
                                            const int32_t *__restrict__ gidx, const float *__restrict__ feats,
                                            int t, int cw, int lane) {
    constexpr int F4 = PRE ? 1 : 1 + K::CF / 4;
#pragma unroll
    for (int i = cw * 64 + lane; i < 32 * F4; i += K::CW * 64) {
        const int r = i / F4, c4 = i - r * F4;
        const size_t row = (size_t)t * 32 + r;
        const float *src = c4 == 0 ? geom + row * 4 : feats + (size_t)gidx[row] * K::CF + (c4 - 1) * 4;
        *reinterpret_cast<float4 *>(buf + r * K::LDSW + c4 * 4) = *reinterpret_cast<const float4 *>(src);
    }
}

// conv stack [geom | feat] -> C1 -> C1 -> C3 through the A/B buffers (group_split.hip
// conv_stack_split); this wave's P3 output tiles in out (epilogue applied).
template <class K, int NP, bool PRE, bool ONE, class WT>
__device__ __forceinline__ void conv_stack_split6(WT &&wt, const float *eb, int gg, int gf,
                                                  int g2, int g3, int e1, int e2, int e3, float *A, float *B,
                                                  int cw, int lane, f32x16 (&out)[K::P3], const Carry6 &cin,
                                                  FragSeq next, Carry6 &cout, const float *pre_row, float2 gin) {
    constexpr int TF = K::TF, P1 = K::P1, P3 = K::P3, LDSW = K::LDSW, N1 = K::N1, NF = K::NF;
    const int h = lane >> 5, j = lane & 31;
    const int c1 = cw * P1, c3 = cw * P3;
    const FragSeq sg{gg + c1, 1}, sf{gf + c1 * NF, NF}, s2{g2 + c1 * N1, N1}, s3{g3 + c3 * N1, N1};
    const float *arow = A + j * LDSW, *brow = B + j * LDSW;
    Carry6 ca, cb;
    f32x16 h1[P1];
    // geometry chunk: f32 k-steps 0, 1 (channels 2h, 2h + 1), the rest zero
    auto geom_b = [&](int st0, float (&v)[4]) {
        if (st0 == 0) {
            const float2 t = ONE ? gin : *reinterpret_cast<const float2 *>(arow + 2 * h);
            v[0] = t.x; v[1] = t.y;
        } else {
            v[0] = 0.f; v[1] = 0.f;
        }
        v[2] = 0.f; v[3] = 0.f;
    };
    if constexpr (PRE) {
        load_tiles<P1>(h1, pre_row + c1 * 32, h);  // engine.level_pre6: alpha-folded W_f f + beta
        pipe_lds6<1, P1, P1>(wt, lane, sg, geom_b, h1, cin, s2, cb);
        (void)sf;
    } else {
        beta_p<P1, K::T1 * 32>(eb + e1, c1, h, h1);
        pipe_lds6<1, P1, P1>(wt, lane, sg, geom_b, h1, cin, sf, ca);
        pipe_lds6<NF, P1, P1>(
            wt, lane, sf,
            [&](int st0, float (&v)[4]) {
                const float4 t = *reinterpret_cast<const float4 *>(arow + 4 + h * TF + st0);
                v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
            },
            h1, ca, s2, cb);
    }
    relu_tiles(h1);
#pragma unroll
    for (int i = 0; i < P1; ++i) put_tile<LDSW>(B, c1 + i, j, h, h1[i]);
    tile_sync();
    f32x16 h2[P1];
    beta_p<P1, K::T1 * 32>(eb + e2, c1, h, h2);
    pipe_lds6<N1, P1, P3>(wt, lane, s2, ChanB{brow, h}, h2, cb, s3, ca);
    relu_tiles(h2);
    if constexpr (ONE) tile_sync();  // one buffer: every wave has read layer 2's input
#pragma unroll
    for (int i = 0; i < P1; ++i) put_tile<LDSW>(A, c1 + i, j, h, h2[i]);
    tile_sync();
    beta_p<P3, K::T3 * 32>(eb + e3, c3, h, out);
    pipe_lds6<N1, P3, NP>(wt, lane, s3, ChanB{arow, h}, out, ca, next, cout);
    relu_tiles(out);
}

// HREG_SPLIT_1BUF (default, PRE form): one activation buffer instead of two -- the
// geometry comes from registers, and a barrier before each write that replaces a layer's
// input (4 more per tile) -- so the LDS footprint drops from 80 to 47 KB (level 3) and three
// workgroups fit per CU (3 waves per SIMD at <= 168 VGPRs) instead of two.
#ifndef HREG_SPLIT_1BUF
#define HREG_SPLIT_1BUF 1
#endif

// HREG_SPLIT_RING (level 3, PRE form): one workgroup of RING_RT row tiles x 4 channel
// groups (12 waves, 3 per SIMD), the weight pieces through the channel-split LDS ring
// (split_chain.h RingCW: the RING_RT waves of a channel group share every piece), the
// epilogue constants read from the table in global memory; LDS 3 x 33 KB activations + 48 KB
// ring + 8 KB = 153 KB, one workgroup per CU.  Measured slower (off): 249 vs 195 us in the
// bench, 267 vs 190 standalone -- a step is only 6-12 MFMAs per wave between barriers that
// span all 12 waves of the CU, with no second workgroup to fill the gaps.
#ifndef HREG_SPLIT_RING
#define HREG_SPLIT_RING 0
#endif
constexpr int RING_RT = 3;

template <class K, bool PRE, bool ONE = (HREG_SPLIT_1BUF && PRE), bool RING = false>
__global__ __launch_bounds__(RING ? RING_RT * 256 : 256, RING ? 1 : ONE ? 3 : 2) void group_split6_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc, const float *__restrict__ pre) {
    constexpr int C3 = K::T3 * 32, CM2 = K::TM2 * 32, LDSW = K::LDSW, X2W = K::X2W;
    constexpr int T3 = K::T3, TM1 = K::TM1, P3 = K::P3, PM1 = K::PM1, PM2 = K::PM2;
    constexpr int N3 = K::N3, NM1 = K::NM1;
    constexpr int NE = K::TABLE - K::F_END, KN = K::KN, GPT = K::GPT, CW = K::CW;
    constexpr int RT = RING ? RING_RT : K::RT;
    static_assert(!RING || (ONE && PRE), "ring: one-buffer PRE form");
    __shared__ float ep[RING ? 1 : NE];
    __shared__ __attribute__((aligned(16))) float sA[RT][32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sB[ONE ? 1 : RT][ONE ? 4 : 32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sX2[RT][GPT * X2W];
    __shared__ int sMax[RT][CW][32];
    constexpr int PMAX = K::P3 > K::PM2 ? (K::P3 > K::P1 ? K::P3 : K::P1) : (K::PM2 > K::PM1 ? K::PM2 : K::PM1);
    __shared__ __attribute__((aligned(16))) u32x4 ring_lds[RING ? 2 * CW * PMAX * 192 : 1];
    if constexpr (!RING)
        for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    const float *eb = RING ? table : ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rt = w / CW, cw = w % CW;
    const int h = lane >> 5, j = lane & 31;
    const int NT = G / GPT;
    float *A = sA[rt], *B = ONE ? sA[rt] : sB[rt], *X2 = sX2[rt];
    const bool writer = KN == 32 ? j == 31 : (j & 15) == 15;
    auto gsum_w = [&](float v) { return KN == 32 ? half_sum_hi(v) : row_sum16(v); };
    auto gsum_b = [&](float v) { return KN == 32 ? half_bcast(half_sum_hi(v), h) : row_sum16(v); };
    auto gmax_w = [&](float v) { return KN == 32 ? half_max_hi_nonneg(v) : row_max16_nonneg(v); };
    auto gmax_b = [&](float v) {
        return KN == 32 ? half_bcast(half_max_hi_nonneg(v), h) : row_max16_nonneg(v);
    };
    const int c3 = cw * P3, m1 = cw * PM1, m2 = cw * PM2;
    const FragSeq det_g{K::G_DG + cw * K::P1, 1}, desc_g{K::G_EG + cw * K::P1, 1};
    const FragSeq m1x1{K::G_M1 + m1 * 3 * N3 + N3, 3 * N3};
    const FragSeq m1em{K::G_M1 + m1 * 3 * N3 + 2 * N3, 3 * N3};
    const FragSeq fm2{K::G_M2 + m2 * NM1, NM1};

    Carry6 carry;
    RingCW<CW * PMAX, RT * CW, CW> ring{reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table)),
                                       (lds_u32x4 *)ring_lds, 0, w, cw};
    if constexpr (RING) {
        ring_fill_cw<K::P1>(ring, 0, FragSeq{K::G_DG, 1}, K::P1, 0, lane);
    } else {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int i = 0; i < K::P1; ++i) ld6(wt, det_g.base + i * det_g.stride, lane, carry[i]);
    }
    for (int base = blockIdx.x * RT; base < NT; base += gridDim.x * RT) {
        // every wave of the workgroup runs the same trip count (barriers): a row tile
        // past the end recomputes the last tile (identical values, identical stores)
        const int t = min(base + rt, NT - 1);
        const int g = t * GPT + (KN == 32 ? 0 : j >> 4);
        const size_t row = (size_t)t * 32 + j;
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wtp = reinterpret_cast<const gu32x4 *>(tba);
        ring.wt = wtp;  // (opaque per tile: the DMA addresses are not hoisted out of the loop)
        auto &&wt = [&]() -> decltype(auto) {
            if constexpr (RING) return (ring);
            else return wtp;
        }();
        Carry6 ca, cb;

        const float *prow = PRE ? pre + (size_t)gidx[row] * (2 * K::T1 * 32) : nullptr;
        const float2 gin = ONE ? *reinterpret_cast<const float2 *>(geom + row * 4 + 2 * h) : make_float2(0.f, 0.f);
        tile_sync();  // previous tile's readers of A are done (and ep is loaded)
        if constexpr (!ONE) {
            stage_rows6<K, PRE>(A, geom, gidx, feats, t, cw, lane);
            tile_sync();
        }

        // ---- detector -> emb (this wave's P3 tiles)
        f32x16 emb[P3];
        conv_stack_split6<K, PM1, PRE, ONE>(wt, eb, K::G_DG, K::G_DF, K::G_D2, K::G_D3, K::E_D1, K::E_D2,
                                            K::E_D3, A, B, cw, lane, emb, carry, m1em, ca, prow, gin);

        // ---- attention (group_split.hip): row max over all C3 channels through LDS,
        // softmax over the group, keypoint and attentive feature
        int mi = __float_as_int(emb[0][0]);
#pragma unroll
        for (int i = 0; i < P3; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[i][q]));
        mi = max(mi, __shfl_xor(mi, 32));
        if (h == 0) sMax[rt][cw][j] = mi;
        tile_sync();
        int xm = sMax[rt][0][j];
#pragma unroll
        for (int c = 1; c < CW; ++c) xm = max(xm, sMax[rt][c][j]);
        const float x1 = __int_as_float(xm);
        const float mx = gmax_b(x1);
        const float e = expf(fsub_rn(x1, mx));
        const float a = e / gsum_b(e);
        if (cw == 0) {
            const float *p = knn_xyz + row * 3;
            const float kx = gsum_w(fmul_rn(a, p[0]));
            const float ky = gsum_w(fmul_rn(a, p[1]));
            const float kz = gsum_w(fmul_rn(a, p[2]));
            if (writer && h == 0) {
                kp[(size_t)g * 3 + 0] = kx;
                kp[(size_t)g * 3 + 1] = ky;
                kp[(size_t)g * 3 + 2] = kz;
            }
        }
#pragma unroll
        for (int i = 0; i < P3; ++i) {
            f32x16 v, ea;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                ea[q] = fmul_rn(emb[i][q], a);
                v[q] = gsum_w(ea[q]);
            }
            store_tile(att_feat + (size_t)g * C3, c3 + i, v, writer, h);
            put_tile<LDSW>(B, c3 + i, j, h, ea);
        }
        tile_sync();

        // ---- mlp1, emb*a part (y1 stays in registers through the descriptor stack)
        f32x16 y1[PM1];
        beta_p<PM1, TM1 * 32>(eb + K::E_M1, m1, h, y1);
        pipe_lds6<N3, PM1, K::P1>(wt, lane, m1em, ChanB{B + j * LDSW, h}, y1, ca, desc_g, cb);
        if constexpr (!ONE) stage_rows6<K, PRE>(A, geom, gidx, feats, t, cw, lane);
        tile_sync();  // (one buffer: every wave has read emb * a)

        // ---- descriptor -> x1d
        f32x16 x1d[P3];
        conv_stack_split6<K, PM1, PRE, ONE>(wt, eb, K::G_EG, K::G_EF, K::G_E2, K::G_E3, K::E_E1, K::E_E2,
                                            K::E_E3, A, B, cw, lane, x1d, cb, m1x1, ca,
                                            PRE ? prow + K::T1 * 32 : nullptr, gin);
        if constexpr (ONE) tile_sync();  // every wave has read layer 3's input
#pragma unroll
        for (int i = 0; i < P3; ++i) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = gmax_w(x1d[i][q]);
            if (writer) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<float4 *>(X2 + (KN == 32 ? 0 : j >> 4) * X2W + (c3 + i) * 32 + 8 * r +
                                                4 * h) = make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2],
                                                                     v[4 * r + 3]);
            }
            put_tile<LDSW>(B, c3 + i, j, h, x1d[i]);
        }
        tile_sync();

        // ---- mlp1, x2 part as one matrix-vector product per group (group_split.hip), f32
        {
            constexpr int CH = C3 / 2;
            float v[PM1][GPT];
#pragma unroll
            for (int i = 0; i < PM1; ++i) {
#pragma unroll
                for (int g2 = 0; g2 < GPT; ++g2) v[i][g2] = 0.f;
                const float *wr = table + K::F_X2 + (size_t)((m1 + i) * 32 + j) * C3 + h * CH;
#pragma unroll 8
                for (int c4 = 0; c4 < CH / 4; ++c4) {
                    const float4 wv = *reinterpret_cast<const float4 *>(wr + c4 * 4);
#pragma unroll
                    for (int g2 = 0; g2 < GPT; ++g2) {
                        const float4 xv = *reinterpret_cast<const float4 *>(X2 + g2 * X2W + h * CH + c4 * 4);
                        v[i][g2] = fmaf(wv.x, xv.x, v[i][g2]);
                        v[i][g2] = fmaf(wv.y, xv.y, v[i][g2]);
                        v[i][g2] = fmaf(wv.z, xv.z, v[i][g2]);
                        v[i][g2] = fmaf(wv.w, xv.w, v[i][g2]);
                    }
                }
#pragma unroll
                for (int g2 = 0; g2 < GPT; ++g2) v[i][g2] = fadd_rn(v[i][g2], __shfl_xor(v[i][g2], 32));
            }
            const int mg = KN == 32 ? 0 : j >> 4;
#pragma unroll
            for (int i = 0; i < PM1; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int src = (q & 3) + 8 * (q >> 2) + 4 * h;
                    float av = __shfl(v[i][0], src);
                    if constexpr (GPT == 2) {
                        const float bv = __shfl(v[i][1], src);
                        av = mg ? bv : av;
                    }
                    y1[i][q] = fadd_rn(y1[i][q], av);
                }
        }
        pipe_lds6<N3, PM1, PM2>(wt, lane, m1x1, ChanB{B + j * LDSW, h}, y1, ca, fm2, cb);
        relu_tiles(y1);
        if constexpr (ONE) tile_sync();  // every wave has read x1d
#pragma unroll
        for (int i = 0; i < PM1; ++i) put_tile<LDSW>(A, m1 + i, j, h, y1[i]);
        tile_sync();

        // ---- mlp2 + k-max -> descriptor; prefetches the next tile's first chunk
        f32x16 y2[PM2];
        beta_p<PM2, CM2>(eb + K::E_M2, m2, h, y2);
        pipe_lds6<NM1, PM2, K::P1>(wt, lane, fm2, ChanB{A + j * LDSW, h}, y2, cb, det_g, carry);
        relu_tiles(y2);
#pragma unroll
        for (int i = 0; i < PM2; ++i) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = gmax_w(y2[i][q]);
            store_tile(desc + (size_t)g * CM2, m2 + i, v, writer, h);
        }
    }
}

// ---------------------------------------------------------------------------------------
// Two row tiles per wave (level 3, PRE + one-buffer form): each wave of channel group cw runs
// the same layers as group_split6_kernel on two 32-row tiles at once (split_chain.h
// pipe_lds6_jt), so every weight piece it streams feeds the MFMAs of both tiles -- half the
// weight bytes per row on the L2 -> CU path that bounds the channel-split kernel (DESIGN.md
// 4c: "no weight loads" -26 % at level 3).  The two tiles' activations share one LDS buffer
// (64 rows); the epilogue constants are read from the table in global memory (the LDS copy
// would leave one workgroup per CU), so two 4-wave workgroups fit per CU.  Same products,
// same order per output as group_split6_kernel (bitwise equal, tests/test_gpu_model.py).
#ifndef HREG_L3_SJT
#define HREG_L3_SJT 2
#endif

template <int P, int C, int SJT>
__device__ __forceinline__ void beta_pj(const float *ab, int co0, int h, f32x16 (&acc)[P][SJT]) {
#pragma unroll
    for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 a = *reinterpret_cast<const float4 *>(ab + C + (co0 + i) * 32 + 8 * r + 4 * h);
                acc[i][jt][4 * r] = a.x; acc[i][jt][4 * r + 1] = a.y;
                acc[i][jt][4 * r + 2] = a.z; acc[i][jt][4 * r + 3] = a.w;
            }
}

template <int P, int SJT>
__device__ __forceinline__ void relu_j(f32x16 (&t)[P][SJT]) {
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
            for (int q = 0; q < 16; ++q) t[i][jt][q] = relu_i(t[i][jt][q]);
}

template <int LDSW, int P, int SJT>
__device__ __forceinline__ void put_j(float *buf, int co0, int j, int h, const f32x16 (&t)[P][SJT]) {
#pragma unroll
    for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
        for (int i = 0; i < P; ++i) put_tile<LDSW>(buf + jt * 32 * LDSW, co0 + i, j, h, t[i][jt]);
}

// conv stack [geom | precomputed feature block] -> C1 -> C1 -> C3 on two row tiles
template <class K, int NP, int SJT, class WT>
__device__ __forceinline__ void conv_stack_split6j(WT wt, const float *eb, int gg, int g2, int g3, int e2, int e3,
                                                   float *A, int cw, int lane, f32x16 (&out)[K::P3][SJT],
                                                   const Carry6 &cin, FragSeq next, Carry6 &cout,
                                                   const float *const (&pre_row)[SJT], const float2 (&gin)[SJT]) {
    constexpr int P1 = K::P1, P3 = K::P3, LDSW = K::LDSW, N1 = K::N1;
    const int h = lane >> 5, j = lane & 31;
    const int c1 = cw * P1, c3 = cw * P3;
    const FragSeq sg{gg + c1, 1}, s2{g2 + c1 * N1, N1}, s3{g3 + c3 * N1, N1};
    const float *arow = A + j * LDSW;
    Carry6 ca, cb;
    f32x16 h1[P1][SJT];
#pragma unroll
    for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
        for (int i = 0; i < P1; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // engine.level_pre6: alpha-folded W_f f + beta
                const float4 a = *reinterpret_cast<const float4 *>(pre_row[jt] + (c1 + i) * 32 + 8 * r + 4 * h);
                h1[i][jt][4 * r] = a.x; h1[i][jt][4 * r + 1] = a.y;
                h1[i][jt][4 * r + 2] = a.z; h1[i][jt][4 * r + 3] = a.w;
            }
    // geometry chunk: f32 k-steps 0, 1 (channels 2h, 2h + 1), the rest zero
    pipe_lds6_jt<1, P1, P1, SJT>(
        wt, lane, sg,
        [&](int jt, int st0, float (&v)[4]) {
            v[0] = st0 == 0 ? gin[jt].x : 0.f;
            v[1] = st0 == 0 ? gin[jt].y : 0.f;
            v[2] = 0.f; v[3] = 0.f;
        },
        h1, cin, s2, cb);
    relu_j(h1);
    put_j<LDSW>(A, c1, j, h, h1);
    tile_sync();
    f32x16 h2[P1][SJT];
    beta_pj<P1, K::T1 * 32, SJT>(eb + e2, c1, h, h2);
    pipe_lds6_jt<N1, P1, P3, SJT>(wt, lane, s2, ChanBJ<LDSW>{arow, h}, h2, cb, s3, ca);
    relu_j(h2);
    tile_sync();  // one buffer: every wave has read layer 2's input
    put_j<LDSW>(A, c1, j, h, h2);
    tile_sync();
    beta_pj<P3, K::T3 * 32, SJT>(eb + e3, c3, h, out);
    pipe_lds6_jt<N1, P3, NP, SJT>(wt, lane, s3, ChanBJ<LDSW>{arow, h}, out, ca, next, cout);
    relu_j(out);
}

template <class K, int SJT>
__global__ __launch_bounds__(256, SJT >= 4 ? 1 : 2) void group_split6j_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc, const float *__restrict__ pre) {
    constexpr int C3 = K::T3 * 32, CM2 = K::TM2 * 32, LDSW = K::LDSW, X2W = K::X2W;
    constexpr int TM1 = K::TM1, P3 = K::P3, PM1 = K::PM1, PM2 = K::PM2;
    constexpr int N3 = K::N3, NM1 = K::NM1;
    constexpr int KN = K::KN, GPT = K::GPT, CW = K::CW;
    static_assert(K::RT == 1 && CW == 4, "level-3 configuration");
    __shared__ __attribute__((aligned(16))) float sA[SJT * 32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sX2[SJT][GPT * X2W];
    __shared__ int sMax[SJT][CW][32];
    const float *eb = table;  // epilogue constants from global memory
    const int lane = threadIdx.x & 63, cw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G / GPT;
    const int NPAIR = (NT + SJT - 1) / SJT;  // row-tile sets of SJT
    float *A = sA;
    const bool writer = KN == 32 ? j == 31 : (j & 15) == 15;
    auto gsum_w = [&](float v) { return KN == 32 ? half_sum_hi(v) : row_sum16(v); };
    auto gsum_b = [&](float v) { return KN == 32 ? half_bcast(half_sum_hi(v), h) : row_sum16(v); };
    auto gmax_w = [&](float v) { return KN == 32 ? half_max_hi_nonneg(v) : row_max16_nonneg(v); };
    auto gmax_b = [&](float v) {
        return KN == 32 ? half_bcast(half_max_hi_nonneg(v), h) : row_max16_nonneg(v);
    };
    const int c3 = cw * P3, m1 = cw * PM1, m2 = cw * PM2;
    const FragSeq det_g{K::G_DG + cw * K::P1, 1}, desc_g{K::G_EG + cw * K::P1, 1};
    const FragSeq m1x1{K::G_M1 + m1 * 3 * N3 + N3, 3 * N3};
    const FragSeq m1em{K::G_M1 + m1 * 3 * N3 + 2 * N3, 3 * N3};
    const FragSeq fm2{K::G_M2 + m2 * NM1, NM1};

    Carry6 carry;
    {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int i = 0; i < K::P1; ++i) ld6(wt, det_g.base + i * det_g.stride, lane, carry[i]);
    }
    for (int pb = blockIdx.x; pb < NPAIR; pb += gridDim.x) {
        // a tile past the end recomputes the last tile (identical values, identical stores)
        int t[SJT], g[SJT];
        size_t row[SJT];
        const float *prow[SJT];
        float2 gin[SJT];
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt) {
            t[jt] = min(SJT * pb + jt, NT - 1);
            g[jt] = t[jt] * GPT + (KN == 32 ? 0 : j >> 4);
            row[jt] = (size_t)t[jt] * 32 + j;
            prow[jt] = pre + (size_t)gidx[row[jt]] * (2 * K::T1 * 32);
            gin[jt] = *reinterpret_cast<const float2 *>(geom + row[jt] * 4 + 2 * h);
        }
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
        Carry6 ca, cb;
        tile_sync();  // previous pair's readers of A are done

        // ---- detector -> emb
        f32x16 emb[P3][SJT];
        conv_stack_split6j<K, PM1, SJT>(wt, eb, K::G_DG, K::G_D2, K::G_D3, K::E_D2, K::E_D3, A, cw, lane, emb, carry,
                                   m1em, ca, prow, gin);

        // ---- attention per tile
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt) {
            int mi = __float_as_int(emb[0][jt][0]);
#pragma unroll
            for (int i = 0; i < P3; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[i][jt][q]));
            mi = max(mi, __shfl_xor(mi, 32));
            if (h == 0) sMax[jt][cw][j] = mi;
        }
        tile_sync();
        float a[SJT];
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt) {
            int xm = sMax[jt][0][j];
#pragma unroll
            for (int c = 1; c < CW; ++c) xm = max(xm, sMax[jt][c][j]);
            const float x1 = __int_as_float(xm);
            const float mx = gmax_b(x1);
            const float e = expf(fsub_rn(x1, mx));
            a[jt] = e / gsum_b(e);
            if (cw == 0) {
                const float *p = knn_xyz + row[jt] * 3;
                const float kx = gsum_w(fmul_rn(a[jt], p[0]));
                const float ky = gsum_w(fmul_rn(a[jt], p[1]));
                const float kz = gsum_w(fmul_rn(a[jt], p[2]));
                if (writer && h == 0) {
                    kp[(size_t)g[jt] * 3 + 0] = kx;
                    kp[(size_t)g[jt] * 3 + 1] = ky;
                    kp[(size_t)g[jt] * 3 + 2] = kz;
                }
            }
#pragma unroll
            for (int i = 0; i < P3; ++i) {
                f32x16 v, ea;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    ea[q] = fmul_rn(emb[i][jt][q], a[jt]);
                    v[q] = gsum_w(ea[q]);
                }
                store_tile(att_feat + (size_t)g[jt] * C3, c3 + i, v, writer, h);
                put_tile<LDSW>(A + jt * 32 * LDSW, c3 + i, j, h, ea);
            }
        }
        tile_sync();

        // ---- mlp1, emb * a part (y1 stays in registers through the descriptor stack)
        f32x16 y1[PM1][SJT];
        beta_pj<PM1, TM1 * 32, SJT>(eb + K::E_M1, m1, h, y1);
        pipe_lds6_jt<N3, PM1, K::P1, SJT>(wt, lane, m1em, ChanBJ<LDSW>{A + j * LDSW, h}, y1, ca, desc_g, cb);
        tile_sync();  // every wave has read emb * a

        // ---- descriptor -> x1d
        f32x16 x1d[P3][SJT];
        const float *prow_d[SJT];
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt) prow_d[jt] = prow[jt] + K::T1 * 32;
        conv_stack_split6j<K, PM1, SJT>(wt, eb, K::G_EG, K::G_E2, K::G_E3, K::E_E2, K::E_E3, A, cw, lane, x1d, cb, m1x1,
                                   ca, prow_d, gin);
        tile_sync();  // every wave has read layer 3's input
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
            for (int i = 0; i < P3; ++i) {
                f32x16 v;
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q] = gmax_w(x1d[i][jt][q]);
                if (writer) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        *reinterpret_cast<float4 *>(sX2[jt] + (KN == 32 ? 0 : j >> 4) * X2W + (c3 + i) * 32 + 8 * r +
                                                    4 * h) = make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2],
                                                                         v[4 * r + 3]);
                }
                put_tile<LDSW>(A + jt * 32 * LDSW, c3 + i, j, h, x1d[i][jt]);
            }
        tile_sync();

        // ---- mlp1, x2 part: one matrix-vector product per group, the weight rows shared by
        // both tiles' groups
        {
            constexpr int CH = C3 / 2;
            float v[PM1][SJT][GPT];
#pragma unroll
            for (int i = 0; i < PM1; ++i) {
#pragma unroll
                for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
                    for (int g2 = 0; g2 < GPT; ++g2) v[i][jt][g2] = 0.f;
                const float *wr = table + K::F_X2 + (size_t)((m1 + i) * 32 + j) * C3 + h * CH;
#pragma unroll 8
                for (int c4 = 0; c4 < CH / 4; ++c4) {
                    const float4 wv = *reinterpret_cast<const float4 *>(wr + c4 * 4);
#pragma unroll
                    for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
                        for (int g2 = 0; g2 < GPT; ++g2) {
                            const float4 xv = *reinterpret_cast<const float4 *>(sX2[jt] + g2 * X2W + h * CH + c4 * 4);
                            v[i][jt][g2] = fmaf(wv.x, xv.x, v[i][jt][g2]);
                            v[i][jt][g2] = fmaf(wv.y, xv.y, v[i][jt][g2]);
                            v[i][jt][g2] = fmaf(wv.z, xv.z, v[i][jt][g2]);
                            v[i][jt][g2] = fmaf(wv.w, xv.w, v[i][jt][g2]);
                        }
                }
#pragma unroll
                for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
                    for (int g2 = 0; g2 < GPT; ++g2) v[i][jt][g2] = fadd_rn(v[i][jt][g2], __shfl_xor(v[i][jt][g2], 32));
            }
            const int mg = KN == 32 ? 0 : j >> 4;
#pragma unroll
            for (int i = 0; i < PM1; ++i)
#pragma unroll
                for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int src = (q & 3) + 8 * (q >> 2) + 4 * h;
                        float av = __shfl(v[i][jt][0], src);
                        if constexpr (GPT == 2) {
                            const float bv = __shfl(v[i][jt][1], src);
                            av = mg ? bv : av;
                        }
                        y1[i][jt][q] = fadd_rn(y1[i][jt][q], av);
                    }
        }
        pipe_lds6_jt<N3, PM1, PM2, SJT>(wt, lane, m1x1, ChanBJ<LDSW>{A + j * LDSW, h}, y1, ca, fm2, cb);
        relu_j(y1);
        tile_sync();  // every wave has read x1d
        put_j<LDSW>(A, m1, j, h, y1);
        tile_sync();

        // ---- mlp2 + k-max -> descriptor; prefetches the next pair's first chunk
        f32x16 y2[PM2][SJT];
        beta_pj<PM2, CM2, SJT>(eb + K::E_M2, m2, h, y2);
        pipe_lds6_jt<NM1, PM2, K::P1, SJT>(wt, lane, fm2, ChanBJ<LDSW>{A + j * LDSW, h}, y2, cb, det_g, carry);
        relu_j(y2);
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
            for (int i = 0; i < PM2; ++i) {
                f32x16 v;
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q] = gmax_w(y2[i][jt][q]);
                store_tile(desc + (size_t)g[jt] * CM2, m2 + i, v, writer, h);
            }
    }
}

// ---------------------------------------------------------------------------------------
// Pieces form (level 3, PRE; hreg_group_split6p_l3).  In the channel-split kernels every wave
// splits every B chunk it reads into its bf16 pieces -- the same chunk once per channel group
// (4 x at level 3, ~75 % of the kernel's VALU).  Here the activations live in LDS already
// split: the wave that produces an output tile splits it once (split8 of its accumulator
// registers, mfma_chain.h) and stores the three pieces, and every consumer reads them with
// ds_read_b128 straight into the MFMA B operand.  Pieces take 6 B per value instead of 4, so
// one 8-wave workgroup (two 32-row tiles, 2 waves per SIMD) holds a 256-channel layer (96 KB):
//   * 256-channel layers (conv3, mlp2): wave w owns output tile w of both row tiles;
//   * 128-channel convs (conv1, conv2): wave w owns tile w % 4 of row tile w / 4;
//   * mlp1 (768 -> 128): wave w owns tile w % 4 of both row tiles over half of the K chunks
//     (w / 4), the two halves' partial sums meet in LDS (the x2 matrix-vector product of row
//     tile w / 4 is added to its wave's partial first) -- the weight pieces stream once per
//     workgroup as in group_split6j.
// Piece layout: ((chunk * 3 + piece) * 2 + lane half) * 64 + row -> one ds_read_b128 of a
// chunk's piece is 1 KB contiguous (conflict-free); the writer lanes' slots are the same.
// Same products per output element as group_split6j except mlp1's two-partial sum (kp and
// the attentive features bitwise, descriptors to fp32 rounding; tests/test_gpu_model.py).
namespace l3p {
constexpr int NWV = 8, PBUF = 16 * 3 * 2 * 64;  // waves; u32x4 pieces of a 256-channel layer (96 KB)

__device__ __forceinline__ int pslot(int kc, int p, int h, int r) { return ((kc * 3 + p) * 2 + h) * 64 + r; }

// the pieces of output tile co (lane (j, h): channels chan(co, q, h) of row rt * 32 + j) =
// B chunks 2 co (q 0..7) and 2 co + 1 (q 8..15) of the next layer
__device__ __forceinline__ void put_pieces(lds_u32x4 *buf, int co, int rt, int lane, const f32x16 &v) {
    const int h = lane >> 5, r = rt * 32 + (lane & 31);
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
        float x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = v[8 * c2 + i];
        u32x4 o[3];
        split8(x, o);
#pragma unroll
        for (int p = 0; p < 3; ++p) buf[pslot(2 * co + c2, p, h, r)] = o[p];
    }
}

// acc[jt] += sum_{c < NCH} A(fragment fb + c0 + c) x B_jt(chunk c0 + c); weights and B pieces
// one chunk ahead of the MFMAs (double-buffered registers)
template <int NCH, int NJ>
__device__ __forceinline__ void pipe_pc(const gu32x4 *__restrict__ wt, int lane, int fb, int c0,
                                        const lds_u32x4 *buf, const int (&roff)[NJ], f32x16 (&acc)[NJ]) {
    const int h = lane >> 5, j = lane & 31;
    u32x4 a[2][3], b[2][NJ][3];
    auto ldb = [&](int c, u32x4 (&d)[NJ][3]) {
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
            for (int p = 0; p < 3; ++p) d[jt][p] = buf[pslot(c0 + c, p, h, roff[jt] + j)];
    };
    ld6(wt, fb + c0, lane, a[0]);
    ldb(0, b[0]);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) {
            ld6(wt, fb + c0 + c + 1, lane, a[(c + 1) & 1]);
            ldb(c + 1, b[(c + 1) & 1]);
        }
#pragma unroll
        for (int jt = 0; jt < NJ; ++jt) acc[jt] = mma6(a[c & 1], b[c & 1][jt], acc[jt]);
        __builtin_amdgcn_sched_barrier(0);
    }
}
}  // namespace l3p

template <class K>
__global__ __launch_bounds__(512, 1) void group_split6p_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, int G, float *__restrict__ kp, float *__restrict__ att_feat,
    float *__restrict__ desc, const float *__restrict__ pre) {
    using namespace l3p;
    static_assert(K::KN == 16 && K::T1 == 4 && K::T3 == NWV && K::TM1 == 4 && K::TM2 == NWV, "level-3 shapes");
    constexpr int C1 = K::T1 * 32, C3 = K::T3 * 32, CM1 = K::TM1 * 32, CM2 = K::TM2 * 32, X2W = K::X2W;
    constexpr int N1 = K::N1, N3 = K::N3, NM1 = K::NM1, GPT = K::GPT;
    static_assert(N1 == 8 && N3 == 16 && NM1 == 8 && GPT == 2, "chunks");
    __shared__ __attribute__((aligned(16))) u32x4 pbuf[PBUF];
    __shared__ __attribute__((aligned(16))) float sX2[2][GPT * X2W];
    __shared__ int sMax[2][NWV][32];
    lds_u32x4 *bufA = (lds_u32x4 *)pbuf, *bufB = bufA + PBUF / 2;  // 128-channel layers (48 KB each)
    lds_u32x4 *bufE = bufA;                                         // 256-channel layers
    float *sR = (float *)pbuf;                                      // mlp1 partials (32 KB, below bufB)
    const float *eb = table;  // epilogue constants from global memory
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int t4 = w & 3, kh = w >> 2;  // 128-channel tile; row tile (convs) / K half (mlp1)
    const int NT = G / GPT, NPAIR = (NT + 1) / 2;
    const bool writer = (j & 15) == 15;
    const int r01[2] = {0, 32}, rk[1] = {kh * 32};

    for (int pb = blockIdx.x; pb < NPAIR; pb += gridDim.x) {
        // a tile past the end recomputes the last tile (identical values, identical stores)
        int t[2], g[2];
        size_t row[2];
        const float *prow[2];
        float2 gin[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            t[jt] = min(2 * pb + jt, NT - 1);
            g[jt] = t[jt] * GPT + (j >> 4);
            row[jt] = (size_t)t[jt] * 32 + j;
            prow[jt] = pre + (size_t)gidx[row[jt]] * (2 * C1);
            gin[jt] = *reinterpret_cast<const float2 *>(geom + row[jt] * 4 + 2 * h);
        }
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);

        // conv stack [geom | precomputed feature block] -> C1 -> C1 -> C3: out = tile w of both
        // row tiles (ReLU applied); gg .. e3: the stack's table blocks; poff: its pre_row block
        auto conv_stack = [&](int gg, int g2, int g3, int e2, int e3, int poff, f32x16 (&out)[2]) {
            f32x16 h1[1];
            load_tiles<1>(h1, prow[kh] + poff + t4 * 32, h);  // engine.level_pre6: alpha-folded W_f f + beta
            {
                const float x[8] = {gin[kh].x, gin[kh].y, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                u32x4 a[3], b[3];
                split8(x, b);  // geometry chunk: f32 k-steps 0, 1 (channels 2h, 2h + 1), the rest zero
                ld6(wt, gg + t4, lane, a);
                h1[0] = mma6(a, b, h1[0]);
            }
            relu_tiles(h1);
            put_pieces(bufA, t4, kh, lane, h1[0]);
            __syncthreads();
            f32x16 h2[1];
            load_tiles<1>(h2, eb + e2 + C1 + t4 * 32, h);
            pipe_pc<N1, 1>(wt, lane, g2 + t4 * N1, 0, bufA, rk, h2);
            relu_tiles(h2);
            put_pieces(bufB, t4, kh, lane, h2[0]);
            __syncthreads();
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) load_tiles<1>(*reinterpret_cast<f32x16(*)[1]>(&out[jt]), eb + e3 + C3 + w * 32, h);
            pipe_pc<N1, 2>(wt, lane, g3 + w * N1, 0, bufB, r01, out);
            relu_tiles(out);
        };

        // ---- detector -> emb (tile w of both row tiles)
        f32x16 emb[2];
        conv_stack(K::G_DG, K::G_D2, K::G_D3, K::E_D2, K::E_D3, 0, emb);

        // ---- attention per row tile: row max over all C3 channels through LDS (every wave has
        // also finished reading bufB at the barrier), softmax over the group
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            int mi = __float_as_int(emb[jt][0]);
#pragma unroll
            for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[jt][q]));
            mi = max(mi, __shfl_xor(mi, 32));
            if (h == 0) sMax[jt][w][j] = mi;
        }
        __syncthreads();
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            int xm = sMax[jt][0][j];
#pragma unroll
            for (int c = 1; c < NWV; ++c) xm = max(xm, sMax[jt][c][j]);
            const float x1 = __int_as_float(xm);
            const float mx = row_max16_nonneg(x1);
            const float e = expf(fsub_rn(x1, mx));
            const float a = e / row_sum16(e);
            if (w == 0) {
                const float *pp = knn_xyz + row[jt] * 3;
                const float kx = row_sum16(fmul_rn(a, pp[0]));
                const float ky = row_sum16(fmul_rn(a, pp[1]));
                const float kz = row_sum16(fmul_rn(a, pp[2]));
                if (writer && h == 0) {
                    kp[(size_t)g[jt] * 3 + 0] = kx;
                    kp[(size_t)g[jt] * 3 + 1] = ky;
                    kp[(size_t)g[jt] * 3 + 2] = kz;
                }
            }
            f32x16 v, ea;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                ea[q] = fmul_rn(emb[jt][q], a);
                v[q] = row_sum16(ea[q]);
            }
            store_tile(att_feat + (size_t)g[jt] * C3, w, v, writer, h);
            put_pieces(bufE, w, jt, lane, ea);
        }
        __syncthreads();

        // ---- mlp1, emb * a block: tile t4 of both row tiles over K half kh (the partial P stays in
        // registers through the descriptor stack; half 0 starts from beta)
        f32x16 P[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            if (kh == 0)
                load_tiles<1>(*reinterpret_cast<f32x16(*)[1]>(&P[jt]), eb + K::E_M1 + CM1 + t4 * 32, h);
            else
                P[jt] = zero16();
        }
        const int m1t = K::G_M1 + t4 * 3 * N3;
        pipe_pc<N3 / 2, 2>(wt, lane, m1t + 2 * N3, kh * (N3 / 2), bufE, r01, P);
        __syncthreads();  // every wave has read emb * a

        // ---- descriptor -> x1d; the group k-max rows x2 -> sX2
        f32x16 x1d[2];
        conv_stack(K::G_EG, K::G_E2, K::G_E3, K::E_E2, K::E_E3, C1, x1d);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = row_max16_nonneg(x1d[jt][q]);
            if (writer) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<float4 *>(sX2[jt] + (j >> 4) * X2W + w * 32 + 8 * r + 4 * h) =
                        make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
            }
        }
        __syncthreads();  // every wave has read layer 3's input; sX2 complete
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) put_pieces(bufE, w, jt, lane, x1d[jt]);
        __syncthreads();

        // ---- mlp1, x1d block (K half kh), then the x2 block of row tile kh as a matrix-vector
        // product per group (group_split6j), f32, added to this wave's partial
        pipe_pc<N3 / 2, 2>(wt, lane, m1t + N3, kh * (N3 / 2), bufE, r01, P);
        {
            constexpr int CH = C3 / 2;
            float v[GPT];
#pragma unroll
            for (int g2 = 0; g2 < GPT; ++g2) v[g2] = 0.f;
            const float *wr = table + K::F_X2 + (size_t)(t4 * 32 + j) * C3 + h * CH;
#pragma unroll 8
            for (int c4 = 0; c4 < CH / 4; ++c4) {
                const float4 wv = *reinterpret_cast<const float4 *>(wr + c4 * 4);
#pragma unroll
                for (int g2 = 0; g2 < GPT; ++g2) {
                    const float4 xv = *reinterpret_cast<const float4 *>(sX2[kh] + g2 * X2W + h * CH + c4 * 4);
                    v[g2] = fmaf(wv.x, xv.x, v[g2]);
                    v[g2] = fmaf(wv.y, xv.y, v[g2]);
                    v[g2] = fmaf(wv.z, xv.z, v[g2]);
                    v[g2] = fmaf(wv.w, xv.w, v[g2]);
                }
            }
#pragma unroll
            for (int g2 = 0; g2 < GPT; ++g2) v[g2] = fadd_rn(v[g2], __shfl_xor(v[g2], 32));
            const int mg = j >> 4;
            f32x16 &pk = kh ? P[1] : P[0];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int src = (q & 3) + 8 * (q >> 2) + 4 * h;
                const float av = __shfl(v[0], src), bv = __shfl(v[1], src);
                pk[q] = fadd_rn(pk[q], mg ? bv : av);
            }
        }
        __syncthreads();  // every wave has read x1d
        if (kh == 1) {
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<float4 *>(sR + ((t4 * 2 + jt) * 64 + lane) * 16 + 4 * r) =
                        make_float4(P[jt][4 * r], P[jt][4 * r + 1], P[jt][4 * r + 2], P[jt][4 * r + 3]);
        }
        __syncthreads();
        if (kh == 0) {
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) {
                f32x16 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float4 o = *reinterpret_cast<const float4 *>(sR + ((t4 * 2 + jt) * 64 + lane) * 16 + 4 * r);
                    y[4 * r] = relu_i(fadd_rn(P[jt][4 * r], o.x));
                    y[4 * r + 1] = relu_i(fadd_rn(P[jt][4 * r + 1], o.y));
                    y[4 * r + 2] = relu_i(fadd_rn(P[jt][4 * r + 2], o.z));
                    y[4 * r + 3] = relu_i(fadd_rn(P[jt][4 * r + 3], o.w));
                }
                put_pieces(bufB, t4, jt, lane, y);  // mlp2's input (128 channels) above the partials
            }
        }
        __syncthreads();

        // ---- mlp2 (tile w of both row tiles) + k-max -> descriptor
        f32x16 y2[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
            load_tiles<1>(*reinterpret_cast<f32x16(*)[1]>(&y2[jt]), eb + K::E_M2 + CM2 + w * 32, h);
        pipe_pc<NM1, 2>(wt, lane, K::G_M2 + w * NM1, 0, bufB, r01, y2);
        relu_tiles(y2);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = row_max16_nonneg(y2[jt][q]);
            store_tile(desc + (size_t)g[jt] * CM2, w, v, writer, h);
        }
    }
}

template <class K>
int launch_split6(const float *table, const float *geom, const float *knn_xyz, const int32_t *gidx,
                  const float *feats, int G, float *kp, float *att_feat, float *desc, const float *pre,
                  void *stream) {
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(feats) & 15) ||
        (reinterpret_cast<uintptr_t>(geom) & 15) || (reinterpret_cast<uintptr_t>(att_feat) & 15) ||
        (reinterpret_cast<uintptr_t>(desc) & 15) || (reinterpret_cast<uintptr_t>(pre) & 15))
        return HREG_ERR_INVALID;
    if (G % K::GPT) return HREG_ERR_INVALID;  // whole 32-row tiles
    if (!G) return HREG_OK;
    const int NT = G / K::GPT;
    constexpr bool RING = HREG_SPLIT_RING && HREG_SPLIT_1BUF && K::KN == 16;  // level 3
    if (RING && pre) {
        int grid = (NT + RING_RT - 1) / RING_RT;
        if (grid > 1024) grid = 1024;
        hipLaunchKernelGGL((group_split6_kernel<K, true, true, RING>), dim3(grid), dim3(RING_RT * 256), 0,
                           as_stream(stream), table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
        HREG_CHECK_LAUNCH();
        return HREG_OK;
    }
    int grid = (NT + K::RT - 1) / K::RT;
    const int cap = 256 * (HREG_SPLIT_1BUF && pre ? 3 : 2) * 2;  // resident workgroups per CU, two rounds
    if (grid > cap) grid = cap;
    if (pre)
        hipLaunchKernelGGL((group_split6_kernel<K, true>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    else
        hipLaunchKernelGGL((group_split6_kernel<K, false>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_group_split6_l2_table_floats(void) { return S2x6::TABLE; }
extern "C" int hreg_group_split6_l3_table_floats(void) { return S3x6::TABLE; }

extern "C" int hreg_group_split6_l2(const float *table, const float *geom, const float *knn_xyz,
                                    const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                                    float *desc, const float *pre, void *stream) {
    return launch_split6<S2x6>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}

// level 3 with two row tiles per wave (group_split6j_kernel): the precomputed-block form only
extern "C" int hreg_group_split6j_l3(const float *table, const float *geom, const float *knn_xyz,
                                     const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                                     float *desc, const float *pre, void *stream) {
    using K = S3x6;
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || !pre || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(geom) & 15) ||
        (reinterpret_cast<uintptr_t>(att_feat) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15) ||
        (reinterpret_cast<uintptr_t>(pre) & 15))
        return HREG_ERR_INVALID;
    if (G % K::GPT) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    constexpr int SJ = HREG_L3_SJT;
    const int NT = G / K::GPT, NSET = (NT + SJ - 1) / SJ;
    int grid = NSET;
    const int cap = 256 * (SJ >= 4 ? 1 : 2) * 2;  // resident workgroups per CU, two rounds
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL((group_split6j_kernel<K, SJ>), dim3(grid), dim3(256), 0, as_stream(stream), table, geom,
                       knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_split6_l3(const float *table, const float *geom, const float *knn_xyz,
                                    const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                                    float *desc, const float *pre, void *stream) {
    return launch_split6<S3x6>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}

// level 3, pieces form (group_split6p_kernel): the precomputed-block form only; same table
extern "C" int hreg_group_split6p_l3(const float *table, const float *geom, const float *knn_xyz,
                                     const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                                     float *desc, const float *pre, void *stream) {
    using K = S3x6;
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || !pre || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(geom) & 15) ||
        (reinterpret_cast<uintptr_t>(att_feat) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15) ||
        (reinterpret_cast<uintptr_t>(pre) & 15))
        return HREG_ERR_INVALID;
    if (G % K::GPT) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    const int NT = G / K::GPT, NPAIR = (NT + 1) / 2;
    int grid = NPAIR;
    const int cap = 256 * 2;  // one workgroup per CU, two rounds
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(group_split6p_kernel<K>, dim3(grid), dim3(512), 0, as_stream(stream), table, geom, knn_xyz,
                       gidx, G, kp, att_feat, desc, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
