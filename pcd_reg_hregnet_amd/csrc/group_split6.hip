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

// ONE (the PRE form): one activation buffer instead of two -- the geometry comes from registers,
// and a barrier before each write that replaces a layer's input (4 more per tile) -- so the LDS
// footprint drops from 80 to 47 KB (level 3) and three workgroups fit per CU (3 waves per SIMD at
// <= 168 VGPRs) instead of two.  (r3, measured and removed: a channel-split LDS weight ring of 12-wave
// workgroups, 249 vs 195 us -- a step is only 6-12 MFMAs per wave between barriers spanning all 12
// waves of the CU, with no second workgroup to fill the gaps.)
template <class K, bool PRE, bool ONE = PRE>
__global__ __launch_bounds__(256, ONE ? 3 : 2) void group_split6_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc, const float *__restrict__ pre) {
    constexpr int C3 = K::T3 * 32, CM2 = K::TM2 * 32, LDSW = K::LDSW, X2W = K::X2W;
    constexpr int T3 = K::T3, TM1 = K::TM1, P3 = K::P3, PM1 = K::PM1, PM2 = K::PM2;
    constexpr int N3 = K::N3, NM1 = K::NM1;
    constexpr int NE = K::TABLE - K::F_END, KN = K::KN, GPT = K::GPT, CW = K::CW;
    constexpr int RT = K::RT;
    __shared__ float ep[NE];
    __shared__ __attribute__((aligned(16))) float sA[RT][32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sB[ONE ? 1 : RT][ONE ? 4 : 32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sX2[RT][GPT * X2W];
    __shared__ int sMax[RT][CW][32];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    const float *eb = ep - K::F_END;
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
    {
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
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
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
// (r5, measured and removed: four row tiles per wave -- one wave per SIMD, 256 VGPR + 248 AGPR --
// 169 -> 245 us.)

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
    pipe_lds6_jt<1, P1, P1, SJT, false>(
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
    pipe_lds6_jt<N1, P1, P3, SJT, false>(wt, lane, s2, ChanBJ<LDSW>{arow, h}, h2, cb, s3, ca);
    relu_j(h2);
    tile_sync();  // one buffer: every wave has read layer 2's input
    put_j<LDSW>(A, c1, j, h, h2);
    tile_sync();
    beta_pj<P3, K::T3 * 32, SJT>(eb + e3, c3, h, out);
    pipe_lds6_jt<N1, P3, NP, SJT, false>(wt, lane, s3, ChanBJ<LDSW>{arow, h}, out, ca, next, cout);
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
        pipe_lds6_jt<N3, PM1, K::P1, SJT, false>(wt, lane, m1em, ChanBJ<LDSW>{A + j * LDSW, h}, y1, ca, desc_g, cb);
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
        pipe_lds6_jt<N3, PM1, PM2, SJT, false>(wt, lane, m1x1, ChanBJ<LDSW>{A + j * LDSW, h}, y1, ca, fm2, cb);
        relu_j(y1);
        tile_sync();  // every wave has read x1d
        put_j<LDSW>(A, m1, j, h, y1);
        tile_sync();

        // ---- mlp2 + k-max -> descriptor; prefetches the next pair's first chunk
        f32x16 y2[PM2][SJT];
        beta_pj<PM2, CM2, SJT>(eb + K::E_M2, m2, h, y2);
        pipe_lds6_jt<NM1, PM2, K::P1, SJT, false>(wt, lane, fm2, ChanBJ<LDSW>{A + j * LDSW, h}, y2, cb, det_g, carry);
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
    int grid = (NT + K::RT - 1) / K::RT;
    const int cap = 256 * (pre ? 3 : 2) * 2;  // resident workgroups per CU, two rounds
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
    constexpr int SJ = 2;
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
