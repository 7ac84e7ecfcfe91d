// group_split.hip -- level-2 / level-3 keypoint detector + descriptor, channel-split.
//
// Same computation and weight order as group_fused.hip (layers.py:115-121,150-159,
// 183-208; see that file), different decomposition.  group_fused.hip keeps a whole
// 32-row tile's activations in one wave's accumulators, which at level 3 needs all
// 512 VGPRs (one wave per SIMD, spills): any wait of that wave idles the SIMD's
// matrix core.  Here a workgroup of 4 waves owns RT row tiles; the waves of a row
// tile split every layer's output channels CW ways (wave cw computes tiles
// co = cw*P + i), the activations of a layer go through LDS (row-major, stride
// LDSW = widest layer + 4 floats, written and read as float4 in the MFMA
// accumulator's channel order), and the next layer streams its B operand from LDS
// one window ahead, like the A fragments from the L2-resident table.  Per wave:
// P <= 2 output tiles, ~130 VGPRs; two workgroups per CU (LDS 2 x ~70 KB), so one
// workgroup's barriers / epilogues overlap the other's MFMAs.  A-fragment windows
// hold 32 fragments (2 x the chained kernel's), hiding a longer L2 latency.
//
// Per 32-row tile (4 waves, 11 workgroup barriers):
//   stage [geom 4 | gathered feature CF] rows -> A
//   det conv1 A->B, conv2 B->A, conv3 A->emb (registers)
//   attention: per-wave channel max -> LDS -> row max, softmax over the group,
//              keypoint and attentive feature (each wave its channels)
//   emb*a -> B; mlp1 (emb*a part) B -> y1 (registers, kept)
//   stage again -> A; desc conv1 A->B, conv2 B->A, conv3 A->x1d
//   x2 = k-max(x1d) -> X2 (one row per group), x1d -> B; mlp1 (x2, x1d parts) -> y1
//   y1 -> A; mlp2 A -> y2, k-max -> descriptor
#include "../split_chain.h"

namespace {

using namespace hreg_chain;
using namespace hreg_split;

// KN neighbours per group, CF gathered feature channels, conv widths C1/C3, mlp
// widths CM1/CM2; RT row tiles x CW channel-split waves = 4 waves per workgroup.
// Table layout: group_fused.hip Cfg offsets, fragments grouped 4 k-steps
// innermost per lane ([co][step/4][lane][4]; the 2-step geometry block: [co][lane][2]),
// engine.split_table.
template <int KN_, int CF_, int C1, int C3, int CM1, int CM2, int RT_, int CW_>
struct SCfg {
    static constexpr int KN = KN_, CF = CF_, RT = RT_, CW = CW_;
    static constexpr int TF = CF / 2;
    static constexpr int T1 = C1 / 32, T3 = C3 / 32, TM1 = CM1 / 32, TM2 = CM2 / 32;
    static constexpr int P1 = T1 / CW, P3 = T3 / CW, PM1 = TM1 / CW, PM2 = TM2 / CW;
    static_assert(P1 * CW == T1 && P3 * CW == T3 && PM1 * CW == TM1 && PM2 * CW == TM2, "split");
    static_assert(RT * CW == 4, "4 waves");
    static constexpr int F_DG = 0;
    static constexpr int F_DF = F_DG + T1 * 2 * 64;
    static constexpr int F_D2 = F_DF + T1 * TF * 64;
    static constexpr int F_D3 = F_D2 + T1 * T1 * 16 * 64;
    static constexpr int F_EG = F_D3 + T3 * T1 * 16 * 64;
    static constexpr int F_EF = F_EG + T1 * 2 * 64;
    static constexpr int F_E2 = F_EF + T1 * TF * 64;
    static constexpr int F_E3 = F_E2 + T1 * T1 * 16 * 64;
    static constexpr int F_M1 = F_E3 + T3 * T1 * 16 * 64;
    static constexpr int F_M2 = F_M1 + TM1 * 3 * T3 * 16 * 64;
    static constexpr int F_X2 = F_M2 + TM2 * TM1 * 16 * 64;  // mlp1 x2 block, row-major [CM1][C3]
    static constexpr int F_END = F_X2 + CM1 * C3;
    static constexpr int E_D1 = F_END, E_D2 = E_D1 + 2 * C1, E_D3 = E_D2 + 2 * C1,
                         E_E1 = E_D3 + 2 * C3, E_E2 = E_E1 + 2 * C1, E_E3 = E_E2 + 2 * C1,
                         E_M1 = E_E3 + 2 * C3, E_M2 = E_M1 + 2 * CM1, TABLE = E_M2 + 2 * CM2;
    static constexpr int W0 = C3 > 4 + CF ? C3 : 4 + CF;
    static constexpr int LDSW = (W0 > CM1 ? W0 : CM1) + 4;  // row stride (floats)
    static constexpr int GPT = 32 / KN;                      // groups per row tile
    static constexpr int X2W = C3 + 4;
};

using S2 = SCfg<32, 64, 64, 128, 64, 128, 2, 2>;
using S3 = SCfg<16, 128, 128, 256, 128, 256, 1, 4>;

// stage [geom 4 | feats[gidx[row]] CF] of the tile's 32 rows into buf (the CW waves
// of the row tile share the float4 loads)
template <class K, bool PRE = false>
__device__ __forceinline__ void stage_rows(float *buf, const float *__restrict__ geom,
                                           const int32_t *__restrict__ gidx,
                                           const float *__restrict__ feats, int t, int cw, int lane) {
    constexpr int F4 = PRE ? 1 : 1 + K::CF / 4;  // PRE: the first layer reads geometry only
#pragma unroll
    for (int i = cw * 64 + lane; i < 32 * F4; i += K::CW * 64) {
        const int r = i / F4, c4 = i - r * F4;
        const size_t row = (size_t)t * 32 + r;
        const float *src = c4 == 0 ? geom + row * 4 : feats + (size_t)gidx[row] * K::CF + (c4 - 1) * 4;
        *reinterpret_cast<float4 *>(buf + r * K::LDSW + c4 * 4) = *reinterpret_cast<const float4 *>(src);
    }
}

// conv stack [geom | feat] -> C1 -> C1 -> C3 through the A/B buffers; result tiles
// in out (epilogue applied).  Ends with out in registers; A / B free after the
// caller's next barrier.
// PRE: the first layer's feature part precomputed per source point (pre_row = W_f f of
// the row's neighbour, C1 channels) initialises this wave's P1 tiles; only the 2
// geometry k-steps run here.
template <class K, int NP, int NWN, bool PRE = false>
__device__ __forceinline__ void conv_stack_split(const gfloat *__restrict__ tb, const float *eb, int fg,
                                                 int ff, int f2, int f3, int e1, int e2, int e3,
                                                 float *A, float *B, int cw, int lane,
                                                 f32x16 (&out)[K::P3], const float (&cin)[SCARRY],
                                                 FragSeq next, float (&cout)[SCARRY],
                                                 const float *pre_row = nullptr) {
    constexpr int T1 = K::T1, TF = K::TF, P1 = K::P1, P3 = K::P3, LDSW = K::LDSW;
    const int h = lane >> 5, j = lane & 31;
    const int c1 = cw * P1, c3 = cw * P3;
    const FragSeq sg{fg / 64 + c1 * 2, 2}, sf{ff / 64 + c1 * TF, TF};
    const FragSeq s2{f2 / 64 + c1 * T1 * 16, T1 * 16}, s3{f3 / 64 + c3 * T1 * 16, T1 * 16};
    const float *arow = A + j * LDSW, *brow = B + j * LDSW;
    float ca[SCARRY], cb[SCARRY];
    f32x16 h1[P1];
    auto geom_b = [&](int st0, float (&v)[2]) {
        const float2 t = *reinterpret_cast<const float2 *>(arow + 2 * h);
        v[0] = t.x; v[1] = t.y;
    };
    if constexpr (PRE) {
        load_tiles<P1>(h1, pre_row + c1 * 32, h);
        pipe_lds<2, P1, P1, swin<T1 * 16>()>(tb, lane, sg, geom_b, h1, cin, s2, cb);
        (void)sf;
    } else {
        zero_tiles(h1);
        pipe_lds<2, P1, P1, swin<TF>()>(tb, lane, sg, geom_b, h1, cin, sf, ca);
        pipe_lds<TF, P1, P1, swin<T1 * 16>()>(
            tb, lane, sf,
            [&](int st0, float (&v)[4]) {
                const float4 t = *reinterpret_cast<const float4 *>(arow + 4 + h * TF + st0);
                v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
            },
            h1, ca, s2, cb);
    }
    epi<P1, K::T1 * 32>(eb + e1, c1, h, h1);
#pragma unroll
    for (int i = 0; i < P1; ++i) put_tile<LDSW>(B, c1 + i, j, h, h1[i]);
    tile_sync();
    f32x16 h2[P1];
    zero_tiles(h2);
    pipe_lds<T1 * 16, P1, P3, swin<T1 * 16>()>(tb, lane, s2, ChanB{brow, h}, h2, cb, s3, ca);
    epi<P1, K::T1 * 32>(eb + e2, c1, h, h2);
#pragma unroll
    for (int i = 0; i < P1; ++i) put_tile<LDSW>(A, c1 + i, j, h, h2[i]);
    tile_sync();
    zero_tiles(out);
    pipe_lds<T1 * 16, P3, NP, NWN>(tb, lane, s3, ChanB{arow, h}, out, ca, next, cout);
    epi<P3, K::T3 * 32>(eb + e3, c3, h, out);
}

template <class K, bool PRE>
__global__ __launch_bounds__(256, 2) void group_split_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc, const float *__restrict__ pre) {
    constexpr int C3 = K::T3 * 32, CM2 = K::TM2 * 32, LDSW = K::LDSW, X2W = K::X2W;
    constexpr int T3 = K::T3, TM1 = K::TM1, P3 = K::P3, PM1 = K::PM1, PM2 = K::PM2;
    constexpr int NE = K::TABLE - K::F_END, KN = K::KN, GPT = K::GPT, RT = K::RT, CW = K::CW;
    __shared__ float ep[NE];
    __shared__ __attribute__((aligned(16))) float sA[RT][32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sB[RT][32 * LDSW];
    __shared__ __attribute__((aligned(16))) float sX2[RT][GPT * X2W];
    __shared__ int sMax[RT][CW][32];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rt = w / CW, cw = w % CW;
    const int h = lane >> 5, j = lane & 31;
    const int NT = G / GPT;
    float *A = sA[rt], *B = sB[rt], *X2 = sX2[rt];
    const bool writer = KN == 32 ? j == 31 : (j & 15) == 15;
    auto gsum_w = [&](float v) { return KN == 32 ? half_sum_hi(v) : row_sum16(v); };
    auto gsum_b = [&](float v) { return KN == 32 ? half_bcast(half_sum_hi(v), h) : row_sum16(v); };
    auto gmax_w = [&](float v) { return KN == 32 ? half_max_hi_nonneg(v) : row_max16_nonneg(v); };
    auto gmax_b = [&](float v) {
        return KN == 32 ? half_bcast(half_max_hi_nonneg(v), h) : row_max16_nonneg(v);
    };
    const int c3 = cw * P3, m1 = cw * PM1, m2 = cw * PM2;
    constexpr int MS = 3 * T3 * 16;  // mlp1 fragment stride per output tile
    const FragSeq det_g{K::F_DG / 64 + cw * K::P1 * 2, 2}, desc_g{K::F_EG / 64 + cw * K::P1 * 2, 2};
    const FragSeq m1x1{K::F_M1 / 64 + m1 * MS + T3 * 16, MS};
    const FragSeq m1em{K::F_M1 / 64 + m1 * MS + 2 * T3 * 16, MS};
    const FragSeq fm2{K::F_M2 / 64 + m2 * TM1 * 16, TM1 * 16};

    float carry[SCARRY];
    {
        const gfloat *tb = reinterpret_cast<const gfloat *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int i = 0; i < K::P1; ++i) {
            float v[2];
            ldgroup<2>(tb, det_g.base + i * 2, lane, v);
            carry[i] = v[0];
            carry[K::P1 + i] = v[1];
        }
    }
    for (int base = blockIdx.x * RT; base < NT; base += gridDim.x * RT) {
        // every wave of the workgroup runs the same trip count (barriers): a row tile
        // past the end recomputes the last tile (identical values, identical stores)
        const int t = min(base + rt, NT - 1);
        const int g = t * GPT + (KN == 32 ? 0 : j >> 4);
        const size_t row = (size_t)t * 32 + j;
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gfloat *tb = reinterpret_cast<const gfloat *>(tba);
        float ca[SCARRY], cb[SCARRY];

        // PRE: this lane's row of the precomputed first-layer products [det C1 | desc C1]
        const float *prow = PRE ? pre + (size_t)gidx[row] * (2 * K::T1 * 32) : nullptr;
        tile_sync();  // previous tile's readers of A are done (and ep is loaded)
        stage_rows<K, PRE>(A, geom, gidx, feats, t, cw, lane);
        tile_sync();

        // ---- detector -> emb (this wave's P3 tiles)
        f32x16 emb[P3];
        conv_stack_split<K, PM1, swin<T3 * 16>(), PRE>(tb, eb, K::F_DG, K::F_DF, K::F_D2, K::F_D3,
                                                       K::E_D1, K::E_D2, K::E_D3, A, B, cw, lane, emb,
                                                       carry, m1em, ca, prow);

        // ---- attention: row max over all C3 channels (per-wave partial maxima through
        // LDS; emb >= 0 after ReLU: integer max on the bit patterns), softmax over the group
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
        zero_tiles(y1);
        pipe_lds<T3 * 16, PM1, K::P1, 2>(tb, lane, m1em, ChanB{B + j * LDSW, h}, y1, ca, desc_g,
                                         cb);
        stage_rows<K, PRE>(A, geom, gidx, feats, t, cw, lane);
        tile_sync();

        // ---- descriptor -> x1d
        f32x16 x1d[P3];
        conv_stack_split<K, PM1, swin<T3 * 16>(), PRE>(tb, eb, K::F_EG, K::F_EF, K::F_E2, K::F_E3,
                                                       K::E_E1, K::E_E2, K::E_E3, A, B, cw, lane, x1d,
                                                       cb, m1x1, ca, PRE ? prow + K::T1 * 32 : nullptr);
        // x2 = k-max of x1d (one row per group) -> X2; x1d -> B
#pragma unroll
        for (int i = 0; i < P3; ++i) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = gmax_w(x1d[i][q]);
            if (writer) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<float4 *>(X2 + (KN == 32 ? 0 : j >> 4) * X2W + (c3 + i) * 32 +
                                                8 * r + 4 * h) =
                        make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
            }
            put_tile<LDSW>(B, c3 + i, j, h, x1d[i]);
        }
        tile_sync();

        // ---- mlp1, x2 part: x2 (the k-max row, layers.py:204-206) is the same for every
        // row of a group, so W_x2 x2 is a matrix-vector product per group -- lane j of
        // half h: output channel (m1 + i) * 32 + j over the half's C3 / 2 input channels
        // (W_x2 rows from the L2-resident table, x2 from X2 as LDS broadcasts), halves
        // summed, then moved into the accumulator layout -- instead of MFMAs over the
        // group's 16 / 32 identical rows.  Then the x1d part.
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
                for (int g2 = 0; g2 < GPT; ++g2)  // commutative: both halves get the same bits
                    v[i][g2] = fadd_rn(v[i][g2], __shfl_xor(v[i][g2], 32));
            }
            const int mg = KN == 32 ? 0 : j >> 4;
#pragma unroll
            for (int i = 0; i < PM1; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int src = (q & 3) + 8 * (q >> 2) + 4 * h;  // lane holding chan(m1+i, q, h)
                    float a = __shfl(v[i][0], src);
                    if constexpr (GPT == 2) {
                        const float b = __shfl(v[i][1], src);
                        a = mg ? b : a;
                    }
                    y1[i][q] = fadd_rn(y1[i][q], a);
                }
        }
        pipe_lds<T3 * 16, PM1, PM2, swin<TM1 * 16>()>(tb, lane, m1x1, ChanB{B + j * LDSW, h}, y1,
                                                      ca, fm2, cb);
        epi<PM1, TM1 * 32>(eb + K::E_M1, m1, h, y1);
#pragma unroll
        for (int i = 0; i < PM1; ++i) put_tile<LDSW>(A, m1 + i, j, h, y1[i]);
        tile_sync();

        // ---- mlp2 + k-max -> descriptor; prefetches the next tile's first window
        f32x16 y2[PM2];
        zero_tiles(y2);
        pipe_lds<TM1 * 16, PM2, K::P1, 2>(tb, lane, fm2, ChanB{A + j * LDSW, h}, y2, cb, det_g,
                                          carry);
        epi<PM2, CM2>(eb + K::E_M2, m2, h, y2);
#pragma unroll
        for (int i = 0; i < PM2; ++i) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = gmax_w(y2[i][q]);
            store_tile(desc + (size_t)g * CM2, m2 + i, v, writer, h);
        }
    }
}

template <class K>
int launch_split(const float *table, const float *geom, const float *knn_xyz, const int32_t *gidx,
                 const float *feats, int G, float *kp, float *att_feat, float *desc, const float *pre,
                 void *stream) {
    if (reinterpret_cast<uintptr_t>(pre) & 15) return HREG_ERR_INVALID;
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(feats) & 15) || (reinterpret_cast<uintptr_t>(geom) & 15) ||
        (reinterpret_cast<uintptr_t>(att_feat) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15))
        return HREG_ERR_INVALID;
    if (G % K::GPT) return HREG_ERR_INVALID;  // whole 32-row tiles
    if (!G) return HREG_OK;
    const int NT = G / K::GPT;
    int grid = (NT + K::RT - 1) / K::RT;
    const int cap = 256 * 2 * 2;  // two resident workgroups per CU, two rounds
    if (grid > cap) grid = cap;
    if (pre)
        hipLaunchKernelGGL((group_split_kernel<K, true>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    else
        hipLaunchKernelGGL((group_split_kernel<K, false>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_group_split_l2_table_floats(void) { return S2::TABLE; }
extern "C" int hreg_group_split_l3_table_floats(void) { return S3::TABLE; }

extern "C" int hreg_group_split_l2(const float *table, const float *geom, const float *knn_xyz,
                                   const int32_t *gidx, const float *feats, int G, float *kp,
                                   float *att_feat, float *desc, const float *pre, void *stream) {
    return launch_split<S2>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}

extern "C" int hreg_group_split_l3(const float *table, const float *geom, const float *knn_xyz,
                                   const int32_t *gidx, const float *feats, int G, float *kp,
                                   float *att_feat, float *desc, const float *pre, void *stream) {
    return launch_split<S3>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}
