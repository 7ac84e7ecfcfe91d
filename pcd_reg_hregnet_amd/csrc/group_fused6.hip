// group_fused6.hip -- the fused level-2 / level-3 keypoint detector + descriptor of
// group_fused.hip (same layers, same decomposition: one wave owns one 32-row tile
// with every layer's activations in its MFMA accumulators, layers.py:115-121,
// 150-159, 183-208) with the products on the bf16 matrix cores at fp32 accuracy
// (bf16x6, mfma_chain.h): each 16-deep k-chunk is 6 v_mfma_f32_32x32x16_bf16 (192
// cycles) instead of 8 v_mfma_f32_32x32x2_f32 (512 cycles).  The B operand of a
// chunk (8 consecutive f32 k-steps of the lane: accumulator registers of the previous
// layer, gathered feature channels or the geometry) is split into its three bf16
// pieces in registers; the weights come pre-split from the table
// (engine.l2_table6: [co][chunk][piece][lane] 16-byte pieces, L2-resident, streamed
// one chunk ahead and across call boundaries as in group_fused.hip).  The 4-column
// geometry block is one zero-padded chunk.  BN is folded (engine._fold_bn: alpha in the
// weights, the accumulators start from beta, the epilogue is the ReLU).  Attention as in
// group_fused.hip; the per-channel reductions over a group's rows (attentive feature, x2,
// descriptor k-max) are butterflies over a tile's 16 values (rowred.h).
#include "mfma_jt.h"
#include "rowred.h"

namespace {

using namespace hreg_chain;
using namespace hreg_rowred;

constexpr int WAVES = 4;

template <int KN_, int CF, int C1, int C3, int CM1, int CM2, int WPS_>
struct Cfg6 {
    static constexpr int KN = KN_, WPS = WPS_;
    static constexpr int TF = CF / 2, NF = TF / 8;  // feature k-steps / chunks
    static constexpr int T1 = C1 / 32, T3 = C3 / 32, TM1 = CM1 / 32, TM2 = CM2 / 32;
    static constexpr int N1 = T1 * 2, N3 = T3 * 2, NM1 = TM1 * 2;  // chunks over C1 / C3 / CM1 inputs
    // chunk-fragment table (units of 3 pieces x 64 lanes x 16 B), engine.l2_table6
    static constexpr int G_DG = 0;                    // det conv1, geom [T1][1]
    static constexpr int G_DF = G_DG + T1;            // det conv1, feat [T1][NF]
    static constexpr int G_D2 = G_DF + T1 * NF;       // det conv2 [T1][N1]
    static constexpr int G_D3 = G_D2 + T1 * N1;       // det conv3 [T3][N1]
    static constexpr int G_EG = G_D3 + T3 * N1;
    static constexpr int G_EF = G_EG + T1;
    static constexpr int G_E2 = G_EF + T1 * NF;
    static constexpr int G_E3 = G_E2 + T1 * N1;
    static constexpr int G_M1 = G_E3 + T3 * N1;       // mlp1 [TM1][3 N3]: x2 | x1d | emb*a
    static constexpr int G_M2 = G_M1 + TM1 * 3 * N3;  // mlp2 [TM2][NM1]
    static constexpr int G_END = G_M2 + TM2 * NM1;
    static constexpr int F_END = G_END * 3 * 64 * 4;  // floats; the f32 epilogue section follows
    static constexpr int E_D1 = F_END, E_D2 = E_D1 + 2 * C1, E_D3 = E_D2 + 2 * C1,
                         E_E1 = E_D3 + 2 * C3, E_E2 = E_E1 + 2 * C1, E_E3 = E_E2 + 2 * C1,
                         E_M1 = E_E3 + 2 * C3, E_M2 = E_M1 + 2 * CM1, TABLE = E_M2 + 2 * CM2;
};

using L2 = Cfg6<32, 64, 64, 128, 64, 128, 2>;
using L3 = Cfg6<16, 128, 128, 256, 128, 256, 1>;

using hreg_jt::Carry;

// conv stack [geom 4 | gathered feature CF] -> C1 -> C1 -> C3 (+ BN/ReLU epilogues);
// NC: output tiles of the call that follows (its first chunk is prefetched into cout).
// PRE: the feature part of the first layer comes precomputed per source point and
// initialises the accumulators (group_fused.hip).
template <class K, int NC, bool PRE, class WT>
__device__ __forceinline__ void conv_stack6(WT &&wt, const float *eb, int gg, int gf,
                                            int g2, int g3, int e1, int e2, int e3, int lane, float2 gin,
                                            const float4 (&fin)[K::TF / 4], const float *pre_row,
                                            f32x16 (&out)[K::T3], const Carry &cin, FragSeq next,
                                            Carry &cout) {
    constexpr int T1 = K::T1, T3 = K::T3, NF = K::NF, N1 = K::N1;
    const FragSeq sg{gg, 1}, sf{gf, NF}, s2{g2, N1}, s3{g3, N1};
    f32x16 h1[T1], h2[T1];
    Carry c1, c2, c3;
    const int h = lane >> 5;
    // geometry chunk: f32 k-steps 0, 1 (channels 2h, 2h + 1), the rest zero
    auto geom = [&](int st) { return st == 0 ? gin.x : st == 1 ? gin.y : 0.f; };
    if constexpr (PRE) {
        load_tiles<T1>(h1, pre_row, h);  // engine.level_pre6: alpha-folded W_f f + beta
        mfma_pipe6<1, T1, T1>(wt, lane, sg, geom, h1, cin, s2, c2);
        (void)c1; (void)sf; (void)fin;
    } else {
        beta_tiles<T1>(eb + e1, lane, h1);
        mfma_pipe6<1, T1, T1>(wt, lane, sg, geom, h1, cin, sf, c1);
        mfma_pipe6<NF, T1, T1>(
            wt, lane, sf, [&](int st) { return (&fin[st >> 2].x)[st & 3]; }, h1, c1, s2, c2);
    }
    relu_tiles(h1);
    beta_tiles<T1>(eb + e2, lane, h2);
    mfma_pipe6<N1, T1, T3>(wt, lane, s2, [&](int st) { return h1[st >> 4][st & 15]; }, h2, c2, s3, c3);
    relu_tiles(h2);
    beta_tiles<T3>(eb + e3, lane, out);
    mfma_pipe6<N1, T3, NC>(wt, lane, s3, [&](int st) { return h2[st >> 4][st & 15]; }, out, c3, next, cout);
    relu_tiles(out);
}

// The weight pieces through the workgroup-shared LDS stream (mfma_chain.h Ring6) instead of one
// register stream per wave (r2, level 2: 187 -> 171 us, TD 86 -> 59 % busy), at 3 waves per SIMD
// (2: 192 us); level 3 on the ring (engine.SPLIT_L3 off: the checker form) at one wave per SIMD.
template <class K>
constexpr bool ring_on() { return true; }
template <class K>
constexpr int ring_wps() { return K::KN == 32 ? 3 : 1; }

// Level 2 on the ring: mlp1's x2 block batched over the workgroup.  x2 (the k-max row of the
// descriptor stack, layers.py:204-206) is the same for all 32 rows of a group, so the per-wave
// block (N3 chunks x TM1 tiles, 96 MFMAs) computes one column 32 times.  Batched: the 4 waves' x2
// rows go to LDS as the 4 columns of one B operand and the block's TM1 x N3 chunk-tiles are dealt
// out, one tile and half of the chunks per wave (24 MFMAs, 4 ring steps instead of 8); the
// partial columns meet in LDS and each wave adds its group's (lower-half + upper-half chunks) to
// mlp1 after the x1d block (r5: 158.6 -> 153.7 us).
template <class K, bool RING>
constexpr bool x2b_on() { return RING && K::KN == 32 && K::TM1 == 2 && WAVES == 4; }

// the batched x2 block (x2b_on): P (zeroed here) <- this wave's tile (w & 1) of W_x2 over
// chunks 4 (w >> 1) .. + 3, the B columns = the workgroup's x2 rows (sX[col][channel]).
// Step s's slot holds tiles {0, 1} x chunks {s, s + 4} (FragSeq tt = 2, cs = 4; the
// previous call prefetched step 0's); the last step prefetches nf's first chunk.
template <class K, class R>
__device__ __forceinline__ void x2_batched(R &ring, int lane, int w, const float *sX, f32x16 &P, FragSeq nf) {
    constexpr int N3 = K::N3, C3 = K::T3 * 32;
    static_assert(N3 == 8 && K::TM1 == 2, "x2 block shape");
    const FragSeq f{K::G_M1, 3 * N3, 2, 4};
    const int h = lane >> 5;
    const float *xr = sX + (lane & 3) * C3 + 4 * h;  // B column = lane % 4 (columns 4..31 repeat)
    P = zero16();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of this step landed
        __syncthreads();
        const int cur = ring.step & 1;
        if (s + 1 < 4)
            ring_fill<4>(ring, cur ^ 1, f, s + 1, lane);
        else
            ring_fill<K::TM1>(ring, cur ^ 1, nf, 0, lane);
        const int c = s + 4 * (w >> 1);  // chunk of the block: channels 16 c + 8 (i >> 2) + 4 h + (i & 3)
        float x[8];
        const float4 lo = *reinterpret_cast<const float4 *>(xr + 16 * c);
        const float4 hi = *reinterpret_cast<const float4 *>(xr + 16 * c + 8);
        x[0] = lo.x; x[1] = lo.y; x[2] = lo.z; x[3] = lo.w;
        x[4] = hi.x; x[5] = hi.y; x[6] = hi.z; x[7] = hi.w;
        u32x4 b[3], a[3];
        split8(x, b);
        const lds_cu32x4 *sp = ring.lds + cur * R::SLOT + w * 192 + lane;  // slot tile w = (w & 1, half w >> 1)
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = sp[p * 64];
        P = mma6(a, b, P);
        __builtin_amdgcn_sched_barrier(0);
        ++ring.step;
    }
}

template <class K, bool PRE, bool RING = false>
__global__ __launch_bounds__(256, RING ? ring_wps<K>() : K::WPS) void group_fused6_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc, const float *__restrict__ pre) {
    constexpr int CF = K::TF * 2, C3 = K::T3 * 32, CM2 = K::TM2 * 32;
    constexpr int T1 = K::T1, T3 = K::T3, TM1 = K::TM1, TM2 = K::TM2, N3 = K::N3, NM1 = K::NM1;
    constexpr int NE = K::TABLE - K::F_END;
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    constexpr int KN = K::KN, GPT = 32 / KN;
    const int NT = G / GPT;
    const bool writer = KN == 32 ? j == 31 : (j & 15) == 15;
    auto gsum_w = [&](float v) { return KN == 32 ? half_sum_hi(v) : row_sum16(v); };
    auto gsum_b = [&](float v) { return KN == 32 ? half_bcast(half_sum_hi(v), h) : row_sum16(v); };
    auto gmax_b = [&](float v) {
        return KN == 32 ? half_bcast(half_max_hi_nonneg(v), h) : row_max16_nonneg(v);
    };

    const FragSeq det_g{K::G_DG, 1}, desc_g{K::G_EG, 1};
    const FragSeq m1x2{K::G_M1, 3 * N3}, m1x1{K::G_M1 + N3, 3 * N3}, m1em{K::G_M1 + 2 * N3, 3 * N3};
    const FragSeq m2{K::G_M2, NM1};

    Carry carry;
    constexpr int RT_TILES = T3 > TM2 ? (T3 > T1 ? T3 : T1) : (TM2 > T1 ? TM2 : T1);
    __shared__ __attribute__((aligned(16))) u32x4 ring_lds[RING ? 2 * RT_TILES * 192 : 1];
    constexpr bool X2B = x2b_on<K, RING>();
    static_assert(!X2B || RT_TILES >= 4, "x2 steps: 4 chunk-tiles per slot");
    __shared__ __attribute__((aligned(16))) float sX[X2B ? WAVES * C3 : 1];       // x2 rows [wave][channel]
    __shared__ __attribute__((aligned(16))) float sZ[X2B ? WAVES * 4 * 32 : 1];   // partials [wave][column][32]
    Ring6<RT_TILES, WAVES> ring{reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table)),
                                (lds_u32x4 *)ring_lds, 0, w};
    if constexpr (RING) {
        ring_fill<T1>(ring, 0, det_g, 0, lane);
    } else {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int co = 0; co < T1; ++co) ld6(wt, det_g.base + co, lane, carry[co]);
    }
    // RING: every wave of the workgroup runs the same tiles count (a tile past the end
    // recomputes the last one: identical values, identical stores)
    const int tstride = gridDim.x * WAVES;
    for (int t0 = blockIdx.x * WAVES + (RING ? 0 : w); t0 < NT; t0 += tstride) {
        const int t = RING ? min(t0 + w, NT - 1) : t0;
        const int g = t * GPT + (KN == 32 ? 0 : j >> 4);  // this lane's group
        // opaque per-tile table pointer: keeps the loop-invariant weight loads in the loop
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wtp = reinterpret_cast<const gu32x4 *>(tba);
        ring.wt = wtp;  // (opaque per tile: the DMA addresses are not hoisted out of the loop)
        auto &&wt = [&]() -> decltype(auto) {
            if constexpr (RING) return (ring);
            else return wtp;
        }();
        const size_t row = (size_t)t * 32 + j;
        const float2 gin = *reinterpret_cast<const float2 *>(geom + row * 4 + 2 * h);
        const size_t src = (size_t)gidx[row];
        const float *fr = feats + src * CF + h * K::TF;
        const float *pr = PRE ? pre + src * (2 * K::T1 * 32) : nullptr;  // [det C1 | desc C1]
        Carry ca, cb;

        // ---- detector convs -> emb [C3][32 rows]
        f32x16 emb[T3];
        {
            float4 fin[K::TF / 4];
            if constexpr (!PRE) {
#pragma unroll
                for (int i = 0; i < K::TF / 4; ++i) fin[i] = *reinterpret_cast<const float4 *>(fr + 4 * i);
            }
            conv_stack6<K, TM1, PRE>(wt, eb, K::G_DG, K::G_DF, K::G_D2, K::G_D3, K::E_D1, K::E_D2, K::E_D3,
                                     lane, gin, fin, pr, emb, carry, m1em, ca);
        }

        // ---- attention: x1 = max_c emb (ReLU outputs: integer max), softmax over the group
        int mi = __float_as_int(emb[0][0]);
#pragma unroll
        for (int co = 0; co < T3; ++co)
#pragma unroll
            for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[co][q]));
        const float x1 = __int_as_float(max(mi, __shfl_xor(mi, 32)));
        const float mx = gmax_b(x1);
        const float e = expf(fsub_rn(x1, mx));
        const float a = e / gsum_b(e);

        const float *p = knn_xyz + row * 3;
        const float kx = gsum_w(fmul_rn(a, p[0]));
        const float ky = gsum_w(fmul_rn(a, p[1]));
        const float kz = gsum_w(fmul_rn(a, p[2]));
        if (writer && h == 0) {
            kp[(size_t)g * 3 + 0] = kx;
            kp[(size_t)g * 3 + 1] = ky;
            kp[(size_t)g * 3 + 2] = kz;
        }
#pragma unroll
        for (int co = 0; co < T3; ++co) {
            float v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = fmul_rn(emb[co][q], a);
            reduce_store<KN, Sum>(att_feat + (size_t)g * C3, co, v, lane);
        }

        // ---- mlp1 = W [x2 | x1d | emb * a] -> CM1, the emb * a part first
        f32x16 y1[TM1];
        beta_tiles<TM1>(eb + K::E_M1, lane, y1);
        mfma_pipe6<N3, TM1, T1>(wt, lane, m1em, [&](int st) { return fmul_rn(emb[st >> 4][st & 15], a); }, y1,
                                ca, desc_g, cb);

        // ---- descriptor convs -> x1d (the gathered rows are re-read: L2 hits)
        f32x16 x1d[T3];
        {
            uint64_t fra = reinterpret_cast<uint64_t>(fr);
            asm volatile("" : "+v"(fra));
            const float *fr2 = reinterpret_cast<const float *>(fra);
            float4 fin[K::TF / 4];
            if constexpr (!PRE) {
#pragma unroll
                for (int i = 0; i < K::TF / 4; ++i) fin[i] = *reinterpret_cast<const float4 *>(fr2 + 4 * i);
            }
            if constexpr (X2B)  // the next call is the batched x2 block: its first step's 4 chunk-tiles
                conv_stack6<K, 4, PRE>(wt, eb, K::G_EG, K::G_EF, K::G_E2, K::G_E3, K::E_E1, K::E_E2, K::E_E3,
                                       lane, gin, fin, PRE ? pr + K::T1 * 32 : nullptr, x1d, cb,
                                       FragSeq{K::G_M1, 3 * N3, 2, 4}, ca);
            else
                conv_stack6<K, TM1, PRE>(wt, eb, K::G_EG, K::G_EF, K::G_E2, K::G_E3, K::E_E1, K::E_E2, K::E_E3,
                                         lane, gin, fin, PRE ? pr + K::T1 * 32 : nullptr, x1d, cb, m1x2, ca);
        }

        if constexpr (X2B) {
            // x2 of this wave's group -> sX[w]; the block over the workgroup's 4 columns
#pragma unroll
            for (int ct = 0; ct < T3; ++ct) {
                float v[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q] = x1d[ct][q];
                reduce_store<32, MaxNN>(sX + w * C3, ct, v, lane);
            }
            f32x16 P;
            x2_batched<K>(ring, lane, w, sX, P, m1x1);
            if (j < 4) {  // column j's partial (tile w & 1, chunk half w >> 1)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<float4 *>(sZ + (w * 4 + j) * 32 + 8 * r + 4 * h) =
                        make_float4(P[4 * r], P[4 * r + 1], P[4 * r + 2], P[4 * r + 3]);
            }
            // (the next call's first barrier publishes sZ)
            mfma_pipe6<N3, TM1, TM2>(wt, lane, m1x1, [&](int st) { return x1d[st >> 4][st & 15]; }, y1, ca, m2,
                                     cb);
#pragma unroll
            for (int t = 0; t < TM1; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float4 za = *reinterpret_cast<const float4 *>(sZ + (t * 4 + w) * 32 + 8 * r + 4 * h);
                    const float4 zb = *reinterpret_cast<const float4 *>(sZ + ((t + 2) * 4 + w) * 32 + 8 * r + 4 * h);
                    y1[t][4 * r] = fadd_rn(y1[t][4 * r], fadd_rn(za.x, zb.x));
                    y1[t][4 * r + 1] = fadd_rn(y1[t][4 * r + 1], fadd_rn(za.y, zb.y));
                    y1[t][4 * r + 2] = fadd_rn(y1[t][4 * r + 2], fadd_rn(za.z, zb.z));
                    y1[t][4 * r + 3] = fadd_rn(y1[t][4 * r + 3], fadd_rn(za.w, zb.w));
                }
        } else {
#pragma unroll
        for (int ct = 0; ct < T3; ++ct) {
            float x2[16];
            if constexpr (KN == 32) {
#pragma unroll
                for (int q = 0; q < 16; ++q) x2[q] = x1d[ct][q];
                bfly32<MaxNN>(x2, lane);
                bcast32(x2, lane);
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) x2[q] = row_max16_nonneg(x1d[ct][q]);
            }
            const FragSeq cur{m1x2.base + ct * 2, m1x2.stride};
            const FragSeq nxt = ct + 1 < T3 ? FragSeq{m1x2.base + (ct + 1) * 2, m1x2.stride} : m1x1;
            if (ct & 1)
                mfma_pipe6<2, TM1, TM1>(wt, lane, cur, [&](int st) { return x2[st]; }, y1, cb, nxt, ca);
            else
                mfma_pipe6<2, TM1, TM1>(wt, lane, cur, [&](int st) { return x2[st]; }, y1, ca, nxt, cb);
        }
        static_assert(T3 % 2 == 0, "carry parity");
        mfma_pipe6<N3, TM1, TM2>(wt, lane, m1x1, [&](int st) { return x1d[st >> 4][st & 15]; }, y1, ca, m2, cb);
        }
        relu_tiles(y1);

        // ---- mlp2 + k-max -> descriptor; prefetches the next tile's first chunk
        f32x16 y2[TM2];
        beta_tiles<TM2>(eb + K::E_M2, lane, y2);
        mfma_pipe6<NM1, TM2, T1>(wt, lane, m2, [&](int st) { return y1[st >> 4][st & 15]; }, y2, cb, det_g,
                                 carry);
        relu_tiles(y2);
#pragma unroll
        for (int co = 0; co < TM2; ++co) {
            float v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = y2[co][q];
            reduce_store<KN, MaxNN>(desc + (size_t)g * CM2, co, v, lane);
        }
    }
}

template <class K>
int launch_group6(const float *table, const float *geom, const float *knn_xyz, const int32_t *gidx,
                  const float *feats, int G, float *kp, float *att_feat, float *desc, const float *pre,
                  void *stream) {
    if (reinterpret_cast<uintptr_t>(pre) & 15) return HREG_ERR_INVALID;
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(feats) & 15) ||
        (reinterpret_cast<uintptr_t>(geom) & 7) || (reinterpret_cast<uintptr_t>(att_feat) & 15) ||
        (reinterpret_cast<uintptr_t>(desc) & 15))
        return HREG_ERR_INVALID;
    if (G % (32 / K::KN)) return HREG_ERR_INVALID;  // whole 32-row tiles
    if (!G) return HREG_OK;
    const int NT = G / (32 / K::KN);
    int grid = (NT + WAVES - 1) / WAVES;
    const int cap = 256 * (ring_on<K>() ? ring_wps<K>() : K::WPS) * 4 / WAVES * 2;  // two rounds
    if (grid > cap) grid = cap;
    constexpr bool RING = ring_on<K>();
    if (RING && pre)
        hipLaunchKernelGGL((group_fused6_kernel<K, true, RING>), dim3(grid), dim3(256), 0, as_stream(stream),
                           table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    else if (pre)
        hipLaunchKernelGGL((group_fused6_kernel<K, true>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    else
        hipLaunchKernelGGL((group_fused6_kernel<K, false>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}


}  // namespace

extern "C" int hreg_group6_l2_table_floats(void) { return L2::TABLE; }
extern "C" int hreg_group6_l3_table_floats(void) { return L3::TABLE; }

extern "C" int hreg_group6_l2(const float *table, const float *geom, const float *knn_xyz, const int32_t *gidx,
                              const float *feats, int G, float *kp, float *att_feat, float *desc,
                              const float *pre, void *stream) {
    return launch_group6<L2>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}

extern "C" int hreg_group6_l3(const float *table, const float *geom, const float *knn_xyz, const int32_t *gidx,
                              const float *feats, int G, float *kp, float *att_feat, float *desc,
                              const float *pre, void *stream) {
    return launch_group6<L3>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}
