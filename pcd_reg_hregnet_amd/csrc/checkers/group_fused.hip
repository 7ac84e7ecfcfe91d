// group_fused.hip -- fused level-2 / level-3 keypoint detector + descriptor for gfx950.
//
// One wave owns one 32-row MFMA column tile: one keypoint group of k = 32
// neighbour rows (level 2) or two groups of k = 16 (level 3).  Every layer of
//   KeypointDetector.convs [geom 4 + feat CF] -> C1 -> C1 -> C3  (layers.py:115-121, 150)
//   attention: max_c -> softmax_k -> keypoint / attentive feature (layers.py:151-159)
//   DescExtractor.convs   [geom 4 + feat CF] -> C1 -> C1 -> C3  (layers.py:183-189, 201)
//   k-max, cat[x2, x1, att_map] -> mlp1 3*C3 -> CM1 -> mlp2 CM2 -> k-max (layers.py:202-208)
// runs on v_mfma_f32_32x32x2_f32 with the activations in the MFMA accumulators
// (accumulator-as-operand chaining, as group_l1.hip).  The input rows are the
// level-1 attentive features gathered through the kNN index: lane half h of
// row j holds channels [h*CF/2, (h+1)*CF/2) of its neighbour's feature row,
// loaded as float4s, and feeds them as the B operand of k-steps 0..CF/2-1.
//
// The folded weights (258 KB at level 2, 1 MB at level 3) exceed the 160 KB of
// LDS, so the A fragments stream from global memory (the table is L2-resident:
// every CU reads the same table).  fp32 MFMA needs 256 B of A per 64-cycle
// 32x32x2 op, i.e. 16 B/clk per CU at peak, well inside the L2->CU rate.
//
// The reference materialises [B, 68..384, 512, 32] tensors for this stage
// (~1 GB of HBM traffic per batch of 8 pairs); here only the group outputs
// (keypoint 3, attentive feature C3, descriptor CM2 floats) reach HBM.
#include "../mfma_chain.h"

namespace {

using namespace hreg_chain;

constexpr int WAVES = 4;

// KN_ neighbours per group (32: level 2, 16: level 3), CF gathered feature channels,
// conv widths C1 / C3, mlp widths CM1 / CM2, WPS waves per SIMD (register budget)
template <int KN_, int CF, int C1, int C3, int CM1, int CM2, int WPS_>
struct Cfg {
    static constexpr int KN = KN_, WPS = WPS_;
    static constexpr int TF = CF / 2;  // feature k-steps (one channel per lane half)
    static constexpr int T1 = C1 / 32, T3 = C3 / 32, TM1 = CM1 / 32, TM2 = CM2 / 32;
    // fragment table (floats): [co][k-step][lane] blocks, see engine.l2_table
    static constexpr int F_DG = 0;                         // det conv1, geom part [T1][2][64]
    static constexpr int F_DF = F_DG + T1 * 2 * 64;        // det conv1, feat part [T1][TF][64]
    static constexpr int F_D2 = F_DF + T1 * TF * 64;       // det conv2 [T1][T1][16][64]
    static constexpr int F_D3 = F_D2 + T1 * T1 * 16 * 64;  // det conv3 [T3][T1][16][64]
    static constexpr int F_EG = F_D3 + T3 * T1 * 16 * 64;
    static constexpr int F_EF = F_EG + T1 * 2 * 64;
    static constexpr int F_E2 = F_EF + T1 * TF * 64;
    static constexpr int F_E3 = F_E2 + T1 * T1 * 16 * 64;
    static constexpr int F_M1 = F_E3 + T3 * T1 * 16 * 64;  // mlp1 [TM1][3*T3][16][64]
    static constexpr int F_M2 = F_M1 + TM1 * 3 * T3 * 16 * 64;  // mlp2 [TM2][TM1][16][64]
    static constexpr int F_END = F_M2 + TM2 * TM1 * 16 * 64;
    // epilogue (alpha[C], beta[C]) per layer
    static constexpr int E_D1 = F_END, E_D2 = E_D1 + 2 * C1, E_D3 = E_D2 + 2 * C1,
                         E_E1 = E_D3 + 2 * C3, E_E2 = E_E1 + 2 * C1, E_E3 = E_E2 + 2 * C1,
                         E_M1 = E_E3 + 2 * C3, E_M2 = E_M1 + 2 * CM1, TABLE = E_M2 + 2 * CM2;
};

using L2 = Cfg<32, 64, 64, 128, 64, 128, 2>;
using L3 = Cfg<16, 128, 128, 256, 128, 256, 1>;

// conv stack [geom 4 | gathered feature CF] -> C1 -> C1 -> C3 (+ BN/ReLU epilogues).
// Offsets (in floats) of the stack's four fragment blocks and three epilogues;
// NC/NWN/next describe the call that follows the stack (for its prefetch).
// PRE: the feature part of the first layer comes precomputed per source point
// (pre_row = W_f f of this row's neighbour, C1 channels, hreg_gemm over the feature
// rows) and initialises the accumulators; only the 2 geometry k-steps run here.
template <class K, int NC, int NWN, bool PRE>
__device__ __forceinline__ void conv_stack(const gfloat *__restrict__ tb, const float *eb, int fg, int ff,
                                           int f2, int f3, int e1, int e2, int e3, int lane, float2 gin,
                                           const float4 (&fin)[K::TF / 4], const float *pre_row,
                                           f32x16 (&out)[K::T3], const float (&cin)[CARRY], FragSeq next,
                                           float (&cout)[CARRY]) {
    constexpr int T1 = K::T1, T3 = K::T3, TF = K::TF;
    const FragSeq sg{fg / 64, 2}, sf{ff / 64, TF}, s2{f2 / 64, T1 * 16}, s3{f3 / 64, T1 * 16};
    f32x16 h1[T1], h2[T1];
    float c1[CARRY], c2[CARRY], c3[CARRY];
    const int h = lane >> 5;
    if constexpr (PRE) {
        load_tiles<T1>(h1, pre_row, h);
        mfma_pipe<2, T1, T1, first_win<T1 * 16, T1>()>(
            tb, lane, sg, [&](int st) { return st == 0 ? gin.x : gin.y; }, h1, cin, s2, c2);
        (void)c1; (void)sf; (void)fin;
    } else {
        zero_tiles(h1);
        // geom part: 2 k-steps (channel 2h + s); feature part: TF k-steps (channel h*TF + s)
        mfma_pipe<2, T1, T1, first_win<TF, T1>()>(
            tb, lane, sg, [&](int st) { return st == 0 ? gin.x : gin.y; }, h1, cin, sf, c1);
        mfma_pipe<TF, T1, T1, first_win<T1 * 16, T1>()>(
            tb, lane, sf, [&](int st) { return (&fin[st >> 2].x)[st & 3]; }, h1, c1, s2, c2);
    }
    epilogue<T1>(eb + e1, lane, h1);
    zero_tiles(h2);
    mfma_pipe<T1 * 16, T1, T3, first_win<T1 * 16, T3>()>(
        tb, lane, s2, [&](int st) { return h1[st >> 4][st & 15]; }, h2, c2, s3, c3);
    epilogue<T1>(eb + e2, lane, h2);
    zero_tiles(out);
    mfma_pipe<T1 * 16, T3, NC, NWN>(
        tb, lane, s3, [&](int st) { return h2[st >> 4][st & 15]; }, out, c3, next, cout);
    epilogue<T3>(eb + e3, lane, out);
}

// gathered feature rows (a non-temporal variant that was meant to keep the weight table in L2
// measured no faster and was removed)
__device__ __forceinline__ float4 ld_rows(const float *p) { return *reinterpret_cast<const float4 *>(p); }

template <class K, bool PRE>
__global__ __launch_bounds__(256, K::WPS) void group_fused_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc, const float *__restrict__ pre) {
    constexpr int CF = K::TF * 2, C3 = K::T3 * 32, CM2 = K::TM2 * 32;
    constexpr int T1 = K::T1, T3 = K::T3, TM1 = K::TM1, TM2 = K::TM2;
    constexpr int NE = K::TABLE - K::F_END;
    // epilogue (alpha, beta) of every layer in LDS: LDS-indexed like the table so the
    // conv helpers take one base pointer (ep - F_END)
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    constexpr int KN = K::KN, GPT = 32 / KN;  // groups per 32-row tile
    const int NT = G / GPT;
    // per-group reductions over the KN rows of a tile: wave halves (KN = 32) or
    // 16-lane DPP rows (KN = 16); *_b: result in every lane, *_w: in the writer lanes
    const bool writer = KN == 32 ? j == 31 : (j & 15) == 15;
    auto gsum_w = [&](float v) { return KN == 32 ? half_sum_hi(v) : row_sum16(v); };
    auto gsum_b = [&](float v) { return KN == 32 ? half_bcast(half_sum_hi(v), h) : row_sum16(v); };
    auto gmax_w = [&](float v) { return KN == 32 ? half_max_hi_nonneg(v) : row_max16_nonneg(v); };
    auto gmax_b = [&](float v) {
        return KN == 32 ? half_bcast(half_max_hi_nonneg(v), h) : row_max16_nonneg(v);
    };

    // the group's call sequence (fragment blocks, see Cfg)
    const FragSeq det_g{K::F_DG / 64, 2}, desc_g{K::F_EG / 64, 2};
    const FragSeq m1x2{K::F_M1 / 64, 3 * T3 * 16};            // + ct * 16
    const FragSeq m1x1{K::F_M1 / 64 + T3 * 16, 3 * T3 * 16};
    const FragSeq m1em{K::F_M1 / 64 + 2 * T3 * 16, 3 * T3 * 16};
    const FragSeq m2{K::F_M2 / 64, TM1 * 16};
    constexpr int WM1 = win_for<TM1>(), WM2 = win_for<TM2>();

    float carry[CARRY];
    {
        const gfloat *tb = reinterpret_cast<const gfloat *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int co = 0; co < T1; ++co) {
            float v[2];
            ldgroup<2>(tb, det_g.base + co * 2, lane, v);
            carry[co] = v[0];
            carry[T1 + co] = v[1];
        }
    }
    for (int t = blockIdx.x * WAVES + w; t < NT; t += gridDim.x * WAVES) {
        const int g = t * GPT + (KN == 32 ? 0 : j >> 4);  // this lane's group
        // the weight fragments are loop-invariant: an opaque per-group copy of the
        // table pointer keeps the compiler from hoisting all 1032 fragment loads
        // out of the group loop (and spilling them)
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gfloat *tb = reinterpret_cast<const gfloat *>(tba);
        const size_t row = (size_t)t * 32 + j;
        const float2 gin = *reinterpret_cast<const float2 *>(geom + row * 4 + 2 * h);
        const size_t src = (size_t)gidx[row];
        const float *fr = feats + src * CF + h * K::TF;
        const float *pr = PRE ? pre + src * (2 * K::T1 * 32) : nullptr;  // [det C1 | desc C1]
        float ca[CARRY], cb[CARRY];

        // ---- detector convs -> emb [C3][32 rows]
        f32x16 emb[T3];
        {
            float4 fin[K::TF / 4];
            if constexpr (!PRE) {
#pragma unroll
                for (int i = 0; i < K::TF / 4; ++i) fin[i] = ld_rows(fr + 4 * i);
            }
            conv_stack<K, TM1, WM1, PRE>(tb, eb, K::F_DG, K::F_DF, K::F_D2, K::F_D3, K::E_D1, K::E_D2,
                                         K::E_D3, lane, gin, fin, pr, emb, carry, m1em, ca);
        }

        // ---- attention: x1 = max_c emb, a = softmax over the group's rows (emb >= 0
        // after ReLU: maxima on the integer bit patterns)
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
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                v[q] = gsum_w(fmul_rn(emb[co][q], a));
            store_tile(att_feat + (size_t)g * C3, co, v, writer, h);
        }

        // ---- mlp1 = W [x2 (k-max of x1d, repeated) | x1d | emb * a] -> CM1: the
        // emb * a part first, so emb is dead before the descriptor convs run
        f32x16 y1[TM1];
        zero_tiles(y1);
        mfma_pipe<T3 * 16, TM1, T1, 2>(
            tb, lane, m1em, [&](int st) { return fmul_rn(emb[st >> 4][st & 15], a); }, y1, ca, desc_g, cb);

        // ---- descriptor convs -> x1d [C3][32]; the gathered rows are re-read (L2 hits)
        // rather than kept live across the detector
        f32x16 x1d[T3];
        {
            uint64_t fra = reinterpret_cast<uint64_t>(fr);
            asm volatile("" : "+v"(fra));
            const float *fr2 = reinterpret_cast<const float *>(fra);
            float4 fin[K::TF / 4];
            if constexpr (!PRE) {
#pragma unroll
                for (int i = 0; i < K::TF / 4; ++i) fin[i] = ld_rows(fr2 + 4 * i);
            }
            conv_stack<K, TM1, WM1, PRE>(tb, eb, K::F_EG, K::F_EF, K::F_E2, K::F_E3, K::E_E1, K::E_E2,
                                         K::E_E3, lane, gin, fin, PRE ? pr + K::T1 * 32 : nullptr, x1d,
                                         cb, m1x2, ca);
        }

#pragma unroll
        for (int ct = 0; ct < T3; ++ct) {
            f32x16 x2[1];
#pragma unroll
            for (int q = 0; q < 16; ++q) x2[0][q] = gmax_b(x1d[ct][q]);
            const FragSeq cur{m1x2.base + ct * 16, m1x2.stride};
            const FragSeq nxt = ct + 1 < T3 ? FragSeq{m1x2.base + (ct + 1) * 16, m1x2.stride} : m1x1;
            // ct even: ca -> cb, odd: cb -> ca
            if (ct & 1)
                mfma_pipe<16, TM1, TM1, WM1>(tb, lane, cur, [&](int st) { return x2[0][st]; }, y1, cb,
                                             nxt, ca);
            else
                mfma_pipe<16, TM1, TM1, WM1>(tb, lane, cur, [&](int st) { return x2[0][st]; }, y1, ca,
                                             nxt, cb);
        }
        static_assert(T3 % 2 == 0, "carry parity");
        mfma_pipe<T3 * 16, TM1, TM2, WM2>(tb, lane, m1x1, [&](int st) { return x1d[st >> 4][st & 15]; },
                                          y1, ca, m2, cb);
        epilogue<TM1>(eb + K::E_M1, lane, y1);

        // ---- mlp2: CM1 -> CM2, then max over the rows; prefetches the next group's
        // first window into carry
        f32x16 y2[TM2];
        zero_tiles(y2);
        mfma_pipe<TM1 * 16, TM2, T1, 2>(tb, lane, m2, [&](int st) { return y1[st >> 4][st & 15]; },
                                        y2, cb, det_g, carry);
        epilogue<TM2>(eb + K::E_M2, lane, y2);
#pragma unroll
        for (int co = 0; co < TM2; ++co) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = gmax_w(y2[co][q]);
            store_tile(desc + (size_t)g * CM2, co, v, writer, h);
        }
    }
}

template <class K>
int launch_group(const float *table, const float *geom, const float *knn_xyz, const int32_t *gidx,
                 const float *feats, int G, float *kp, float *att_feat, float *desc, const float *pre,
                 void *stream) {
    if (reinterpret_cast<uintptr_t>(pre) & 15) return HREG_ERR_INVALID;
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(feats) & 15) || (reinterpret_cast<uintptr_t>(geom) & 7) ||
        (reinterpret_cast<uintptr_t>(att_feat) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15))
        return HREG_ERR_INVALID;
    if (G % (32 / K::KN)) return HREG_ERR_INVALID;  // whole 32-row tiles
    if (!G) return HREG_OK;
    const int NT = G / (32 / K::KN);
    int grid = (NT + WAVES - 1) / WAVES;
    const int cap = 256 * K::WPS * 4 / WAVES * 2;  // two rounds of resident blocks
    if (grid > cap) grid = cap;
    if (pre)
        hipLaunchKernelGGL((group_fused_kernel<K, true>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    else
        hipLaunchKernelGGL((group_fused_kernel<K, false>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_group_l2_table_floats(void) { return L2::TABLE; }
extern "C" int hreg_group_l3_table_floats(void) { return L3::TABLE; }

extern "C" int hreg_group_l2(const float *table, const float *geom, const float *knn_xyz,
                             const int32_t *gidx, const float *feats, int G, float *kp,
                             float *att_feat, float *desc, const float *pre, void *stream) {
    return launch_group<L2>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}

extern "C" int hreg_group_l3(const float *table, const float *geom, const float *knn_xyz,
                             const int32_t *gidx, const float *feats, int G, float *kp,
                             float *att_feat, float *desc, const float *pre, void *stream) {
    return launch_group<L3>(table, geom, knn_xyz, gidx, feats, G, kp, att_feat, desc, pre, stream);
}
