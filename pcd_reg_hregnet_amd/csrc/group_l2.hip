// group_l2.hip -- fused level-2 keypoint detector + descriptor for gfx950.
//
// One wave owns one keypoint group: its k = 32 neighbour rows = one 32-row MFMA
// column tile.  Every layer of
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
// At level 2 the folded weights are 258 KB -- more than the 160 KB of LDS -- so
// the A fragments stream from global memory (the table is L2-resident: every
// CU reads the same 258 KB).  fp32 MFMA needs 256 B of A per 64-cycle
// 32x32x2 op, i.e. 16 B/clk per CU at peak, well inside the L2->CU rate.
//
// The reference materialises [B, 68..384, 512, 32] tensors for this stage
// (~1 GB of HBM traffic per batch of 8 pairs); here only the group outputs
// (keypoint 3, attentive feature C3, descriptor CM2 floats) reach HBM.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
// global address space: loads through it are global_load (vmcnt-ordered), not flat
typedef __attribute__((address_space(1))) const float gfloat;

constexpr int WAVES = 4;
constexpr int KN = 32;  // neighbours per group (level 2)

template <int CF, int C1, int C3, int CM1, int CM2>
struct Cfg {
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

using L2 = Cfg<64, 64, 128, 64, 128>;

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
    return z;
}

__device__ __forceinline__ int chan(int co, int q, int h) {
    return co * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
}

// acc[co] += sum_{step < NSTEP} A(co, step) x B(step) on v_mfma_f32_32x32x2_f32, with
// the A fragments (wf + frag(co, step) * 64 + lane, L2-resident) software-
// pipelined one window of WIN k-steps ahead: the loads of window w+1 are issued
// before the MFMAs of window w, so the ~200-500-cycle L2 latency hides behind
// WIN * COUT_T * 64 cycles of MFMA work (sched_barrier keeps that order).
template <int NSTEP, int COUT_T, int WIN, class Frag, class BVal>
__device__ __forceinline__ void mfma_pipe(const gfloat *__restrict__ wf, int lane, Frag frag, BVal bval,
                                          f32x16 (&acc)[COUT_T]) {
    static_assert(NSTEP % WIN == 0, "window");
    constexpr int NW = NSTEP / WIN;
    // two fragment buffers used alternately (window index is compile-time: no copies)
    float buf[2][WIN][COUT_T];
#pragma unroll
    for (int s = 0; s < WIN; ++s)
#pragma unroll
        for (int co = 0; co < COUT_T; ++co) buf[0][s][co] = wf[frag(co, s) * 64 + lane];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (w + 1 < NW) {
#pragma unroll
            for (int s = 0; s < WIN; ++s)
#pragma unroll
                for (int co = 0; co < COUT_T; ++co)
                    buf[(w + 1) & 1][s][co] = wf[frag(co, (w + 1) * WIN + s) * 64 + lane];
        }
#pragma unroll
        for (int s = 0; s < WIN; ++s) {
            const float b = bval(w * WIN + s);
#pragma unroll
            for (int co = 0; co < COUT_T; ++co)
                acc[co] = __builtin_amdgcn_mfma_f32_32x32x2f32(buf[w & 1][s][co], b, acc[co], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int COUT_T>
constexpr int win_for() { return COUT_T >= 4 ? 4 : 8; }

// acc[co] += sum over input tiles ct of W-fragments x in[ct] (accumulator layout);
// fragment block of (co, ct) at wf + ((co * CIN_ALL + CT0 + ct) * 16 + q) * 64
template <int CIN_T, int COUT_T, int CIN_ALL, int CT0, bool SCALED>
__device__ __forceinline__ void mfma_accum(const gfloat *__restrict__ wf, int lane,
                                           const f32x16 (&in)[CIN_T], f32x16 (&acc)[COUT_T],
                                           float scale = 1.f) {
    mfma_pipe<CIN_T * 16, COUT_T, win_for<COUT_T>()>(
        wf, lane, [](int co, int st) { return (co * CIN_ALL + CT0 + (st >> 4)) * 16 + (st & 15); },
        [&](int st) {
            float b = in[st >> 4][st & 15];
            if (SCALED) b = fmul_rn(b, scale);
            return b;
        },
        acc);
}

template <int COUT_T>
__device__ __forceinline__ void epilogue(const float *ab, int lane, f32x16 (&acc)[COUT_T]) {
    const int h = lane >> 5;
    constexpr int C = COUT_T * 32;
#pragma unroll
    for (int co = 0; co < COUT_T; ++co)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = chan(co, q, h);
            acc[co][q] = fmaxf(fadd_rn(fmul_rn(acc[co][q], ab[c]), ab[C + c]), 0.f);
        }
}

// first conv over [geom (4) | gathered feature (CF)]
template <class K>
__device__ __forceinline__ void conv_in(const gfloat *__restrict__ tb, const float *eb, int fg, int ff, int e, int lane,
                                        float2 gin, const float4 (&fin)[K::TF / 4],
                                        f32x16 (&acc)[K::T1]) {
#pragma unroll
    for (int co = 0; co < K::T1; ++co) acc[co] = zero16();
    // geom part: 2 k-steps (channel 2h + s); feature part: TF k-steps (channel h*TF + s)
    mfma_pipe<2, K::T1, 2>(
        tb + fg, lane, [](int co, int st) { return co * 2 + st; },
        [&](int st) { return st == 0 ? gin.x : gin.y; }, acc);
    mfma_pipe<K::TF, K::T1, win_for<K::T1>()>(
        tb + ff, lane, [](int co, int st) { return co * K::TF + st; },
        [&](int st) { return (&fin[st >> 2].x)[st & 3]; }, acc);
    epilogue<K::T1>(eb + e, lane, acc);
}

template <class K>
__device__ __forceinline__ void conv_stack(const gfloat *__restrict__ tb, const float *eb, int fg, int ff, int f2, int f3,
                                           int e1, int e2, int e3, int lane, float2 gin,
                                           const float4 (&fin)[K::TF / 4], f32x16 (&out)[K::T3]) {
    f32x16 h1[K::T1], h2[K::T1];
    conv_in<K>(tb, eb, fg, ff, e1, lane, gin, fin, h1);
#pragma unroll
    for (int co = 0; co < K::T1; ++co) h2[co] = zero16();
    mfma_accum<K::T1, K::T1, K::T1, 0, false>(tb + f2, lane, h1, h2);
    epilogue<K::T1>(eb + e2, lane, h2);
#pragma unroll
    for (int co = 0; co < K::T3; ++co) out[co] = zero16();
    mfma_accum<K::T1, K::T3, K::T1, 0, false>(tb + f3, lane, h2, out);
    epilogue<K::T3>(eb + e3, lane, out);
}

// one channel tile of a per-group result reduced over the rows (valid in lanes 31 /
// 63): channels co*32 + 8r + 4h + {0..3} for registers q = 4r..4r+3 -> 4 float4 stores
__device__ __forceinline__ void store_tile(float *out, int co, const f32x16 &v, int j, int h) {
    if (j == 31) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            *reinterpret_cast<float4 *>(out + co * 32 + 8 * r + 4 * h) =
                make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
    }
}

template <class K>
__global__ __launch_bounds__(256, 2) void group_l2_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    const int32_t *__restrict__ gidx, const float *__restrict__ feats, int G, float *__restrict__ kp,
    float *__restrict__ att_feat, float *__restrict__ desc) {
    constexpr int CF = K::TF * 2, C3 = K::T3 * 32, CM2 = K::TM2 * 32;
    constexpr int NE = K::TABLE - K::F_END;
    // epilogue (alpha, beta) of every layer in LDS: LDS-indexed like the table so the
    // conv helpers take one base pointer (ep - F_END)
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int h = lane >> 5, j = lane & 31;
    for (int g = blockIdx.x * WAVES + w; g < G; g += gridDim.x * WAVES) {
        // the weight fragments are loop-invariant: an opaque per-group copy of the
        // table pointer keeps the compiler from hoisting all 1032 fragment loads
        // out of the group loop (and spilling them)
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gfloat *tb = reinterpret_cast<const gfloat *>(tba);
        const size_t row = (size_t)g * KN + j;
        const float2 gin = *reinterpret_cast<const float2 *>(geom + row * 4 + 2 * h);
        const float *fr = feats + (size_t)gidx[row] * CF + h * K::TF;
        float4 fin[K::TF / 4];
#pragma unroll
        for (int i = 0; i < K::TF / 4; ++i) fin[i] = *reinterpret_cast<const float4 *>(fr + 4 * i);

        // ---- detector convs -> emb [C3][32 rows]
        f32x16 emb[K::T3];
        conv_stack<K>(tb, eb, K::F_DG, K::F_DF, K::F_D2, K::F_D3, K::E_D1, K::E_D2, K::E_D3, lane, gin,
                      fin, emb);

        // ---- attention: x1 = max_c emb, a = softmax over the 32 rows (emb >= 0 after
        // ReLU: maxima on the integer bit patterns)
        int mi = __float_as_int(emb[0][0]);
#pragma unroll
        for (int co = 0; co < K::T3; ++co)
#pragma unroll
            for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[co][q]));
        const float x1 = __int_as_float(max(mi, __shfl_xor(mi, 32)));
        const float mx = half_bcast(half_max_hi_nonneg(x1), h);
        const float e = expf(fsub_rn(x1, mx));
        const float a = e / half_bcast(half_sum_hi(e), h);

        const float *p = knn_xyz + row * 3;
        const float kx = half_sum_hi(fmul_rn(a, p[0]));
        const float ky = half_sum_hi(fmul_rn(a, p[1]));
        const float kz = half_sum_hi(fmul_rn(a, p[2]));
        if (lane == 31) {
            kp[(size_t)g * 3 + 0] = kx;
            kp[(size_t)g * 3 + 1] = ky;
            kp[(size_t)g * 3 + 2] = kz;
        }
#pragma unroll
        for (int co = 0; co < K::T3; ++co) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = half_sum_hi(fmul_rn(emb[co][q], a));
            store_tile(att_feat + (size_t)g * C3, co, v, j, h);
        }

        // ---- descriptor convs -> x1d [C3][32]
        f32x16 x1d[K::T3];
        conv_stack<K>(tb, eb, K::F_EG, K::F_EF, K::F_E2, K::F_E3, K::E_E1, K::E_E2, K::E_E3, lane, gin,
                      fin, x1d);

        // ---- mlp1: cat[x2 = k-max of x1d (repeated over rows), x1d, emb * a] -> CM1
        f32x16 y1[K::TM1];
#pragma unroll
        for (int co = 0; co < K::TM1; ++co) y1[co] = zero16();
#pragma unroll
        for (int ct = 0; ct < K::T3; ++ct) {
            f32x16 x2[1];
#pragma unroll
            for (int q = 0; q < 16; ++q) x2[0][q] = half_bcast(half_max_hi_nonneg(x1d[ct][q]), h);
            mfma_accum<1, K::TM1, 3 * K::T3, 0, false>(tb + K::F_M1 + ct * 16 * 64, lane, x2, y1);
        }
        mfma_accum<K::T3, K::TM1, 3 * K::T3, K::T3, false>(tb + K::F_M1, lane, x1d, y1);
        mfma_accum<K::T3, K::TM1, 3 * K::T3, 2 * K::T3, true>(tb + K::F_M1, lane, emb, y1, a);
        epilogue<K::TM1>(eb + K::E_M1, lane, y1);

        // ---- mlp2: CM1 -> CM2, then max over the rows
        f32x16 y2[K::TM2];
#pragma unroll
        for (int co = 0; co < K::TM2; ++co) y2[co] = zero16();
        mfma_accum<K::TM1, K::TM2, K::TM1, 0, false>(tb + K::F_M2, lane, y1, y2);
        epilogue<K::TM2>(eb + K::E_M2, lane, y2);
#pragma unroll
        for (int co = 0; co < K::TM2; ++co) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = half_max_hi_nonneg(y2[co][q]);
            store_tile(desc + (size_t)g * CM2, co, v, j, h);
        }
    }
}

}  // namespace

extern "C" int hreg_group_l2_table_floats(void) { return L2::TABLE; }

extern "C" int hreg_group_l2(const float *table, const float *geom, const float *knn_xyz,
                             const int32_t *gidx, const float *feats, int G, float *kp,
                             float *att_feat, float *desc, void *stream) {
    if (!table || !geom || !knn_xyz || !gidx || !feats || !kp || !att_feat || !desc || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(feats) & 15) || (reinterpret_cast<uintptr_t>(geom) & 7))
        return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    int grid = (G + WAVES - 1) / WAVES;
    if (grid > 2048) grid = 2048;
    hipLaunchKernelGGL(group_l2_kernel<L2>, dim3(grid), dim3(256), 0, as_stream(stream), table,
                       geom, knn_xyz, gidx, feats, G, kp, att_feat, desc);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
