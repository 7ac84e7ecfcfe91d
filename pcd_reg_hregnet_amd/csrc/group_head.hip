// group_head.hip -- fused FineReg correspondence head for gfx950.
//
// FineReg.forward (layers.py:433-454) per keypoint i of the source and its k = 8
// nearest destination points n_ij: the feature row
//   [p - q (3), |p - q| (1), q (3), p (3), w_src (1), w_dst (1), 0 (4) | f_src C | f_dst[n_ij] C]
// (columns of convs_1 permuted to this order on the host, engine._perm_fine, and
// zero-padded 12 -> 16) runs through convs_1 (3 x [1x1 Conv2d + BN + ReLU],
// 2C+16 -> N1 -> N1 -> N1), then the attention of layers.py:446-451: a = softmax
// over the 8 rows of max over channels, corres = sum_j a_j p_j, attentive feature
// = sum_j a_j f_j (N1 channels) -- all in one kernel.  One wave owns a 32-row MFMA
// tile = 4 keypoints; the activations stay in the MFMA accumulators (as in
// group_fused.hip) and the reductions over a keypoint's 8 rows are 3 DPP steps.
// The first layer's B operand streams from the three row sources (one window of
// k-steps ahead, like the A fragments), so the 2C+16-wide rows are never held.
//
// nbr_head_kernel is CoarseReg's neighbour branch (layers.py:315-337): rows
// [desc[nbr_ij] C | p_ij - q_i, |p_ij - q_i|] through convs_2 (C+4 -> 256 -> 256 -> 256),
// attention over the 8 xyz neighbours, output sum_j a_j desc[nbr_ij] (C channels).
#include "mfma_chain.h"

namespace {

using namespace hreg_chain;

constexpr int WAVES = 4;
constexpr int KH = 8;  // neighbours per keypoint (models.py:71-73)

template <int C_, int N1_, int WPS_>
struct HeadCfg {
    static constexpr int C = C_, N1 = N1_, WPS = WPS_;
    static constexpr int T1 = N1 / 32, TA = C / 2;  // conv tiles; k-steps per descriptor segment
    // fragment table (floats), engine.fine_head_table
    static constexpr int F_S = 0;                         // small features [T1][8][64]
    static constexpr int F_A = F_S + T1 * 8 * 64;          // source descriptor [T1][TA][64]
    static constexpr int F_B = F_A + T1 * TA * 64;         // destination descriptor [T1][TA][64]
    static constexpr int F_2 = F_B + T1 * TA * 64;         // conv 2 [T1][T1][16][64]
    static constexpr int F_3 = F_2 + T1 * T1 * 16 * 64;    // conv 3
    static constexpr int F_END = F_3 + T1 * T1 * 16 * 64;
    static constexpr int E_1 = F_END, E_2 = E_1 + 2 * N1, E_3 = E_2 + 2 * N1, TABLE = E_3 + 2 * N1;
};

using Fine1 = HeadCfg<64, 128, 2>;
using Fine2 = HeadCfg<128, 256, 1>;

// acc[co] += sum_st A(co, st) x rowp[st]: the B operand read from this lane's row
// (GS-float vector loads) in the same one-window-ahead pipeline as the A fragments.
template <int NSTEP, int COUT_T, int NCOUT, int NWIN>
__device__ __forceinline__ void mfma_pipe_rows(const gfloat *__restrict__ wf, int lane, FragSeq f,
                                               const float *__restrict__ rowp, f32x16 (&acc)[COUT_T],
                                               const float (&cin)[CARRY], FragSeq nf,
                                               float (&cout)[CARRY]) {
    constexpr int WIN = first_win<NSTEP, COUT_T>();
    constexpr int GS = WIN < 4 ? WIN : 4, NGS = NWIN < 4 ? NWIN : 4;
    static_assert(NSTEP % WIN == 0 && WIN % GS == 0 && NWIN % NGS == 0, "window");
    constexpr int NW = NSTEP / WIN;
    float buf[2][WIN][COUT_T], bb[2][WIN];
    auto load_b = [&](int slot, int s0w) {
#pragma unroll
        for (int s0 = 0; s0 < WIN; s0 += GS) {
            if constexpr (GS == 4) {
                const float4 t = *reinterpret_cast<const float4 *>(rowp + s0w + s0);
                bb[slot][s0] = t.x; bb[slot][s0 + 1] = t.y; bb[slot][s0 + 2] = t.z; bb[slot][s0 + 3] = t.w;
            } else {
                const float2 t = *reinterpret_cast<const float2 *>(rowp + s0w + s0);
                bb[slot][s0] = t.x; bb[slot][s0 + 1] = t.y;
            }
        }
    };
    load_b(0, 0);
#pragma unroll
    for (int s = 0; s < WIN; ++s)
#pragma unroll
        for (int co = 0; co < COUT_T; ++co) buf[0][s][co] = cin[s * COUT_T + co];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (w + 1 < NW) {
            load_b((w + 1) & 1, (w + 1) * WIN);
#pragma unroll
            for (int s0 = 0; s0 < WIN; s0 += GS)
#pragma unroll
                for (int co = 0; co < COUT_T; ++co) {
                    float v[GS];
                    ldgroup<GS>(wf, f.base + co * f.stride + (w + 1) * WIN + s0, lane, v);
#pragma unroll
                    for (int i = 0; i < GS; ++i) buf[(w + 1) & 1][s0 + i][co] = v[i];
                }
        } else {
#pragma unroll
            for (int s0 = 0; s0 < NWIN; s0 += NGS)
#pragma unroll
                for (int co = 0; co < NCOUT; ++co) {
                    float v[NGS];
                    ldgroup<NGS>(wf, nf.base + co * nf.stride + s0, lane, v);
#pragma unroll
                    for (int i = 0; i < NGS; ++i) cout[(s0 + i) * NCOUT + co] = v[i];
                }
        }
        __builtin_amdgcn_sched_barrier(0);  // loads stay at the top of the window
#pragma unroll
        for (int s = 0; s < WIN; ++s)
#pragma unroll
            for (int co = 0; co < COUT_T; ++co)
                acc[co] = __builtin_amdgcn_mfma_f32_32x32x2f32(buf[w & 1][s][co], bb[w & 1][s], acc[co], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}


// FineReg attention over the keypoint's 8 rows (f >= 0 after ReLU, layers.py:446-451):
// corres = sum_j a_j p_j, attentive feature sum_j a_j f_j
template <int T1>
__device__ __forceinline__ void fine_attend(const f32x16 (&f)[T1], int lane, int row,
                                            const float *__restrict__ knn_xyz, float *__restrict__ corres,
                                            float *__restrict__ att) {
    const int h = lane >> 5, j = lane & 31, g = row / KH;
    int mi = __float_as_int(f[0][0]);
#pragma unroll
    for (int co = 0; co < T1; ++co)
#pragma unroll
        for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(f[co][q]));
    const float x1 = __int_as_float(max(mi, __shfl_xor(mi, 32)));
    const float e = expf(fsub_rn(x1, grp8_max_nonneg(x1)));
    const float a = e / grp8_sum(e);
    const bool writer = (j & 7) == 7;
    const float *p = knn_xyz + (size_t)row * 3;
    const float cx = grp8_sum(fmul_rn(a, p[0]));
    const float cy = grp8_sum(fmul_rn(a, p[1]));
    const float cz = grp8_sum(fmul_rn(a, p[2]));
    if (writer && h == 0) {
        corres[(size_t)g * 3 + 0] = cx;
        corres[(size_t)g * 3 + 1] = cy;
        corres[(size_t)g * 3 + 2] = cz;
    }
#pragma unroll
    for (int co = 0; co < T1; ++co) {
        f32x16 v;
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = grp8_sum(fmul_rn(f[co][q], a));
        store_tile(att + (size_t)g * (T1 * 32), co, v, writer, h);
    }
}

// CoarseReg neighbour-branch attention over the 8 rows (f >= 0 after ReLU), applied to
// the input descriptors (layers.py:326-337): out = sum_j a_j desc[nbr_ij]
template <int T1, int C>
__device__ __forceinline__ void nbr_attend(const f32x16 (&f)[T1], int lane, int row,
                                           const float *__restrict__ drow, float *__restrict__ out) {
    constexpr int TA = C / 2;
    const int h = lane >> 5, j = lane & 31, g = row / KH;
    int mi = __float_as_int(f[0][0]);
#pragma unroll
    for (int co = 0; co < T1; ++co)
#pragma unroll
        for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(f[co][q]));
    const float x1 = __int_as_float(max(mi, __shfl_xor(mi, 32)));
    const float e = expf(fsub_rn(x1, grp8_max_nonneg(x1)));
    const float a = e / grp8_sum(e);
    const bool writer = (j & 7) == 7;
    // lane half h owns channels [h*C/2, (h+1)*C/2) of its row's descriptor
#pragma unroll 4
    for (int c4i = 0; c4i < TA / 4; ++c4i) {
        const float4 v = *reinterpret_cast<const float4 *>(drow + h * TA + c4i * 4);
        const float4 r = make_float4(grp8_sum(fmul_rn(v.x, a)), grp8_sum(fmul_rn(v.y, a)),
                                     grp8_sum(fmul_rn(v.z, a)), grp8_sum(fmul_rn(v.w, a)));
        if (writer) *reinterpret_cast<float4 *>(out + (size_t)g * C + h * TA + c4i * 4) = r;
    }
}

template <class K, bool PRE>
__global__ __launch_bounds__(256, K::WPS) void fine_head_kernel(
    const float *__restrict__ table, const float *__restrict__ small, const float *__restrict__ src_desc,
    const float *__restrict__ dst_desc, const int32_t *__restrict__ gidx,
    const float *__restrict__ knn_xyz, int G, float *__restrict__ corres, float *__restrict__ att,
    const float *__restrict__ pre_src, const float *__restrict__ pre_dst) {
    constexpr int C = K::C, N1 = K::N1, T1 = K::T1, TA = K::TA;
    constexpr int NE = K::TABLE - K::F_END;
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G * KH / 32;
    constexpr int WT = win_for<T1>();
    const FragSeq fs{K::F_S / 64, 8}, fa{K::F_A / 64, TA}, fb{K::F_B / 64, TA};
    const FragSeq f2{K::F_2 / 64, T1 * 16}, f3{K::F_3 / 64, T1 * 16};

    float carry[CARRY];
    {
        const gfloat *tb = reinterpret_cast<const gfloat *>(reinterpret_cast<uint64_t>(table));
        constexpr int GS0 = first_win<8, T1>() < 4 ? first_win<8, T1>() : 4;
#pragma unroll
        for (int s0 = 0; s0 < first_win<8, T1>(); s0 += GS0)
#pragma unroll
            for (int co = 0; co < T1; ++co) {
                float v[GS0];
                ldgroup<GS0>(tb, fs.base + co * fs.stride + s0, lane, v);
#pragma unroll
                for (int i = 0; i < GS0; ++i) carry[(s0 + i) * T1 + co] = v[i];
            }
    }
    for (int t = blockIdx.x * WAVES + w; t < NT; t += gridDim.x * WAVES) {
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gfloat *tb = reinterpret_cast<const gfloat *>(tba);
        const int row = t * 32 + j;
        const int g = row / KH;
        float c1[CARRY], c2[CARRY], c3[CARRY], c4[CARRY];

        f32x16 h1[T1], h2[T1];
        if constexpr (PRE) {
            init_from_rows<N1, T1>(h1, pre_src + (size_t)g * N1, pre_dst + (size_t)gidx[row] * N1, h);
            mfma_pipe_rows<8, T1, T1, WT>(tb, lane, fs, small + (size_t)row * 16 + h * 8, h1, carry, f2, c3);
            (void)c1; (void)c2;
        } else {
            zero_tiles(h1);
            mfma_pipe_rows<8, T1, T1, first_win<TA, T1>()>(tb, lane, fs, small + (size_t)row * 16 + h * 8,
                                                           h1, carry, fa, c1);
            mfma_pipe_rows<TA, T1, T1, first_win<TA, T1>()>(tb, lane, fa, src_desc + (size_t)g * C + h * TA,
                                                            h1, c1, fb, c2);
            mfma_pipe_rows<TA, T1, T1, WT>(tb, lane, fb, dst_desc + (size_t)gidx[row] * C + h * TA, h1, c2,
                                           f2, c3);
        }
        epilogue<T1>(eb + K::E_1, lane, h1);
        zero_tiles(h2);
        mfma_pipe<T1 * 16, T1, T1, WT>(tb, lane, f2, [&](int st) { return h1[st >> 4][st & 15]; }, h2, c3,
                                       f3, c4);
        epilogue<T1>(eb + K::E_2, lane, h2);
        f32x16 f[T1];
        zero_tiles(f);
        mfma_pipe<T1 * 16, T1, T1, first_win<8, T1>()>(
            tb, lane, f3, [&](int st) { return h2[st >> 4][st & 15]; }, f, c4, fs, carry);
        epilogue<T1>(eb + K::E_3, lane, f);
        fine_attend<T1>(f, lane, row, knn_xyz, corres, att);
    }
}

template <int C_>
struct NbrCfg {
    static constexpr int C = C_, N1 = 256, WPS = 1;
    static constexpr int T1 = N1 / 32, TA = C / 2;
    static constexpr int F_D = 0;                          // descriptor part [T1][TA][64]
    static constexpr int F_G = F_D + T1 * TA * 64;          // geometry part [T1][2][64]
    static constexpr int F_2 = F_G + T1 * 2 * 64;
    static constexpr int F_3 = F_2 + T1 * T1 * 16 * 64;
    static constexpr int F_END = F_3 + T1 * T1 * 16 * 64;
    static constexpr int E_1 = F_END, E_2 = E_1 + 2 * N1, E_3 = E_2 + 2 * N1, TABLE = E_3 + 2 * N1;
};
using Nbr = NbrCfg<256>;

// PRE: pre[n] = W_d desc[n] ([*][256], hreg_gemm) initialises the accumulators from
// the row's gathered neighbour; only the 4 geometry columns run on the MFMA here.
template <class K, bool PRE>
__global__ __launch_bounds__(256, K::WPS) void nbr_head_kernel(
    const float *__restrict__ table, const float *__restrict__ desc, const int32_t *__restrict__ gidx,
    const float *__restrict__ geom, int G, float *__restrict__ out, const float *__restrict__ pre) {
    constexpr int C = K::C, T1 = K::T1, TA = K::TA;
    constexpr int NE = K::TABLE - K::F_END;
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G * KH / 32;
    constexpr int WT = win_for<T1>();
    const FragSeq fd{K::F_D / 64, TA}, fg{K::F_G / 64, 2};
    const FragSeq f2{K::F_2 / 64, T1 * 16}, f3{K::F_3 / 64, T1 * 16};
    constexpr int W0 = PRE ? first_win<2, T1>() : first_win<TA, T1>();
    const FragSeq f0 = PRE ? fg : fd;  // the first call of a tile

    float carry[CARRY];
    {
        const gfloat *tb = reinterpret_cast<const gfloat *>(reinterpret_cast<uint64_t>(table));
        constexpr int GS0 = W0 < 4 ? W0 : 4;
#pragma unroll
        for (int s0 = 0; s0 < W0; s0 += GS0)
#pragma unroll
            for (int co = 0; co < T1; ++co) {
                float v[GS0];
                ldgroup<GS0>(tb, f0.base + co * f0.stride + s0, lane, v);
#pragma unroll
                for (int i = 0; i < GS0; ++i) carry[(s0 + i) * T1 + co] = v[i];
            }
    }
    for (int t = blockIdx.x * WAVES + w; t < NT; t += gridDim.x * WAVES) {
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gfloat *tb = reinterpret_cast<const gfloat *>(tba);
        const int row = t * 32 + j;
        const int g = row / KH;
        const float *drow = desc + (size_t)gidx[row] * C;
        float c1[CARRY], c2[CARRY], c3[CARRY], c4[CARRY];

        f32x16 h1[T1], h2[T1];
        if constexpr (PRE) {
            init_from_rows<K::N1, T1>(h1, pre + (size_t)gidx[row] * K::N1, nullptr, h);
            mfma_pipe_rows<2, T1, T1, WT>(tb, lane, fg, geom + (size_t)row * 4 + h * 2, h1, carry, f2, c2);
            (void)c1;
        } else {
            zero_tiles(h1);
            mfma_pipe_rows<TA, T1, T1, 2>(tb, lane, fd, drow + h * TA, h1, carry, fg, c1);
            mfma_pipe_rows<2, T1, T1, WT>(tb, lane, fg, geom + (size_t)row * 4 + h * 2, h1, c1, f2, c2);
        }
        epilogue<T1>(eb + K::E_1, lane, h1);
        zero_tiles(h2);
        mfma_pipe<T1 * 16, T1, T1, WT>(tb, lane, f2, [&](int st) { return h1[st >> 4][st & 15]; }, h2, c2,
                                       f3, c3);
        epilogue<T1>(eb + K::E_2, lane, h2);
        f32x16 f[T1];
        zero_tiles(f);
        mfma_pipe<T1 * 16, T1, T1, W0>(tb, lane, f3, [&](int st) { return h2[st >> 4][st & 15]; }, f, c3,
                                       f0, carry);
        epilogue<T1>(eb + K::E_3, lane, f);
        (void)c4;
        nbr_attend<T1, C>(f, lane, row, drow, out);
    }
}

// ------------------------------------------------------------------------
// The same two heads with the products on the bf16 matrix cores at fp32 accuracy
// (bf16x6, mfma_chain.h mfma_pipe6; group_fused6.hip for the level kernels), for the
// precomputed-descriptor form only (HEAD_PRE): the accumulators start from the
// per-point products, the narrow first block (FineReg: the 16 small columns = one
// 16-deep chunk; neighbour branch: the 4 geometry columns, zero-padded to a chunk)
// and the two N1 x N1 layers run as 6 v_mfma_f32_32x32x16_bf16 per chunk instead of
// 8 v_mfma_f32_32x32x2_f32.  Table (engine.head_table6): [T1][1] first-block chunk
// fragments, [T1][2 T1] conv 2, [T1][2 T1] conv 3 (units of 3 pieces x 64 lanes x
// 16 B), then the f32 epilogues.
template <int N1_, int WPS_>
struct Head6Cfg {
    static constexpr int N1 = N1_, WPS = WPS_, T1 = N1 / 32, NC = 2 * T1;
    static constexpr int G_S = 0, G_2 = T1, G_3 = G_2 + T1 * NC, G_END = G_3 + T1 * NC;
    static constexpr int F_END = G_END * 3 * 64 * 4;
    static constexpr int E_1 = F_END, E_2 = E_1 + 2 * N1, E_3 = E_2 + 2 * N1, TABLE = E_3 + 2 * N1;
};
using Fine1x6 = Head6Cfg<128, 2>;
using Fine2x6 = Head6Cfg<256, 1>;
using Nbrx6 = Head6Cfg<256, 1>;

typedef u32x4 Carry6[CARRY6][3];

// the three conv layers of a head tile: h1 holds the precomputed products; b0 gives the
// first block's B values (f32 k-steps 0..7 of the lane); f receives the last layer
// BN folded (engine._fold_bn): the precomputed products and the weight pieces carry alpha;
// h1 starts from them (plus beta where the caller's rows do not hold it), layers 2 and 3
// start from beta; every epilogue is the ReLU.
template <class K, class B0>
__device__ __forceinline__ void head_chain6(const gu32x4 *__restrict__ wt, const float *eb, int lane, B0 b0,
                                            f32x16 (&h1)[K::T1], f32x16 (&f)[K::T1], Carry6 &carry) {
    constexpr int T1 = K::T1, NC = K::NC;
    const FragSeq fs{K::G_S, 1}, f2{K::G_2, NC}, f3{K::G_3, NC};
    Carry6 c2, c3;
    mfma_pipe6<1, T1, T1>(wt, lane, fs, b0, h1, carry, f2, c2);
    relu_tiles(h1);
    f32x16 h2[T1];
    beta_tiles<T1>(eb + K::E_2, lane, h2);
    mfma_pipe6<NC, T1, T1>(wt, lane, f2, [&](int st) { return h1[st >> 4][st & 15]; }, h2, c2, f3, c3);
    relu_tiles(h2);
    beta_tiles<T1>(eb + K::E_3, lane, f);
    mfma_pipe6<NC, T1, T1>(wt, lane, f3, [&](int st) { return h2[st >> 4][st & 15]; }, f, c3, fs, carry);
    relu_tiles(f);
}

template <class K>
__global__ __launch_bounds__(256, K::WPS) void fine_head6_kernel(
    const float *__restrict__ table, const float *__restrict__ small, const int32_t *__restrict__ gidx,
    const float *__restrict__ knn_xyz, int G, float *__restrict__ corres, float *__restrict__ att,
    const float *__restrict__ pre_src, const float *__restrict__ pre_dst) {
    constexpr int N1 = K::N1, T1 = K::T1;
    constexpr int NE = K::TABLE - K::F_END;
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G * KH / 32;
    Carry6 carry;
    {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int co = 0; co < T1; ++co) ld6(wt, K::G_S + co, lane, carry[co]);
    }
    for (int t = blockIdx.x * WAVES + w; t < NT; t += gridDim.x * WAVES) {
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
        const int row = t * 32 + j;
        const int g = row / KH;
        // the 8 small columns of this lane's half (k-step s <-> column 8h + s)
        const float4 s0 = *reinterpret_cast<const float4 *>(small + (size_t)row * 16 + h * 8);
        const float4 s1 = *reinterpret_cast<const float4 *>(small + (size_t)row * 16 + h * 8 + 4);
        const float sm[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        f32x16 h1[T1], f[T1];
        init_from_rows<N1, T1>(h1, pre_src + (size_t)g * N1, pre_dst + (size_t)gidx[row] * N1, h);
#pragma unroll
        for (int co = 0; co < T1; ++co)  // + beta of convs_1[0] (the pre GEMM is batch-2)
#pragma unroll
            for (int q = 0; q < 16; ++q) h1[co][q] = fadd_rn(h1[co][q], eb[K::E_1 + N1 + chan(co, q, h)]);
        head_chain6<K>(wt, eb, lane, [&](int st) { return sm[st]; }, h1, f, carry);
        fine_attend<T1>(f, lane, row, knn_xyz, corres, att);
    }
}

template <class K, int C>
__global__ __launch_bounds__(256, K::WPS) void nbr_head6_kernel(
    const float *__restrict__ table, const float *__restrict__ desc, const int32_t *__restrict__ gidx,
    const float *__restrict__ geom, int G, float *__restrict__ out, const float *__restrict__ pre) {
    constexpr int N1 = K::N1, T1 = K::T1;
    constexpr int NE = K::TABLE - K::F_END;
    __shared__ float ep[NE];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[K::F_END + i];
    __syncthreads();
    const float *eb = ep - K::F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G * KH / 32;
    Carry6 carry;
    {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int co = 0; co < T1; ++co) ld6(wt, K::G_S + co, lane, carry[co]);
    }
    for (int t = blockIdx.x * WAVES + w; t < NT; t += gridDim.x * WAVES) {
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
        const int row = t * 32 + j;
        const size_t src = (size_t)gidx[row];
        // geometry k-steps 0, 1 (columns 2h, 2h + 1 of [dxyz, |d|]), the rest of the chunk zero
        const float2 gin = *reinterpret_cast<const float2 *>(geom + (size_t)row * 4 + h * 2);
        f32x16 h1[T1], f[T1];
        init_from_rows<N1, T1>(h1, pre + src * N1, nullptr, h);  // engine.nbr_pre6: alpha-folded + beta
        head_chain6<K>(wt, eb, lane, [&](int st) { return st == 0 ? gin.x : st == 1 ? gin.y : 0.f; }, h1, f,
                       carry);
        nbr_attend<T1, C>(f, lane, row, desc + src * C, out);
    }
}

template <class K>
int launch_fine(const float *table, const float *small, const float *src_desc, const float *dst_desc,
                const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                const float *pre_src, const float *pre_dst, void *stream) {
    if ((reinterpret_cast<uintptr_t>(small) & 15) || (reinterpret_cast<uintptr_t>(src_desc) & 15) ||
        (reinterpret_cast<uintptr_t>(dst_desc) & 15) || (reinterpret_cast<uintptr_t>(att) & 15) ||
        (reinterpret_cast<uintptr_t>(pre_src) & 15) || (reinterpret_cast<uintptr_t>(pre_dst) & 15))
        return HREG_ERR_INVALID;
    if (!pre_src != !pre_dst) return HREG_ERR_INVALID;
    if ((G * KH) % 32) return HREG_ERR_INVALID;  // whole 32-row tiles
    const int NT = G * KH / 32;
    int grid = (NT + WAVES - 1) / WAVES;
    const int cap = 256 * K::WPS * 2;
    if (grid > cap) grid = cap;
    if (pre_src)
        hipLaunchKernelGGL((fine_head_kernel<K, true>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           small, src_desc, dst_desc, gidx, knn_xyz, G, corres, att, pre_src, pre_dst);
    else
        hipLaunchKernelGGL((fine_head_kernel<K, false>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           small, src_desc, dst_desc, gidx, knn_xyz, G, corres, att, pre_src, pre_dst);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

template <class K>
int launch_fine6(const float *table, const float *small, const int32_t *gidx, const float *knn_xyz, int G,
                 float *corres, float *att, const float *pre_src, const float *pre_dst, void *stream) {
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(small) & 15) ||
        (reinterpret_cast<uintptr_t>(att) & 15) || (reinterpret_cast<uintptr_t>(pre_src) & 15) ||
        (reinterpret_cast<uintptr_t>(pre_dst) & 15))
        return HREG_ERR_INVALID;
    if ((G * KH) % 32) return HREG_ERR_INVALID;  // whole 32-row tiles
    const int NT = G * KH / 32;
    int grid = (NT + WAVES - 1) / WAVES;
    const int cap = 256 * K::WPS * 2;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL((fine_head6_kernel<K>), dim3(grid), dim3(256), 0, as_stream(stream), table, small, gidx,
                       knn_xyz, G, corres, att, pre_src, pre_dst);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_head6_table_floats(int N1) {
    return N1 == 128 ? Fine1x6::TABLE : N1 == 256 ? Fine2x6::TABLE : 0;
}

extern "C" int hreg_fine_head6(const float *table, int C, const float *small, const int32_t *gidx,
                               const float *knn_xyz, int G, float *corres, float *att, const float *pre_src,
                               const float *pre_dst, void *stream) {
    if (!table || !small || !gidx || !knn_xyz || !corres || !att || !pre_src || !pre_dst || G < 0)
        return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    if (C == 64)
        return launch_fine6<Fine1x6>(table, small, gidx, knn_xyz, G, corres, att, pre_src, pre_dst, stream);
    if (C == 128)
        return launch_fine6<Fine2x6>(table, small, gidx, knn_xyz, G, corres, att, pre_src, pre_dst, stream);
    return HREG_ERR_UNSUPPORTED;
}

extern "C" int hreg_nbr_head6(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                              int G, float *out, const float *pre, void *stream) {
    if (!table || !desc || !gidx || !geom || !out || !pre || G < 0) return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15) ||
        (reinterpret_cast<uintptr_t>(geom) & 7) || (reinterpret_cast<uintptr_t>(out) & 15) ||
        (reinterpret_cast<uintptr_t>(pre) & 15))
        return HREG_ERR_INVALID;
    if ((G * KH) % 32) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    const int NT = G * KH / 32;
    int grid = (NT + WAVES - 1) / WAVES;
    if (grid > 512) grid = 512;
    hipLaunchKernelGGL((nbr_head6_kernel<Nbrx6, 256>), dim3(grid), dim3(256), 0, as_stream(stream), table, desc,
                       gidx, geom, G, out, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_nbr_head_table_floats(void) { return Nbr::TABLE; }

extern "C" int hreg_nbr_head(const float *table, const float *desc, const int32_t *gidx,
                             const float *geom, int G, float *out, const float *pre, void *stream) {
    if (!table || !desc || !gidx || !geom || !out || G < 0) return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(desc) & 15) || (reinterpret_cast<uintptr_t>(geom) & 15) ||
        (reinterpret_cast<uintptr_t>(out) & 15) || (reinterpret_cast<uintptr_t>(pre) & 15))
        return HREG_ERR_INVALID;
    if ((G * KH) % 32) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    const int NT = G * KH / 32;
    int grid = (NT + WAVES - 1) / WAVES;
    if (grid > 512) grid = 512;
    if (pre)
        hipLaunchKernelGGL((nbr_head_kernel<Nbr, true>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           desc, gidx, geom, G, out, pre);
    else
        hipLaunchKernelGGL((nbr_head_kernel<Nbr, false>), dim3(grid), dim3(256), 0, as_stream(stream), table,
                           desc, gidx, geom, G, out, pre);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_fine_head_table_floats(int C) {
    return C == 64 ? Fine1::TABLE : C == 128 ? Fine2::TABLE : 0;
}

extern "C" int hreg_fine_head(const float *table, int C, const float *small, const float *src_desc,
                              const float *dst_desc, const int32_t *gidx, const float *knn_xyz,
                              int G, float *corres, float *att, const float *pre_src,
                              const float *pre_dst, void *stream) {
    if (!table || !small || !src_desc || !dst_desc || !gidx || !knn_xyz || !corres || !att || G < 0)
        return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    if (C == 64)
        return launch_fine<Fine1>(table, small, src_desc, dst_desc, gidx, knn_xyz, G, corres, att, pre_src,
                                  pre_dst, stream);
    if (C == 128)
        return launch_fine<Fine2>(table, small, src_desc, dst_desc, gidx, knn_xyz, G, corres, att, pre_src,
                                  pre_dst, stream);
    return HREG_ERR_UNSUPPORTED;
}
