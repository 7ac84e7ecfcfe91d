// coarse6.hip -- CoarseReg correspondence features in one launch (layers.py:364-390):
// convs_1 (3 x [1x1 Conv2d + BN + ReLU], 528 -> 512 -> 512 -> 512) over the rows of
// every keypoint's 8 descriptor-space neighbours, then the attention of layers.py:384-390
// (a = softmax over the 8 rows of max over channels; corres = sum_j a_j knn_xyz_j; the
// attentive feature sum_j a_j f_j), with the products on the bf16 matrix cores at fp32
// accuracy (bf16x6, mfma_chain.h).
//
// convs_1[0] runs in its split form (engine.COARSE_SPLIT): the desc / knn_desc blocks of
// the 528-wide row are the same for the 8 rows of a keypoint / for every row gathering a
// destination keypoint, so their products ud0[g] = W_d desc_src[g], ud1[n] = W_kd
// desc_dst[n] are made once per keypoint (one batch-2 GEMM) and initialise the
// accumulators; only the 16 small columns [dxyz, |d|, xyz, knn_xyz, w, knn_w, sims 4]
// run here (one 16-deep chunk).
//
// Decomposition (split_chain.h, as mlp_head.hip): a workgroup of 8 waves owns a 32-row
// tile (4 keypoints); each wave computes P = 2 output tiles (64 channels) of every layer;
// a layer's output goes through one LDS buffer (32 x 512 f32, row-major) to the next
// layer's B operand, which each wave splits into bf16 pieces as it reads it.  Weight
// pieces stream from the L2-resident table (engine.coarse_head_table6) one chunk ahead.
// The channel max of the attention is reduced per wave, then across the 8 waves through
// LDS; the reductions over a keypoint's 8 rows are 3 DPP steps.
// chunk c + 1's B split under chunk c's MFMAs in pipe_lds6_jt (split_chain.h, SWP = true): the
// heads measured 127.8 -> 123.5 (CoarseReg), 56.4 -> 54.2 (FineReg), 66.4 -> 64.4 us
// (neighbour branch) eager; level 3's group_split6j (same pipe) neutral, so it stays off there
#include "split_chain.h"

namespace {

using namespace hreg_chain;
using namespace hreg_split;

constexpr int KH = 8;

// conv width C (= attention output channels): CoarseReg C = 512, FineReg N1 = 256 / 128.
// CW waves of P = 2 output tiles each (P = 2: one B split feeds 12 MFMAs).
template <int C_, int P_ = 2>
struct CorrCfg {
    static constexpr int C = C_, T = C / 32, P = P_, CW = T / P, LDSW = C + 4;
    static constexpr int NCH = T * 2;  // 16-deep chunks over C inputs
    // chunk-fragment table (units of 3 pieces x 64 lanes x 16 B), engine.coarse_head_table6
    // (and engine.fine_head_table6: the same layout)
    static constexpr int G_1 = 0;               // layer 0, the 16 small columns: [T][1]
    static constexpr int G_2 = G_1 + T;         // layer 1: [T][NCH]
    static constexpr int G_3 = G_2 + T * NCH;   // layer 2: [T][NCH]
    static constexpr int G_END = G_3 + T * NCH;
    static constexpr int F_END = G_END * 3 * 64 * 4;
    static constexpr int NE = 6 * C;            // alpha, beta of the three layers
    static constexpr int TABLE = F_END + NE;
};

// JT: 32-row tiles per workgroup.  2: every wave computes its P output tiles for both row
// tiles, so each streamed weight chunk feeds twice the MFMAs (the one-tile weight stream,
// 512 B of pieces per MFMA, keeps the CU's texture-data return unit ~82 % busy).  At C = 512
// the 64-row activation buffer (132 KB) leaves one workgroup per CU and measured slower (154
// vs 134 us): JT = 1 there; at C = 256 (FineReg level-2 head, neighbour branch; 73 KB) two
// workgroups still fit per CU: JT = 2 (corr_jt; same products and order: the same bits); the
// C = 128 head (a smaller grid) measured 48 vs 37 us on two tiles and stays on one.  (The
// C = 512 head on two row tiles -- 145 KB of LDS, one workgroup per CU -- measured -2.1 % in the
// bench, r5, and was removed.)
template <class K>
constexpr int corr_jt() { return K::C == 256 ? 2 : 1; }

// NBR: CoarseReg's neighbour branch (layers.py:315-337, nbr_head6_kernel's job): rows
// [desc[nbr] C | dxyz, |d|] through convs_2, the descriptor block precomputed per point
// with its beta (ud1 = engine.nbr_pre6 rows gathered by gidx; no per-keypoint block), the
// 4 geometry columns as k-steps 0, 1 of each lane half (small = geom [rows][4]); output
// sum_j a_j desc[nbr_j] (knn_xyz = desc, att = out; no corres).
template <class K, bool NBR, int JT>
__global__ __launch_bounds__(K::CW * 64) void coarse_head6_kernel(
    const float *__restrict__ table, const float *__restrict__ small, const float *__restrict__ ud0,
    const float *__restrict__ ud1, const int32_t *__restrict__ gidx, const float *__restrict__ knn_xyz, int G,
    float *__restrict__ corres, float *__restrict__ att) {
    constexpr int C = K::C, T = K::T, P = K::P, CW = K::CW, LDSW = K::LDSW, NCH = K::NCH;
    constexpr int G_1 = K::G_1, G_2 = K::G_2, G_3 = K::G_3, F_END = K::F_END, NE = K::NE;
    constexpr int RW = 32 * JT;  // rows per workgroup step
    (void)T;
    __shared__ float ep[NE];
    __shared__ __attribute__((aligned(16))) float sA[RW * LDSW];
    __shared__ int sMax[CW][RW];
    for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[F_END + i];
    __syncthreads();  // the first tile's layer-1 epilogue reads ep before any tile_sync
    const int lane = threadIdx.x & 63, cw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const int NT = G * KH / 32;             // 32-row tiles
    const int NW = (NT + JT - 1) / JT;      // workgroup steps (a last odd tile is recomputed)
    const int c0 = cw * P;
    const FragSeq g1{G_1 + c0, 1}, g2{G_2 + c0 * NCH, NCH}, g3{G_3 + c0 * NCH, NCH};
    const bool writer = (j & 7) == 7;

    Carry6 carry;
    {
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(reinterpret_cast<uint64_t>(table));
#pragma unroll
        for (int i = 0; i < P; ++i) ld6(wt, g1.base + i, lane, carry[i]);
    }
    for (int tw = blockIdx.x; tw < NW; tw += gridDim.x) {
        uint64_t tba = reinterpret_cast<uint64_t>(table);
        asm volatile("" : "+s"(tba));
        const gu32x4 *wt = reinterpret_cast<const gu32x4 *>(tba);
        int row[JT], g[JT];
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            row[jt] = min(tw * JT + jt, NT - 1) * 32 + j;
            g[jt] = row[jt] / KH;
        }
        Carry6 ca, cb;

        // ---- convs_1[0]: precomputed desc / knn_desc products + the 16 small columns
        // (k-step s of lane half h <-> column 8h + s: one chunk)
        f32x16 y[P][JT];
        float sm[JT][8];
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            f32x16 yt[P];
            if constexpr (NBR) {
                init_from_rows<C, P>(yt, ud1 + (size_t)gidx[row[jt]] * C + c0 * 32, nullptr, h);
                const float2 gin = *reinterpret_cast<const float2 *>(small + (size_t)row[jt] * 4 + h * 2);
                sm[jt][0] = gin.x; sm[jt][1] = gin.y;
#pragma unroll
                for (int k = 2; k < 8; ++k) sm[jt][k] = 0.f;
            } else {
                init_from_rows<C, P>(yt, ud0 + (size_t)g[jt] * C + c0 * 32,
                                     ud1 + (size_t)gidx[row[jt]] * C + c0 * 32, h);
                const float4 s0 = *reinterpret_cast<const float4 *>(small + (size_t)row[jt] * 16 + h * 8);
                const float4 s1 = *reinterpret_cast<const float4 *>(small + (size_t)row[jt] * 16 + h * 8 + 4);
                sm[jt][0] = s0.x; sm[jt][1] = s0.y; sm[jt][2] = s0.z; sm[jt][3] = s0.w;
                sm[jt][4] = s1.x; sm[jt][5] = s1.y; sm[jt][6] = s1.z; sm[jt][7] = s1.w;
            }
#pragma unroll
            for (int i = 0; i < P; ++i) y[i][jt] = yt[i];
        }
        pipe_lds6_jt<1, P, P, JT, true>(wt, lane, g1, [&](int jt, int st0, float (&v)[4]) {
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = sm[jt][st0 + k];
        }, y, carry, g2, ca);
        // folded BN (engine._fold_bn: alpha in W_small and in the ud0 / ud1 weights): + beta, ReLU
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    y[i][jt][q] = relu_i(NBR ? y[i][jt][q] : fadd_rn(y[i][jt][q], ep[C + chan(c0 + i, q, h)]));
        tile_sync();  // the previous tile's readers of sA are done
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
            for (int i = 0; i < P; ++i) put_tile<LDSW>(sA + jt * 32 * LDSW, c0 + i, j, h, y[i][jt]);
        tile_sync();

        // ---- convs_1[1]
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
            for (int i = 0; i < P; ++i) load_tiles<1>(*reinterpret_cast<f32x16(*)[1]>(&y[i][jt]), ep + 3 * C + (c0 + i) * 32, h);
        pipe_lds6_jt<NCH, P, P, JT, true>(wt, lane, g2, ChanBJ<LDSW>{sA + j * LDSW, h}, y, ca, g3, cb);
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int q = 0; q < 16; ++q) y[i][jt][q] = relu_i(y[i][jt][q]);
        tile_sync();  // every wave has read the layer input
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
            for (int i = 0; i < P; ++i) put_tile<LDSW>(sA + jt * 32 * LDSW, c0 + i, j, h, y[i][jt]);
        tile_sync();

        // ---- convs_1[2]; prefetches the next step's first chunk
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
            for (int i = 0; i < P; ++i) load_tiles<1>(*reinterpret_cast<f32x16(*)[1]>(&y[i][jt]), ep + 5 * C + (c0 + i) * 32, h);
        pipe_lds6_jt<NCH, P, P, JT, true>(wt, lane, g3, ChanBJ<LDSW>{sA + j * LDSW, h}, y, cb, g1, carry);
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int q = 0; q < 16; ++q) y[i][jt][q] = relu_i(y[i][jt][q]);

        // ---- attention: row max over the 512 channels (ReLU outputs: integer max on the
        // bit patterns; per wave, then across the waves through LDS), softmax over the 8 rows
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            int mi = __float_as_int(y[0][jt][0]);
#pragma unroll
            for (int i = 0; i < P; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(y[i][jt][q]));
            mi = max(mi, __shfl_xor(mi, 32));
            if (h == 0) sMax[cw][jt * 32 + j] = mi;
        }
        tile_sync();
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            int xm = sMax[0][jt * 32 + j];
#pragma unroll
            for (int c = 1; c < CW; ++c) xm = max(xm, sMax[c][jt * 32 + j]);
            const float x1 = __int_as_float(xm);
            const float e = expf(fsub_rn(x1, grp8_max_nonneg(x1)));
            const float a = e / grp8_sum(e);
            if (!NBR && cw == 0) {
                const float *p = knn_xyz + (size_t)row[jt] * 3;
                const float cx = grp8_sum(fmul_rn(a, p[0]));
                const float cy = grp8_sum(fmul_rn(a, p[1]));
                const float cz = grp8_sum(fmul_rn(a, p[2]));
                if (writer && h == 0) {
                    corres[(size_t)g[jt] * 3 + 0] = cx;
                    corres[(size_t)g[jt] * 3 + 1] = cy;
                    corres[(size_t)g[jt] * 3 + 2] = cz;
                }
            }
            if constexpr (NBR) {
                // the attentive sum of the neighbours' descriptors (this wave's P channel tiles)
                f32x16 dv[P];
                init_from_rows<C, P>(dv, knn_xyz + (size_t)gidx[row[jt]] * C + c0 * 32, nullptr, h);
#pragma unroll
                for (int i = 0; i < P; ++i) {
                    f32x16 v;
#pragma unroll
                    for (int q = 0; q < 16; ++q) v[q] = grp8_sum(fmul_rn(dv[i][q], a));
                    store_tile(att + (size_t)g[jt] * C, c0 + i, v, writer, h);
                }
            } else {
#pragma unroll
                for (int i = 0; i < P; ++i) {
                    f32x16 v;
#pragma unroll
                    for (int q = 0; q < 16; ++q) v[q] = grp8_sum(fmul_rn(y[i][jt][q], a));
                    store_tile(att + (size_t)g[jt] * C, c0 + i, v, writer, h);
                }
            }
        }
    }
}

template <class K, bool NBR, int JT>
int launch_corr6_jt(const float *table, const float *small, const float *ud0, const float *ud1, const int32_t *gidx,
                    const float *knn_xyz, int G, float *corres, float *att, void *stream) {
    const int NW = (G * KH / 32 + JT - 1) / JT;
    const int cap = 256 * (JT == 1 ? 4 : 2);  // a few rounds of the resident workgroups
    const int grid = NW < cap ? NW : cap;
    hipLaunchKernelGGL((coarse_head6_kernel<K, NBR, JT>), dim3(grid), dim3(K::CW * 64), 0, as_stream(stream), table,
                       small, ud0, ud1, gidx, knn_xyz, G, corres, att);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// row_tiles: 0 = the configuration's default (corr_jt), 1 or 2 (A/B and the bitwise test)
template <class K, bool NBR = false>
int launch_corr6(const float *table, const float *small, const float *ud0, const float *ud1, const int32_t *gidx,
                 const float *knn_xyz, int G, float *corres, float *att, void *stream, int row_tiles = 0) {
    const int jt = row_tiles ? row_tiles : corr_jt<K>();
    if constexpr (K::C <= 256) {
        if (jt == 2) return launch_corr6_jt<K, NBR, 2>(table, small, ud0, ud1, gidx, knn_xyz, G, corres, att, stream);
    }
    if (jt == 1) return launch_corr6_jt<K, NBR, 1>(table, small, ud0, ud1, gidx, knn_xyz, G, corres, att, stream);
    return HREG_ERR_UNSUPPORTED;
}

}  // namespace

// two output tiles per wave throughout (one B split feeds 12 MFMAs): one tile per wave measured
// faster per launch for the FineReg / neighbour heads (53 / 64.5 vs 54.7 / 67.4 us) but slower
// in the bench (6910 / 6854 vs 6960 / 6965 pairs/s: every extra wave splits and reads the same B
// chunks again), and spilled 42 VGPRs for the 512-wide head (r2-r4)
using Corr512 = CorrCfg<512, 2>;
using Corr256 = CorrCfg<256, 2>;
using Corr128 = CorrCfg<128, 2>;
using Nbr256 = CorrCfg<256, 2>;

extern "C" int hreg_coarse_head6_table_floats(void) { return Corr512::TABLE; }

extern "C" int hreg_corr_head6_table_floats(int N1) {
    return N1 == 512 ? Corr512::TABLE : N1 == 256 ? Corr256::TABLE : N1 == 128 ? Corr128::TABLE : -1;
}

extern "C" int hreg_corr_head6x(const float *table, int N1, const float *small, const float *ud0, const float *ud1,
                                const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                                int row_tiles, void *stream) {
    if (!table || !small || !ud0 || !ud1 || !gidx || !knn_xyz || !corres || !att || G < 0)
        return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(small) & 15) ||
        (reinterpret_cast<uintptr_t>(ud0) & 15) || (reinterpret_cast<uintptr_t>(ud1) & 15) ||
        (reinterpret_cast<uintptr_t>(att) & 15))
        return HREG_ERR_INVALID;
    if ((G * KH) % 32) return HREG_ERR_INVALID;  // whole 32-row tiles
    if (N1 != 512 && N1 != 256 && N1 != 128) return HREG_ERR_UNSUPPORTED;
    if (!G) return HREG_OK;
    if (row_tiles < 0 || row_tiles > 2) return HREG_ERR_INVALID;
    if (N1 == 512)
        return launch_corr6<Corr512>(table, small, ud0, ud1, gidx, knn_xyz, G, corres, att, stream, row_tiles);
    if (N1 == 256)
        return launch_corr6<Corr256>(table, small, ud0, ud1, gidx, knn_xyz, G, corres, att, stream, row_tiles);
    return launch_corr6<Corr128>(table, small, ud0, ud1, gidx, knn_xyz, G, corres, att, stream, row_tiles);
}

extern "C" int hreg_corr_head6(const float *table, int N1, const float *small, const float *ud0, const float *ud1,
                               const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                               void *stream) {
    return hreg_corr_head6x(table, N1, small, ud0, ud1, gidx, knn_xyz, G, corres, att, 0, stream);
}

extern "C" int hreg_coarse_head6(const float *table, const float *small, const float *ud0, const float *ud1,
                                 const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                                 void *stream) {
    return hreg_corr_head6(table, 512, small, ud0, ud1, gidx, knn_xyz, G, corres, att, stream);
}

// hreg_nbr_head6 (group_head.hip) on the channel-split kernel: same arguments and table
// (engine.nbr_head_table6 -- the layout of coarse_head_table6 at C = 256 with a 2-k-step
// first block), bitwise-identical attention sums
extern "C" int hreg_nbr_head6sx(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                                int G, float *out, const float *pre, int row_tiles, void *stream) {
    if (!table || !desc || !gidx || !geom || !out || !pre || G < 0) return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15) ||
        (reinterpret_cast<uintptr_t>(geom) & 7) || (reinterpret_cast<uintptr_t>(out) & 15) ||
        (reinterpret_cast<uintptr_t>(pre) & 15))
        return HREG_ERR_INVALID;
    if ((G * KH) % 32) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    if (row_tiles < 0 || row_tiles > 2) return HREG_ERR_INVALID;
    return launch_corr6<Nbr256, true>(table, geom, nullptr, pre, gidx, desc, G, nullptr, out, stream, row_tiles);
}

extern "C" int hreg_nbr_head6s(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                               int G, float *out, const float *pre, void *stream) {
    return hreg_nbr_head6sx(table, desc, gidx, geom, G, out, pre, 0, stream);
}
