// group_l1_6.hip -- the fused level-1 keypoint detector + descriptor of group_l1.hip
// (same layers, same decomposition: one wave owns one keypoint group = its k = 64
// neighbour rows as two 32-row MFMA column tiles, every activation in the MFMA
// accumulators; layers.py:115-121, 150-159, 183-208) with the products on the bf16
// matrix cores at fp32 accuracy (bf16x6, mfma_chain.h): a 16-deep k-chunk is 6
// v_mfma_f32_32x32x16_bf16 per row tile instead of 8 v_mfma_f32_32x32x2_f32.
//
// Differences from group_l1.hip:
//  * the weight pieces (92 KB, 1.5x the f32 fragments) stream from the L2-resident
//    table one chunk ahead of their MFMAs and across call boundaries (the last chunk of
//    a call loads the first chunk of the next call, the last call of a group the first
//    chunk of the next group), as in group_fused6.hip; only the BN epilogues sit in LDS;
//  * the two row tiles share each chunk's weight pieces; every row tile's B chunk (8
//    f32 k-steps of the lane) is split into its bf16 pieces in registers (once for the
//    k-max row x2, which is the same for both tiles);
//  * mlp1's emb*a block is accumulated right after the attention (then emb is dead
//    through the descriptor stack), then the x2 and x1d blocks;
//  * BN folded (engine._fold_bn): alpha in the weight pieces, the accumulators start from
//    beta, the epilogue is the ReLU;
//  * the per-channel reductions over the 64 rows (attentive feature, x2, descriptor k-max)
//    combine the two row tiles in registers, then run as butterflies over a tile's 16
//    values (rowred.h) and store from the reduced slots;
//  * built without packed fp32 VALU ops (build.NO_PACKED_F32): with them this kernel gave
//    nondeterministic wrong accumulator values whenever two waves shared a SIMD.
#include "mfma_chain.h"
// weight table resident in LDS (below: the LDSW kernel form, hreg_group_l1_6) or streamed
// from global memory (hreg_group_l1_6g)
namespace hreg_chain {
__device__ __forceinline__ void ld6(const __attribute__((address_space(3))) u32x4 *wt, int f, int lane,
                                    u32x4 (&o)[3]) {
    const __attribute__((address_space(3))) u32x4 *fp = wt + f * 192;
#pragma unroll
    for (int p = 0; p < 3; ++p) o[p] = fp[p * 64 + lane];
}
}  // namespace hreg_chain
#include "mfma_jt.h"
#include "rowred.h"

namespace {

using namespace hreg_chain;
using namespace hreg_jt;
using namespace hreg_rowred;

constexpr int WAVES = 4;
constexpr int KN = 64;  // neighbours per group (level 1) = JT 32-row tiles

// chunk-fragment table (units of 3 pieces x 64 lanes x 16 B), engine.l1_table6
constexpr int G_DC1 = 0;             // det conv1 (geom, 2 k-steps zero-padded): 1 co x 1 chunk
constexpr int G_DC2 = G_DC1 + 1;     // det conv2 32 -> 32: 1 co x 2
constexpr int G_DC3 = G_DC2 + 2;     // det conv3 32 -> 64: 2 co x 2
constexpr int G_EC1 = G_DC3 + 4;     // desc convs, same shapes
constexpr int G_EC2 = G_EC1 + 1;
constexpr int G_EC3 = G_EC2 + 2;
constexpr int G_M1 = G_EC3 + 4;      // mlp1 192 -> 32: 1 co x 12 chunks (x2 0..3 | x1d 4..7 | emb*a 8..11)
constexpr int G_M2 = G_M1 + 12;      // mlp2 32 -> 64: 2 co x 2
constexpr int G_END = G_M2 + 4;
constexpr int F_END = G_END * 3 * 64 * 4;  // floats; the f32 epilogues follow (group_l1.hip E_* order)
constexpr int E_DC1 = F_END, E_DC2 = E_DC1 + 64, E_DC3 = E_DC2 + 64, E_EC1 = E_DC3 + 128,
              E_EC2 = E_EC1 + 64, E_EC3 = E_EC2 + 64, E_M1 = E_EC3 + 128, E_M2 = E_M1 + 64,
              TABLE_FLOATS = E_M2 + 128;

// conv stack 4 -> 32 -> 32 -> 64 (+ BN/ReLU); NC: output tiles of the call that follows
template <int NC, class WP>
__device__ __forceinline__ void conv_stack6(WP wt, const float *eb, int g1, int g2, int g3,
                                            int e1, int e2, int e3, int lane, const float2 (&gin)[JT],
                                            f32x16 (&out)[2][JT], const Carry &cin, FragSeq next, Carry &cout) {
    f32x16 h1[1][JT], h2[1][JT];
    Carry c2, c3;
    beta_jt<1>(eb + e1, lane, h1);
    // geometry chunk: f32 k-steps 0, 1 (channels 2h, 2h + 1), the rest zero
    pipe6_jt<1, 1, 1, false>(
        wt, lane, FragSeq{g1, 1},
        [&](int jt, int st) { return st == 0 ? gin[jt].x : st == 1 ? gin[jt].y : 0.f; }, h1, cin,
        FragSeq{g2, 2}, c2);
    relu_jt(h1);
    beta_jt<1>(eb + e2, lane, h2);
    pipe6_jt<2, 1, 2, false>(wt, lane, FragSeq{g2, 2}, [&](int jt, int st) { return h1[st >> 4][jt][st & 15]; },
                             h2, c2, FragSeq{g3, 2}, c3);
    relu_jt(h2);
    beta_jt<2>(eb + e3, lane, out);
    pipe6_jt<2, 2, NC, false>(wt, lane, FragSeq{g3, 2}, [&](int jt, int st) { return h2[st >> 4][jt][st & 15]; },
                              out, c3, next, cout);
    relu_jt(out);
}

// waves per SIMD the register budget targets (the global-table form; 3 spills 49 VGPRs)
constexpr int L16_WPS = 2;
// (measured and removed, r5: the younger half of the 8-wave workgroup at s_setprio 1, 180.7 ->
// 183.3 us)
// LDSW (hreg_group_l1_6): the whole weight-piece table (90 KB) resident in LDS -- each 8-wave
// workgroup copies it once and loops over 16+ groups; chunk fragments are ds_read_b128
// (the per-wave weight streams through the vector-memory path keep the CU's texture-data
// return unit ~70-87 % busy).  The epilogue constants then come through vector memory so
// that the LDS counter tracks the fragment reads alone, and the prefetch is pinned ahead
// of each chunk's MFMAs (mfma_jt.h).  Measured: 172.7 vs 175.2 us in the
// bench, 328k vs 340k cycles standalone.  But the 92 KB of LDS leave no room beside a
// co-running kernel that holds LDS on every CU -- Model_V2's cluster FPS (clouds > 16384
// points) -- so that configuration runs the global-table form (LDSW false, 4-wave
// workgroups): Model_V2 942 vs 856 pairs/s.
template <bool LDSW>
constexpr int l1_waves() { return LDSW ? 8 : WAVES; }
typedef __attribute__((address_space(3))) const u32x4 lu32x4;

template <bool LDSW>
__global__ __launch_bounds__(l1_waves<LDSW>() * 64, LDSW ? 1 : L16_WPS) void group_l1_6_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    int G, float *__restrict__ kp, float *__restrict__ att_feat, float *__restrict__ desc) {
    constexpr int L1_WAVES = l1_waves<LDSW>();
    constexpr int NE = TABLE_FLOATS - F_END;
    __shared__ u32x4 wl[LDSW ? G_END * 192 : 1];
    __shared__ float ep[LDSW ? 1 : NE];
    if constexpr (LDSW) {
        for (int i = threadIdx.x; i < G_END * 192; i += blockDim.x) wl[i] = reinterpret_cast<const u32x4 *>(table)[i];
    } else {
        for (int i = threadIdx.x; i < NE; i += blockDim.x) ep[i] = table[F_END + i];
    }
    __syncthreads();
    const float *eb = LDSW ? table : ep - F_END;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    const FragSeq m1x2{G_M1, 12}, m1x1{G_M1 + 4, 12}, m1em{G_M1 + 8, 12}, m2{G_M2, 2};
    // opaque per-group table pointer: keeps the loop-invariant weight loads in the loop
    auto table_ptr = [&]() {
        if constexpr (LDSW) {
            uint32_t lb = (uint32_t)reinterpret_cast<uintptr_t>((const lu32x4 *)wl);
            asm volatile("" : "+s"(lb));
            return (const lu32x4 *)(uintptr_t)lb;
        } else {
            uint64_t tba = reinterpret_cast<uint64_t>(table);
            asm volatile("" : "+s"(tba));
            return reinterpret_cast<const gu32x4 *>(tba);
        }
    };

    Carry carry;
    ld6(table_ptr(), G_DC1, lane, carry[0]);
    for (int g = blockIdx.x * L1_WAVES + w; g < G; g += gridDim.x * L1_WAVES) {
        const auto wt = table_ptr();
        const size_t r0 = (size_t)g * KN;
        float2 gin[JT];
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
            gin[jt] = *reinterpret_cast<const float2 *>(geom + (r0 + jt * 32 + j) * 4 + 2 * h);
        Carry ca, cb;

        // ---- detector convs -> emb [64 ch][64 rows]
        f32x16 emb[2][JT];
        conv_stack6<1>(wt, eb, G_DC1, G_DC2, G_DC3, E_DC1, E_DC2, E_DC3, lane, gin, emb, carry, m1em, ca);

        // ---- attention: x1 = max_c emb, a = softmax over the 64 rows (group_l1.hip)
        float x1[JT];
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            int mi = __float_as_int(emb[0][jt][0]);
#pragma unroll
            for (int co = 0; co < 2; ++co)
#pragma unroll
                for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[co][jt][q]));
            x1[jt] = __int_as_float(max(mi, __shfl_xor(mi, 32)));
        }
        const float mx = half_bcast(half_max_hi_nonneg(max_nonneg(x1[0], x1[1])), h);
        const float e0 = expf(fsub_rn(x1[0], mx)), e1 = expf(fsub_rn(x1[1], mx));
        const float ssum = half_bcast(half_sum_hi(fadd_rn(e0, e1)), h);
        const float a[JT] = {e0 / ssum, e1 / ssum};

        float kx = 0.f, ky = 0.f, kz = 0.f;
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            const float *p = knn_xyz + (r0 + jt * 32 + j) * 3;
            kx = fadd_rn(kx, fmul_rn(a[jt], p[0]));
            ky = fadd_rn(ky, fmul_rn(a[jt], p[1]));
            kz = fadd_rn(kz, fmul_rn(a[jt], p[2]));
        }
        kx = half_sum_hi(kx); ky = half_sum_hi(ky); kz = half_sum_hi(kz);
        if (lane == 31) {
            kp[(size_t)g * 3 + 0] = kx;
            kp[(size_t)g * 3 + 1] = ky;
            kp[(size_t)g * 3 + 2] = kz;
        }
#pragma unroll
        for (int co = 0; co < 2; ++co) {
            float v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = fadd_rn(fmul_rn(emb[co][0][q], a[0]), fmul_rn(emb[co][1][q], a[1]));
            reduce_store<32, Sum>(att_feat + (size_t)g * 64, co, v, lane);
        }

        // ---- mlp1 = W [x2 | x1d | emb * a] -> 32, the emb * a block first
        f32x16 y1[1][JT];
        beta_jt<1>(eb + E_M1, lane, y1);
        pipe6_jt<4, 1, 1, false>(wt, lane, m1em,
                                 [&](int jt, int st) { return fmul_rn(emb[st >> 4][jt][st & 15], a[jt]); }, y1, ca,
                                 FragSeq{G_EC1, 1}, cb);

        // ---- descriptor convs -> x1d [64][64]
        f32x16 x1d[2][JT];
        conv_stack6<1>(wt, eb, G_EC1, G_EC2, G_EC3, E_EC1, E_EC2, E_EC3, lane, gin, x1d, cb, m1x2, ca);
        // x2 = max over the 64 rows (the repeat of layers.py:204: same for every row)
        float x2[2][16];
#pragma unroll
        for (int co = 0; co < 2; ++co) {
#pragma unroll
            for (int q = 0; q < 16; ++q) x2[co][q] = max_nonneg(x1d[co][0][q], x1d[co][1][q]);
            bfly32<MaxNN>(x2[co], lane);
            bcast32(x2[co], lane);
        }
        {
            // the x2 block (the k-max row repeated over the 64 rows, layers.py:204-206) once: its
            // B, and so its product, is the same for both row tiles; added to both tiles after
            // the x1d block (24 of the group's 360 MFMAs fewer: 177.6 -> 173.1 us, r5)
            f32x16 z[1][1];
            z[0][0] = zero16();
            pipe6_jt<4, 1, 1, true>(wt, lane, m1x2, [&](int, int st) { return x2[st >> 4][st & 15]; }, z, ca,
                                    m1x1, cb);
            pipe6_jt<4, 1, 2, false>(wt, lane, m1x1, [&](int jt, int st) { return x1d[st >> 4][jt][st & 15]; },
                                     y1, cb, m2, ca);
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int q = 0; q < 16; ++q) y1[0][jt][q] = fadd_rn(y1[0][jt][q], z[0][0][q]);
        }
        relu_jt(y1);

        // ---- mlp2: 32 -> 64, k-max -> descriptor; prefetches the next group's first chunk
        f32x16 y2[2][JT];
        beta_jt<2>(eb + E_M2, lane, y2);
        pipe6_jt<2, 2, 1, false>(wt, lane, m2, [&](int jt, int st) { return y1[st >> 4][jt][st & 15]; }, y2, ca,
                                 FragSeq{G_DC1, 1}, carry);
        relu_jt(y2);
#pragma unroll
        for (int co = 0; co < 2; ++co) {
            float v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = max_nonneg(y2[co][0][q], y2[co][1][q]);
            reduce_store<32, MaxNN>(desc + (size_t)g * 64, co, v, lane);
        }
    }
}

}  // namespace

extern "C" int hreg_group_l1_6_table_floats(void) { return TABLE_FLOATS; }

template <bool LDSW>
static int launch_l1_6(const float *table, const float *geom, const float *knn_xyz, int G, float *kp,
                       float *att_feat, float *desc, void *stream) {
    if (!table || !geom || !knn_xyz || !kp || !att_feat || !desc || G < 0) return HREG_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(table) & 15) || (reinterpret_cast<uintptr_t>(geom) & 7) ||
        (reinterpret_cast<uintptr_t>(att_feat) & 15) || (reinterpret_cast<uintptr_t>(desc) & 15))
        return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    constexpr int L1_WAVES = l1_waves<LDSW>();
    int grid = (G + L1_WAVES - 1) / L1_WAVES;
    // LDS table: workgroups of 8 waves x 2+ groups (the 90 KB copy amortised over 16 groups;
    // a fully persistent grid stalls behind CUs held by concurrent kernels)
    const int cap = LDSW ? 1024 : 2048;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(group_l1_6_kernel<LDSW>, dim3(grid), dim3(L1_WAVES * 64), 0, as_stream(stream), table, geom,
                       knn_xyz, G, kp, att_feat, desc);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_group_l1_6(const float *table, const float *geom, const float *knn_xyz, int G, float *kp,
                               float *att_feat, float *desc, void *stream) {
    return launch_l1_6<true>(table, geom, knn_xyz, G, kp, att_feat, desc, stream);
}

extern "C" int hreg_group_l1_6g(const float *table, const float *geom, const float *knn_xyz, int G, float *kp,
                                float *att_feat, float *desc, void *stream) {
    return launch_l1_6<false>(table, geom, knn_xyz, G, kp, att_feat, desc, stream);
}
