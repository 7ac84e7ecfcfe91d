// mfma_jt.h -- bf16x6 accumulator chains over JT = 2 row tiles per wave (group_l1_6.hip,
// group_pair6.hip): each chunk's weight pieces are loaded once and feed the MFMAs of both
// 32-row tiles, halving the weight bytes streamed from L2 per row (the register-chained
// kernels' L2 -> CU weight stream caps a one-tile wave near half the MFMA rate: 512 B of
// pieces per 32x32x16 MFMA).
#pragma once

#include "mfma_chain.h"

namespace hreg_jt {

using namespace hreg_chain;

constexpr int JT = 2;  // 32-row tiles per wave
typedef u32x4 Carry[CARRY6][3];

// acc[co][jt] += sum_{c < NCH} A(co, c) x B_jt(c), B_jt(c) = split(bval(jt, 8c .. 8c+7));
// the A pieces of a chunk are loaded once for both row tiles.  SAMEB: B does not depend
// on jt (split once).  cin / cout as mfma_pipe6 (double-buffered: COUT_T <= 2 here).
template <class T>
struct is_lds_table {
    static constexpr bool value = false;
};
template <>
struct is_lds_table<const __attribute__((address_space(3))) u32x4 *> {
    static constexpr bool value = true;
};

template <int NCH, int COUT_T, int NCOUT, bool SAMEB, class BVal, class WP, int NJ>
__device__ __forceinline__ void pipe6_jt(WP wt, int lane, FragSeq f, BVal bval,
                                         f32x16 (&acc)[COUT_T][NJ], const Carry &cin, FragSeq nf,
                                         Carry &cout) {
    // NJ: row tiles (JT; 1 for a block whose B is the same for every row, group_l1_6.hip x2)
    static_assert(COUT_T <= CARRY6 && NCOUT <= CARRY6, "carry");
    constexpr int NB = SAMEB ? 1 : NJ;
    u32x4 buf[2][COUT_T][3];
#pragma unroll
    for (int co = 0; co < COUT_T; ++co)
#pragma unroll
        for (int p = 0; p < 3; ++p) buf[0][co][p] = cin[co][p];
    auto split_jt = [&](int c, u32x4 (&bb)[NB][3]) {
#pragma unroll
        for (int jb = 0; jb < NB; ++jb) {
            float x[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = bval(jb, 8 * c + i);
            split8(x, bb[jb]);
        }
    };
    u32x4 b[2][NB][3];
    split_jt(0, b[0]);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) {
#pragma unroll
            for (int co = 0; co < COUT_T; ++co) ld6(wt, f.base + co * f.stride + c + 1, lane, buf[(c + 1) & 1][co]);
        } else {
#pragma unroll
            for (int co = 0; co < NCOUT; ++co) ld6(wt, nf.base + co * nf.stride, lane, cout[co]);
        }
        // keep the prefetch ahead of this chunk's MFMAs (LDS-resident tables, group_l1_6.hip: the
        // compiler otherwise sinks each ds_read next to its MFMA, 260 vs 173 us)
        if constexpr (is_lds_table<WP>::value) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int co = 0; co < COUT_T; ++co)
#pragma unroll
            for (int jt = 0; jt < NJ; ++jt)
                acc[co][jt] = mma6(buf[c & 1][co], b[c & 1][SAMEB ? 0 : jt], acc[co][jt]);
        if (c + 1 < NCH) {  // next chunk's split in this chunk's MFMA shadow (mfma_chain.h)
            split_jt(c + 1, b[(c + 1) & 1]);
            interleave_mfma_valu<6 * COUT_T * NJ, 48 * NB>();
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

template <int N>
__device__ __forceinline__ void zero_jt(f32x16 (&t)[N][JT]) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) t[i][jt] = zero16();
}

// folded BN (mfma_chain.h beta_tiles): both row tiles start from the layer's beta; the
// epilogue is the ReLU
template <int COUT_T>
__device__ __forceinline__ void beta_jt(const float *ab, int lane, f32x16 (&acc)[COUT_T][JT]) {
#pragma unroll
    for (int co = 0; co < COUT_T; ++co)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 b = *reinterpret_cast<const float4 *>(ab + COUT_T * 32 + co * 32 + 8 * r + 4 * (lane >> 5));
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) {
                acc[co][jt][4 * r] = b.x; acc[co][jt][4 * r + 1] = b.y;
                acc[co][jt][4 * r + 2] = b.z; acc[co][jt][4 * r + 3] = b.w;
            }
        }
}

template <int N>
__device__ __forceinline__ void relu_jt(f32x16 (&t)[N][JT]) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
#pragma unroll
            for (int q = 0; q < 16; ++q) t[i][jt][q] = relu_i(t[i][jt][q]);
}

}  // namespace hreg_jt
