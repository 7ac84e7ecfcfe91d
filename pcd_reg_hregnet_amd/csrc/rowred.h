// rowred.h -- reductions over the rows of an MFMA accumulator tile, many values at once.
//
// A 32x32 accumulator tile holds row j of a group in lane j (+32 h) and 16 channel values
// per lane.  Reducing every channel over the rows one value at a time costs one DPP step per
// value per lane bit (5 for 32 rows, plus the cross-row step and a broadcast).  Reducing N
// values together as a butterfly halves the number of values at each of the first levels:
// the lanes whose bit b is 0 keep the pair-reduced value a, the others value b, so the next
// level works on half as many registers:
//   bit 4 (lane ^ 16): v_permlane16_swap (gfx950) exchanges the odd DPP rows of one register
//                      with the even rows of the other -- 1 swap + 1 op per pair;
//   bit 3 / bit 2:     row_mirror / row_half_mirror pair every lane with one of opposite bit
//                      -- 2 DPP-fused ops + 1 v_cndmask per pair;
//   bits 1, 0:         quad_perm full reductions on the N/8 (N/4) values left.
// 32 rows, N = 16: 38 VALU instead of 96 (16 x 6); the broadcast back (bcast32) is the
// inverse butterfly, 34 VALU instead of 48.
//
// After bfly32<N> slot i (i < N/8) of lane l holds value i + (N/8)(b2 + 2 b3 + 4 b4),
// b = bits of l (the four lanes of a quad agree); after bfly16<N> (16-row groups = DPP
// rows) slot i (i < N/4) holds value i + (N/4)(b2 + 2 b3).  Sums are reduced as a tree in
// that order (same fp32 rounding as any other pairwise order: one add per level).
#pragma once

#include "common.h"

namespace hreg_rowred {

// max of non-negative floats (ReLU outputs) on the bit patterns (v_max_i32, no NaN
// canonicalisation); op with the DPP-moved value fuses into v_max_i32_dpp
struct MaxNN {
    __device__ static __forceinline__ float op(float a, float b) {
        return __int_as_float(max(__float_as_int(a), __float_as_int(b)));
    }
    template <int CTRL>
    __device__ static __forceinline__ float dop(float v) {
        const int x = __float_as_int(v);
        return __int_as_float(max(x, dpp_all_i<CTRL>(x)));
    }
};
struct Sum {
    __device__ static __forceinline__ float op(float a, float b) { return fadd_rn(a, b); }
    template <int CTRL>
    __device__ static __forceinline__ float dop(float v) { return fadd_rn(v, dpp_all<CTRL>(v)); }
};

// lane bit 4: pairs (v[i], v[i + M]) -> v[i]
template <int M, class Op, int N>
__device__ __forceinline__ void lvl_swap16(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + M]), false,
                                                        false);
        v[i] = Op::op(__uint_as_float(r[0]), __uint_as_float(r[1]));
    }
}

// lane bit BIT through the mirror control CTRL (its pairs differ in BIT): pairs (v[i], v[i + M]) -> v[i]
template <int M, int CTRL, int BIT, class Op, int N>
__device__ __forceinline__ void lvl_mirror(float (&v)[N], int lane) {
    const bool hi = lane & (1 << BIT);
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const float ta = Op::template dop<CTRL>(v[i]);
        const float tb = Op::template dop<CTRL>(v[i + M]);
        v[i] = hi ? tb : ta;
    }
}

template <int M, class Op, int N>
__device__ __forceinline__ void lvl_quads(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < M; ++i) v[i] = Op::template dop<0xb1>(Op::template dop<0x4e>(v[i]));
}

// reduce N values over the 32 rows of each wave half (lane bits 0..4)
template <class Op, int N>
__device__ __forceinline__ void bfly32(float (&v)[N], int lane) {
    static_assert(N % 8 == 0, "N");
    lvl_swap16<N / 2, Op>(v);
    lvl_mirror<N / 4, 0x140, 3, Op>(v, lane);
    lvl_mirror<N / 8, 0x141, 2, Op>(v, lane);
    lvl_quads<N / 8, Op>(v);
}

// reduce N values over the 16 rows of each DPP row (lane bits 0..3)
template <class Op, int N>
__device__ __forceinline__ void bfly16(float (&v)[N], int lane) {
    static_assert(N % 4 == 0, "N");
    lvl_mirror<N / 2, 0x140, 3, Op>(v, lane);
    lvl_mirror<N / 4, 0x141, 2, Op>(v, lane);
    lvl_quads<N / 4, Op>(v);
}

// inverse of lvl_mirror: slots [0, M) -> [0, 2M), every lane
template <int M, int CTRL, int BIT, int N>
__device__ __forceinline__ void unmirror(float (&v)[N], int lane) {
    const bool hi = lane & (1 << BIT);
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const float own = v[i], t = dpp_all<CTRL>(own);
        v[i] = hi ? t : own;
        v[i + M] = hi ? own : t;
    }
}

// bfly32's result back in every lane: v[0 .. N) = the N reduced values
template <int N>
__device__ __forceinline__ void bcast32(float (&v)[N], int lane) {
    unmirror<N / 8, 0x141, 2>(v, lane);
    unmirror<N / 4, 0x140, 3>(v, lane);
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
        const uint32_t x = __float_as_uint(v[i]);
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        v[i] = __uint_as_float(r[0]);
        v[i + N / 2] = __uint_as_float(r[1]);
    }
}

// value index (tile co, register q: co * 16 + q) of bfly32 slot i in lane l; of bfly16
template <int N>
__device__ __forceinline__ int slot32(int i, int lane) {
    return i + (N / 8) * ((lane >> 2) & 7);
}
template <int N>
__device__ __forceinline__ int slot16(int i, int lane) {
    return i + (N / 4) * ((lane >> 2) & 3);
}

// store the reduced values of NT accumulator tiles (tiles co0 .. co0 + NT - 1 of a per-group
// row, channel chan(co, q, h)) from their slots: S consecutive slots are consecutive
// channels (S = 2 or 4: one float2 / float4 per writer lane and group of slots)
template <int N, bool R32>
__device__ __forceinline__ void store_slots(float *out, int co0, const float (&v)[N], int lane) {
    constexpr int NS = R32 ? N / 8 : N / 4;  // slots per lane
    constexpr int S = NS < 4 ? NS : 4;       // slots per store
    static_assert(NS % S == 0 && (S == 2 || S == 4), "slots");
    if (lane & 3) return;
    const int h = (lane >> 5) & 1;
#pragma unroll
    for (int i0 = 0; i0 < NS; i0 += S) {
        const int vi = R32 ? slot32<N>(i0, lane) : slot16<N>(i0, lane);
        const int co = co0 + (vi >> 4), q = vi & 15;
        float *p = out + co * 32 + 8 * (q >> 2) + 4 * h + (q & 3);
        if constexpr (S == 4)
            *reinterpret_cast<float4 *>(p) = make_float4(v[i0], v[i0 + 1], v[i0 + 2], v[i0 + 3]);
        else
            *reinterpret_cast<float2 *>(p) = make_float2(v[i0], v[i0 + 1]);
    }
}

// one accumulator tile's 16 values reduced over the rows of a KN-row group (KN = 32: a wave
// half; 16: a DPP row) and stored as channels co * 32 .. co * 32 + 31 of the group's row
template <int KN, class Op>
__device__ __forceinline__ void reduce_store(float *out, int co, float (&v)[16], int lane) {
    static_assert(KN == 32 || KN == 16, "group rows");
    if constexpr (KN == 32) {
        bfly32<Op>(v, lane);
        store_slots<16, true>(out, co, v, lane);
    } else {
        bfly16<Op>(v, lane);
        store_slots<16, false>(out, co, v, lane);
    }
}

}  // namespace hreg_rowred
