// split_chain.h -- building blocks of the channel-split kernels (group_split.hip,
// mlp_head.hip): a row tile's activations live in LDS (row-major, natural channel
// order); each wave computes P output tiles of a layer with
// v_mfma_f32_32x32x2_f32, A fragments streamed from the L2-resident table one
// window ahead, B streamed from LDS.
#pragma once

#include "mfma_chain.h"

namespace hreg_split {

using namespace hreg_chain;

__device__ __forceinline__ void tile_sync() { __syncthreads(); }

constexpr int SCARRY = 32;
constexpr int SWIN = 16;  // k-steps per window (P <= 2 tiles: <= 32 fragments in flight)

// acc[P] += sum_{st < NSTEP} A(co0 + i, st) x B(st): A fragments from the table
// (grouped 4 k-steps per lane; GS = 2 for a 2-step call), B from LDS through
// bl(st0, v) (GS consecutive k-steps).  cin: this call's first window of A
// fragments (loaded by the previous call); cout: the first window (NWIN steps x NP
// tiles) of the next call nf.  The first B window is read at entry (it is the
// output of the barrier just passed); later windows one window ahead.
template <int NSTEP, int P, int NP, int NWIN, int WMAX = SWIN, class BL>
__device__ __forceinline__ void pipe_lds(const gfloat *__restrict__ wf, int lane, FragSeq f, BL bl,
                                         f32x16 (&acc)[P], const float (&cin)[SCARRY], FragSeq nf,
                                         float (&cout)[SCARRY]) {
    constexpr int WIN = NSTEP < WMAX ? NSTEP : WMAX;
    constexpr int GS = WIN < 4 ? WIN : 4, NGS = NWIN < 4 ? NWIN : 4;
    static_assert(NSTEP % WIN == 0 && WIN % GS == 0 && NWIN % NGS == 0, "window");
    static_assert(WIN * P <= SCARRY && NWIN * NP <= SCARRY, "carry");
    constexpr int NW = NSTEP / WIN;
    float abuf[2][WIN][P];
    float bbuf[2][WIN];
#pragma unroll
    for (int s = 0; s < WIN; ++s)
#pragma unroll
        for (int co = 0; co < P; ++co) abuf[0][s][co] = cin[s * P + co];
#pragma unroll
    for (int s0 = 0; s0 < WIN; s0 += GS) {
        float v[GS];
        bl(s0, v);
#pragma unroll
        for (int i = 0; i < GS; ++i) bbuf[0][s0 + i] = v[i];
    }
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (w + 1 < NW) {
#pragma unroll
            for (int s0 = 0; s0 < WIN; s0 += GS) {
#pragma unroll
                for (int co = 0; co < P; ++co) {
                    float v[GS];
                    ldgroup<GS>(wf, f.base + co * f.stride + (w + 1) * WIN + s0, lane, v);
#pragma unroll
                    for (int i = 0; i < GS; ++i) abuf[(w + 1) & 1][s0 + i][co] = v[i];
                }
                float v[GS];
                bl((w + 1) * WIN + s0, v);
#pragma unroll
                for (int i = 0; i < GS; ++i) bbuf[(w + 1) & 1][s0 + i] = v[i];
            }
        } else {
#pragma unroll
            for (int s0 = 0; s0 < NWIN; s0 += NGS)
#pragma unroll
                for (int co = 0; co < NP; ++co) {
                    float v[NGS];
                    ldgroup<NGS>(wf, nf.base + co * nf.stride + s0, lane, v);
#pragma unroll
                    for (int i = 0; i < NGS; ++i) cout[(s0 + i) * NP + co] = v[i];
                }
        }
#pragma unroll
        for (int s = 0; s < WIN; ++s)
#pragma unroll
            for (int co = 0; co < P; ++co)
                acc[co] = __builtin_amdgcn_mfma_f32_32x32x2f32(abuf[w & 1][s][co], bbuf[w & 1][s],
                                                               acc[co], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int NSTEP>
constexpr int swin() { return NSTEP < SWIN ? NSTEP : SWIN; }

// The same on the bf16 matrix cores at fp32 accuracy (bf16x6, mfma_chain.h): acc[P] +=
// sum_{c < NCH} A(co0 + i, c) x split(B(8c .. 8c+7)).  A: bf16 piece chunk fragments from
// the table (fragment f.base + i * f.stride + c, one chunk ahead, double-buffered); B: 8
// f32 k-steps per chunk read from LDS through bl(st0, v[4]) (two calls, one chunk ahead)
// and split into pieces in registers.  cin: this call's first chunk (P tiles), loaded by
// the previous call; cout: the first chunk of the next call nf (NP tiles).
typedef u32x4 Carry6[CARRY6][3];

template <int NCH, int P, int NP, class BL>
__device__ __forceinline__ void pipe_lds6(const gu32x4 *__restrict__ wt, int lane, FragSeq f, BL bl,
                                          f32x16 (&acc)[P], const Carry6 &cin, FragSeq nf, Carry6 &cout) {
    static_assert(P <= CARRY6 && NP <= CARRY6, "carry");
    u32x4 abuf[2][P][3];
    float bb[2][8];
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) abuf[0][i][p] = cin[i][p];
    {
        float v[4];
        bl(0, v);
#pragma unroll
        for (int k = 0; k < 4; ++k) bb[0][k] = v[k];
        bl(4, v);
#pragma unroll
        for (int k = 0; k < 4; ++k) bb[0][4 + k] = v[k];
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) {
#pragma unroll
            for (int i = 0; i < P; ++i) ld6(wt, f.base + i * f.stride + c + 1, lane, abuf[(c + 1) & 1][i]);
            float v[4];
            bl(8 * (c + 1), v);
#pragma unroll
            for (int k = 0; k < 4; ++k) bb[(c + 1) & 1][k] = v[k];
            bl(8 * (c + 1) + 4, v);
#pragma unroll
            for (int k = 0; k < 4; ++k) bb[(c + 1) & 1][4 + k] = v[k];
        } else {
#pragma unroll
            for (int i = 0; i < NP; ++i) ld6(wt, nf.base + i * nf.stride, lane, cout[i]);
        }
        u32x4 b[3];
        split8(bb[c & 1], b);
#pragma unroll
        for (int i = 0; i < P; ++i) acc[i] = mma6(abuf[c & 1][i], b, acc[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// pipe_lds6 over JT row tiles: each chunk's weight pieces (P tiles) feed the MFMAs of
// every row tile (JT x fewer weight bytes per MFMA); B of row tile jt through bl(jt, st0, v).
// SWP: chunk c + 1's B split under chunk c's MFMAs (r5: the CoarseReg / FineReg / neighbour
// heads 127.8 / 56.4 / 66.4 -> 123.5 / 54.2 / 64.4 us; level 3 174 -> 175, so not there).
template <int NCH, int P, int NP, int JT, bool SWP, class BL>
__device__ __forceinline__ void pipe_lds6_jt(const gu32x4 *__restrict__ wt, int lane, FragSeq f, BL bl,
                                             f32x16 (&acc)[P][JT], const Carry6 &cin, FragSeq nf, Carry6 &cout) {
    static_assert(P <= CARRY6 && NP <= CARRY6, "carry");
    u32x4 abuf[2][P][3];
    float bb[2][JT][8];
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p) abuf[0][i][p] = cin[i][p];
    auto ldb = [&](int c, float (&d)[JT][8]) {
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            float v[4];
            bl(jt, 8 * c, v);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[jt][k] = v[k];
            bl(jt, 8 * c + 4, v);
#pragma unroll
            for (int k = 0; k < 4; ++k) d[jt][4 + k] = v[k];
        }
    };
    ldb(0, bb[0]);
    if constexpr (SWP) {
        // chunk c + 1's B split in chunk c's MFMA shadow (mfma_chain.h), the VALU
        // placed between the MFMAs by sched_group_barrier
        u32x4 bs[2][JT][3];
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) split8(bb[0][jt], bs[0][jt]);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c + 1 < NCH) {
#pragma unroll
                for (int i = 0; i < P; ++i) ld6(wt, f.base + i * f.stride + c + 1, lane, abuf[(c + 1) & 1][i]);
                ldb(c + 1, bb[(c + 1) & 1]);
            } else {
#pragma unroll
                for (int i = 0; i < NP; ++i) ld6(wt, nf.base + i * nf.stride, lane, cout[i]);
            }
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int i = 0; i < P; ++i) acc[i][jt] = mma6(abuf[c & 1][i], bs[c & 1][jt], acc[i][jt]);
            if (c + 1 < NCH) {
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) split8(bb[(c + 1) & 1][jt], bs[(c + 1) & 1][jt]);
                interleave_mfma_valu<6 * P * JT, 44 * JT>();
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) {
#pragma unroll
            for (int i = 0; i < P; ++i) ld6(wt, f.base + i * f.stride + c + 1, lane, abuf[(c + 1) & 1][i]);
            ldb(c + 1, bb[(c + 1) & 1]);
        } else {
#pragma unroll
            for (int i = 0; i < NP; ++i) ld6(wt, nf.base + i * nf.stride, lane, cout[i]);
        }
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            u32x4 b[3];
            split8(bb[c & 1][jt], b);
#pragma unroll
            for (int i = 0; i < P; ++i) acc[i][jt] = mma6(abuf[c & 1][i], b, acc[i][jt]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// BN/ReLU epilogue of output tiles co0 .. co0+P-1 of a C-channel layer
template <int P, int C>
__device__ __forceinline__ void epi(const float *ab, int co0, int h, f32x16 (&acc)[P]) {
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = chan(co0 + i, q, h);
            acc[i][q] = fmaxf(fadd_rn(fmul_rn(acc[i][q], ab[c]), ab[C + c]), 0.f);
        }
}

// folded BN (mfma_chain.h beta_tiles): output tiles co0 .. co0+P-1 of a C-channel layer
// start from the layer's beta ([alpha C | beta C] section)
template <int P, int C>
__device__ __forceinline__ void beta_p(const float *ab, int co0, int h, f32x16 (&acc)[P]) {
    load_tiles<P>(acc, ab + C + co0 * 32, h);
}

// tile co of an activation (channels chan(co, q, h), row j) into a row-major LDS buffer
template <int LDSW>
__device__ __forceinline__ void put_tile(float *buf, int co, int j, int h, const f32x16 &v) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float4 *>(buf + j * LDSW + co * 32 + 8 * r + 4 * h) =
            make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
}

// ChanB over JT row tiles of 32 rows (row tile jt = rows 32 jt .. 32 jt + 31 of the buffer)
template <int LDSW>
struct ChanBJ {
    const float *row;  // buf + j * LDSW
    int h;
    __device__ __forceinline__ void operator()(int jt, int st0, float (&v)[4]) const {
        const int ct = st0 >> 4, r = (st0 & 15) >> 2;
        const float4 t = *reinterpret_cast<const float4 *>(row + jt * 32 * LDSW + ct * 32 + 8 * r + 4 * h);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    }
};

// B loader for a chained layer input: k-step st = ct*16 + q <-> channel chan(ct, q, h)
struct ChanB {
    const float *row;  // buf + j * LDSW
    int h;
    __device__ __forceinline__ void operator()(int st0, float (&v)[4]) const {
        const int ct = st0 >> 4, r = (st0 & 15) >> 2;
        const float4 t = *reinterpret_cast<const float4 *>(row + ct * 32 + 8 * r + 4 * h);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    }
};

}  // namespace hreg_split
