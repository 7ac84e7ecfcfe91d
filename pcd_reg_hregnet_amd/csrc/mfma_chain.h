// mfma_chain.h -- building blocks of the fused group kernels (group_fused.hip,
// group_head.hip): v_mfma_f32_32x32x2_f32 chains whose A fragments stream from an
// L2-resident table one window ahead of use, BN/ReLU epilogues, tile stores.
#pragma once

#include "common.h"

// tools/l2_experiment.py builds variants: 1 = no epilogue / reductions (MFMA +
// loads only), 2 = additionally no weight loads (MFMA issue structure only),
// 3 = feature rows read without the kNN indirection (no dependent gather)
#ifndef HREG_L2_EXP
#define HREG_L2_EXP 0
#endif

namespace hreg_chain {

typedef float f32x16 __attribute__((ext_vector_type(16)));
// global address space: loads through it are global_load (vmcnt-ordered), not flat
typedef __attribute__((address_space(1))) const float gfloat;

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
    return z;
}

__device__ __forceinline__ int chan(int co, int q, int h) {
    return co * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
}

// ------------------------------------------------------------------------
// The A fragments of one group form a fixed sequence of ~1032 loads.  They are
// streamed one window ahead of the MFMAs that use them -- across layer
// boundaries too: the last window of each call loads the first window of the
// next call (into `carry`), and the last call of a group the first window of
// the next group, so no call starts on a cold L2 round trip.

constexpr int CARRY = 16;  // max WIN * COUT_T

// fragment f of call: index base + co * stride + step, in 64-float fragments
struct FragSeq {
    int base, stride;
};

template <int COUT_T>
constexpr int win_for() { return COUT_T >= 8 ? 2 : COUT_T >= 4 ? 4 : 8; }
template <int NSTEP, int COUT_T>
constexpr int first_win() { return NSTEP < win_for<COUT_T>() ? NSTEP : win_for<COUT_T>(); }

// Fragments are stored in groups of GS = min(4, window) consecutive k-steps with
// the steps innermost per lane ([step group][lane][GS], engine.l2_table), so one
// global_load_dwordx4 (x2) brings a lane its A values for 4 (2) k-steps: 4x fewer
// vector-memory instructions than one dword per MFMA.  Address: uniform fragment
// base (SGPR pair) + the lane's byte offset.
template <int GS>
__device__ __forceinline__ void ldgroup(const gfloat *__restrict__ wf, int f0, int lane, float (&v)[GS]) {
    if constexpr (HREG_L2_EXP == 2) {
        // opaque register values: no load, nothing the compiler can hoist or fold
#pragma unroll
        for (int i = 0; i < GS; ++i) {
            float x = __int_as_float(lane);
            asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x));
            v[i] = x;
        }
    } else if constexpr (GS == 4) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const v4f gv4f;
        const v4f t = *reinterpret_cast<const gv4f *>(wf + f0 * 64 + (unsigned)lane * 4);
        v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
        static_assert(GS == 2, "group size");
        typedef float v2f __attribute__((ext_vector_type(2)));
        typedef __attribute__((address_space(1))) const v2f gv2f;
        const v2f t = *reinterpret_cast<const gv2f *>(wf + f0 * 64 + (unsigned)lane * 2);
        v[0] = t[0]; v[1] = t[1];
    }
}

// acc[co] += sum_{st < NSTEP} A(co, st) x bval(st) on v_mfma_f32_32x32x2_f32.
// cin: this call's first window (loaded by the previous call); cout: receives the
// first window (NWIN steps x NCOUT tiles) of the next call `nf`.
template <int NSTEP, int COUT_T, int NCOUT, int NWIN, class BVal>
__device__ __forceinline__ void mfma_pipe(const gfloat *__restrict__ wf, int lane, FragSeq f, BVal bval,
                                          f32x16 (&acc)[COUT_T], const float (&cin)[CARRY],
                                          FragSeq nf, float (&cout)[CARRY]) {
    constexpr int WIN = first_win<NSTEP, COUT_T>();
    constexpr int GS = WIN < 4 ? WIN : 4, NGS = NWIN < 4 ? NWIN : 4;
    static_assert(NSTEP % WIN == 0 && WIN % GS == 0 && NWIN % NGS == 0, "window");
    static_assert(WIN * COUT_T <= CARRY && NWIN * NCOUT <= CARRY, "carry");
    constexpr int NW = NSTEP / WIN;
    // two fragment buffers used alternately (window index is compile-time: no copies)
    float buf[2][WIN][COUT_T];
#pragma unroll
    for (int s = 0; s < WIN; ++s)
#pragma unroll
        for (int co = 0; co < COUT_T; ++co) buf[0][s][co] = cin[s * COUT_T + co];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (w + 1 < NW) {
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
__device__ __forceinline__ void epilogue(const float *ab, int lane, f32x16 (&acc)[COUT_T]) {
    if (HREG_L2_EXP) return;
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

// accumulator tiles initialised from a per-row vector (this lane's row): register q of
// tile co <- row[chan(co, q, h)] (4 float4 loads per tile).  Used for first-layer blocks
// precomputed once per source point (W_f f_n, gathered by the row's neighbour index).
template <int T>
__device__ __forceinline__ void load_tiles(f32x16 (&acc)[T], const float *__restrict__ row, int h) {
#pragma unroll
    for (int co = 0; co < T; ++co)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 a = *reinterpret_cast<const float4 *>(row + co * 32 + 8 * r + 4 * h);
            acc[co][4 * r] = a.x; acc[co][4 * r + 1] = a.y;
            acc[co][4 * r + 2] = a.z; acc[co][4 * r + 3] = a.w;
        }
}

template <int N>
__device__ __forceinline__ void zero_tiles(f32x16 (&t)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) t[i] = zero16();
}

// one channel tile of a per-group result reduced over the rows (valid in the writer
// lanes): channels co*32 + 8r + 4h + {0..3} for registers q = 4r..4r+3 -> 4 float4 stores
__device__ __forceinline__ void store_tile(float *out, int co, const f32x16 &v, bool writer, int h) {
    if (writer) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            *reinterpret_cast<float4 *>(out + co * 32 + 8 * r + 4 * h) =
                make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
    }
}

}  // namespace hreg_chain
