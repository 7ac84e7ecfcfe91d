// mfma_chain.h -- building blocks of the fused group kernels (group_fused.hip,
// group_head.hip): v_mfma_f32_32x32x2_f32 chains whose A fragments stream from an
// L2-resident table one window ahead of use, BN/ReLU epilogues, tile stores.
#pragma once

#include "common.h"

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

// fragment f of call: index base + co * stride + step, in 64-float fragments.
// tt > 0 (workgroup rings only, ring_fill): output slot co of a step is tile co % tt at chunk
// step + (co / tt) * cs -- one step's slot then holds several chunks of the same tiles
// (group_fused6.hip, the batched x2 block).
struct FragSeq {
    int base, stride;
    int tt = 0, cs = 0;
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
    if constexpr (GS == 4) {
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

// Folded BN (the bf16x6 kernels): a layer's alpha is folded into its weight rows on the host
// (engine._fold_bn), so an output tile starts from the per-channel beta -- read from the
// [alpha C | beta C] epilogue section straight into the accumulators -- and the epilogue is
// the ReLU alone (1 VALU per value instead of zeroing + multiply + add + max).
template <int COUT_T>
__device__ __forceinline__ void beta_tiles(const float *ab, int lane, f32x16 (&acc)[COUT_T]) {
    load_tiles<COUT_T>(acc, ab + COUT_T * 32, lane >> 5);
}

// ReLU on the bit patterns: max_i32(x, 0) keeps every non-negative float and maps every
// negative one (and -0) to +0 -- one v_max_i32, where fmaxf(x, 0) on an MFMA result costs a
// NaN-canonicalising v_max_f32 x, x first
__device__ __forceinline__ float relu_i(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
// max of two non-negative floats (ReLU outputs) on the bit patterns
__device__ __forceinline__ float max_nonneg(float a, float b) {
    return __int_as_float(max(__float_as_int(a), __float_as_int(b)));
}

template <int N>
__device__ __forceinline__ void relu_tiles(f32x16 (&t)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) t[i][q] = relu_i(t[i][q]);
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

// sum / max over the 8 rows of a keypoint (8-lane DPP groups), result in all 8 lanes
__device__ __forceinline__ float grp8_sum(float v) {
    v = fadd_rn(v, dpp_all<0xb1>(v));
    v = fadd_rn(v, dpp_all<0x4e>(v));
    return fadd_rn(v, dpp_all<0x141>(v));
}
__device__ __forceinline__ float grp8_max_nonneg(float f) {
    int v = __float_as_int(f);
    v = max(v, dpp_all_i<0xb1>(v));
    v = max(v, dpp_all_i<0x4e>(v));
    return __int_as_float(max(v, dpp_all_i<0x141>(v)));
}

// PRE: the descriptor blocks of the first layer come precomputed per point --
// pre_src[g] = W_f f_src[g], pre_dst[n] = W_kf f_dst[n] ([*][N1], hreg_gemm) -- and
// initialise the accumulators (lane j, register q <- channel chan(co, q, h) of its
// row's two sources); only the 16 small columns run on the MFMA here.  Same sum up to
// fp32 order, 2C k-steps per row fewer (the reference repeats / gathers the
// descriptors into every row first, layers.py:444-445).
template <int N1, int T1>
__device__ __forceinline__ void init_from_rows(f32x16 (&acc)[T1], const float *__restrict__ u,
                                               const float *__restrict__ v, int h) {
#pragma unroll
    for (int co = 0; co < T1; ++co)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = co * 32 + 8 * r + 4 * h;
            const float4 a = *reinterpret_cast<const float4 *>(u + c);
            if (v) {
                const float4 b = *reinterpret_cast<const float4 *>(v + c);
                acc[co][4 * r] = fadd_rn(a.x, b.x); acc[co][4 * r + 1] = fadd_rn(a.y, b.y);
                acc[co][4 * r + 2] = fadd_rn(a.z, b.z); acc[co][4 * r + 3] = fadd_rn(a.w, b.w);
            } else {
                acc[co][4 * r] = a.x; acc[co][4 * r + 1] = a.y;
                acc[co][4 * r + 2] = a.z; acc[co][4 * r + 3] = a.w;
            }
        }
}

// ------------------------------------------------------------------------
// fp32-accurate products on the bf16 matrix cores ("bf16x6").  Every fp32 value is
// split exactly into three bf16 pieces, x = hi + mid + lo (truncation split: hi =
// the top 8 significant bits, mid the next 8 of x - hi, lo the remaining <= 8 bits;
// exact for normal fp32), and a product a*b is accumulated as the six piece
// products down to 2^-16 relative (a_h b_h, a_h b_m, a_m b_h, a_h b_l, a_m b_m,
// a_l b_h; the dropped ones are <= 2^-24 relative), smallest first, in fp32 on
// v_mfma_f32_32x32x16_bf16.  Measured (profiles/r2_split_mfma_micro.txt): the same
// error vs fp64 as the f32-input MFMA (max 1.3e-7..1.8e-7 of sum|a b| at K = 32..512)
// at 2.0-2.2x its throughput in an accumulator-chained layer stack (6 x 32 cycles
// per 16-deep k-chunk instead of 8 x 64).
//
// Operand layout: v_mfma_f32_32x32x16_bf16 lane l holds A[l % 32][8 (l / 32) + i]
// and B[8 (l / 32) + i][l % 32], i = 0..7, and its accumulator is laid out as the
// f32 32x32x2 one.  A 16-deep chunk c therefore holds exactly the f32 k-steps
// 8c .. 8c + 7 of each lane: bval(st) of the f32 pipes is reused unchanged, and
// the weight pieces of chunk c are the lane's f32 fragments 8c .. 8c + 7
// (engine.frag6), 3 x 16 bytes per lane.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

// 8 fp32 values (one lane's chunk of B) -> hi / mid / lo packed bf16x8
__device__ __forceinline__ void split8(const float (&x)[8], u32x4 (&o)[3]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t hb[2], mb[2], lb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float v = x[2 * i + j];
            const uint32_t xb = __float_as_uint(v);
            const float r = fsub_rn(v, __uint_as_float(xb & 0xffff0000u));
            const uint32_t rb = __float_as_uint(r);
            hb[j] = xb;
            mb[j] = rb;
            lb[j] = __float_as_uint(fsub_rn(r, __uint_as_float(rb & 0xffff0000u)));
        }
        o[0][i] = __builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u);
        o[1][i] = __builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u);
        o[2][i] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
    }
}

__device__ __forceinline__ f32x16 mfma16(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// c += A x B for one 16-deep chunk as the six piece products, smallest first
__device__ __forceinline__ f32x16 mma6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
    c = mfma16(a[0], b[2], c);
    c = mfma16(a[1], b[1], c);
    c = mfma16(a[2], b[0], c);
    c = mfma16(a[0], b[1], c);
    c = mfma16(a[1], b[0], c);
    return mfma16(a[0], b[0], c);
}

constexpr int CARRY6 = 8;  // output tiles of a call's first chunk carried between calls

// weight pieces of chunk fragment f (units of 3 x 64 lanes x 16 B)
// (signed pointer arithmetic: a wave-uniform f stays an SGPR base, the lane a VGPR offset,
// the piece an immediate -- no per-fragment VGPR address to hoist and spill)
__device__ __forceinline__ void ld6(const gu32x4 *__restrict__ wt, int f, int lane, u32x4 (&o)[3]) {
    const gu32x4 *fp = wt + f * 192;
#pragma unroll
    for (int p = 0; p < 3; ++p) o[p] = fp[p * 64 + lane];
}

// Software-pipelined split: chunk c + 1's B operand is split into its pieces while chunk c's
// MFMAs run, the scheduler asked (sched_group_barrier) to place about NVALU / NMFMA VALU
// instructions after each MFMA -- an MFMA holds the SIMD's vector issue for 8 of its 32 cycles,
// so ~5 independent VALU per 32x32x16 MFMA issue in its shadow instead of as a 44-instruction
// block between two MFMAs (measured neutral, +-2 %, r2; kept).

template <int NMFMA, int NVALU>
__device__ __forceinline__ void interleave_mfma_valu() {
    constexpr int V = (NVALU + NMFMA - 1) / NMFMA;
#pragma unroll
    for (int k = 0; k < NMFMA; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, V, 0);  // then V VALU
    }
}

template <class BVal>
__device__ __forceinline__ void split_chunk(BVal bval, int c, u32x4 (&b)[3]) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = bval(8 * c + i);
    split8(x, b);
}

// acc[co] += sum_{c < NCH} A(co, c) x B(c) with B(c) = split(bval(8c .. 8c+7)); chunk
// fragment (co, c) = f.base + co * f.stride + c.  cin: this call's first chunk (all
// COUT_T tiles), loaded by the previous call; cout: the first chunk of the next call
// nf (NCOUT tiles).  Weight pieces stream one chunk ahead of their MFMAs.
// ROLL (default for >= 4 output tiles): one buffer; tile co's next chunk is loaded right
// after its 6 MFMAs issue (COUT_T - 1 tiles = 18+ MFMAs of lead), 12 VGPRs per tile
// instead of 24 for the double buffer.
template <int NCH, int COUT_T, int NCOUT, class BVal, bool ROLL = (COUT_T >= 4)>
__device__ __forceinline__ void mfma_pipe6(const gu32x4 *__restrict__ wt, int lane, FragSeq f, BVal bval,
                                           f32x16 (&acc)[COUT_T], const u32x4 (&cin)[CARRY6][3],
                                           FragSeq nf, u32x4 (&cout)[CARRY6][3]) {
    static_assert(COUT_T <= CARRY6 && NCOUT <= CARRY6, "carry");
    if constexpr (ROLL) {
        u32x4 rb[COUT_T][3];
#pragma unroll
        for (int co = 0; co < COUT_T; ++co)
#pragma unroll
            for (int p = 0; p < 3; ++p) rb[co][p] = cin[co][p];
        u32x4 bs[2][3];
        split_chunk(bval, 0, bs[0]);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
#pragma unroll
            for (int co = 0; co < COUT_T; ++co) {
                acc[co] = mma6(rb[co], bs[c & 1], acc[co]);
                if (c + 1 < NCH)
                    ld6(wt, f.base + co * f.stride + c + 1, lane, rb[co]);
                else if (co < NCOUT)
                    ld6(wt, nf.base + co * nf.stride, lane, cout[co]);
            }
            if (c + 1 < NCH) {
                split_chunk(bval, c + 1, bs[(c + 1) & 1]);
                interleave_mfma_valu<6 * COUT_T, 48>();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int co = COUT_T; co < NCOUT; ++co) ld6(wt, nf.base + co * nf.stride, lane, cout[co]);
        return;
    }
    u32x4 buf[2][COUT_T][3];
#pragma unroll
    for (int co = 0; co < COUT_T; ++co)
#pragma unroll
        for (int p = 0; p < 3; ++p) buf[0][co][p] = cin[co][p];
    u32x4 bs[2][3];
    split_chunk(bval, 0, bs[0]);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) {
#pragma unroll
            for (int co = 0; co < COUT_T; ++co) ld6(wt, f.base + co * f.stride + c + 1, lane, buf[(c + 1) & 1][co]);
        } else {
#pragma unroll
            for (int co = 0; co < NCOUT; ++co) ld6(wt, nf.base + co * nf.stride, lane, cout[co]);
        }
#pragma unroll
        for (int co = 0; co < COUT_T; ++co) acc[co] = mma6(buf[c & 1][co], bs[c & 1], acc[co]);
        if (c + 1 < NCH) {
            split_chunk(bval, c + 1, bs[(c + 1) & 1]);
            interleave_mfma_valu<6 * COUT_T, 48>();
        }
        // no barrier after the last chunk -- the next call's ReLU + first split (which waits
        // only for tile 0's result) may issue under this chunk's last MFMAs
        if (c + 1 < NCH) __builtin_amdgcn_sched_barrier(0);
    }
}

// ------------------------------------------------------------------------
// Workgroup-shared weight stream (group_fused6.hip, level 2): the 4 waves of a workgroup
// run the same chunk sequence on different row tiles, so each step's weight pieces are
// brought into LDS ONCE per workgroup by LDS-DMA (global_load_lds_dwordx4, the 3 x NCO
// pieces of a step spread over the waves) and every wave reads them with ds_read_b128 --
// a quarter of the vector-memory return traffic of per-wave streams (the texture-data
// return unit was ~87 % busy).  Two slots: the DMA of step s + 1 is issued right after the
// barrier that opens step s (every wave's DMA of step s landed: vmcnt(0) before it; every
// wave has finished reading step s - 1's slot).  Every wave must run the same steps.
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) const u32x4 lds_cu32x4;

// (measured neutral and removed, r2: chunk c + 1's B split in the shadow of tile 0's MFMAs of
// chunk c; tile co + 1's pieces read right before its MFMAs instead of under tile co's)

template <int SLOT_TILES, int NWAVES>
struct Ring6 {
    static constexpr int SLOT = SLOT_TILES * 192;  // u32x4 per slot
    const gu32x4 *wt;   // the table (global)
    lds_u32x4 *lds;     // 2 slots
    int step, w;        // uniform: steps so far, this wave's index in the workgroup
};

template <int NCO, class R>
__device__ __forceinline__ void ring_fill(R &ring, int slot, FragSeq f, int c, int lane) {
    static_assert(NCO * 192 <= R::SLOT, "slot");
    constexpr int NP = 3 * NCO;
#pragma unroll
    for (int i0 = 0; i0 < NP; i0 += 4) {
        const int i = i0 + ring.w;  // piece i = co * 3 + p of this wave
        if (i < NP) {
            const int co = i / 3, p = i - 3 * co;
            const int fi = f.tt ? f.base + (co % f.tt) * f.stride + c + (co / f.tt) * f.cs : f.base + co * f.stride + c;
            const gu32x4 *src = ring.wt + fi * 192 + p * 64 + lane;
#if __HIP_DEVICE_COMPILE__  // (the gfx950 builtin does not exist in the host pass)
            __builtin_amdgcn_global_load_lds(src, ring.lds + slot * R::SLOT + i * 64, 16, 0, 0);
#else
            (void)src;
#endif
        }
    }
}

template <int NCH, int COUT_T, int NCOUT, class BVal, int ST, int NWV>
__device__ __forceinline__ void mfma_pipe6(Ring6<ST, NWV> &ring, int lane, FragSeq f, BVal bval,
                                           f32x16 (&acc)[COUT_T], const u32x4 (&)[CARRY6][3], FragSeq nf,
                                           u32x4 (&)[CARRY6][3]) {
    static_assert(NWV == 4, "4 waves share the stream");
    u32x4 b[3];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of this step landed
        __syncthreads();
        const int cur = ring.step & 1;
        if (c + 1 < NCH)
            ring_fill<COUT_T>(ring, cur ^ 1, f, c + 1, lane);
        else
            ring_fill<NCOUT>(ring, cur ^ 1, nf, 0, lane);
        split_chunk(bval, c, b);
        const lds_cu32x4 *sp = ring.lds + cur * Ring6<ST, NWV>::SLOT + lane;
        // tile co + 1's pieces are read while tile co's six MFMAs run (one tile of pieces
        // in flight: 12 VGPRs, not the whole step's)
        u32x4 a[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[0][p] = sp[p * 64];
#pragma unroll
        for (int co = 0; co < COUT_T; ++co) {
            if (co + 1 < COUT_T) {
#pragma unroll
                for (int p = 0; p < 3; ++p) a[(co + 1) & 1][p] = sp[((co + 1) * 3 + p) * 64];
            }
            acc[co] = mma6(a[co & 1], b, acc[co]);
            __builtin_amdgcn_sched_barrier(0);
        }
        ++ring.step;
    }
}

}  // namespace hreg_chain
