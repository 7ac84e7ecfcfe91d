// fps.hip -- farthest point sampling (plain and weighted) for gfx950.
//
// Replaces furthest_point_sampling_kernel / weighted_furthest_point_sampling_kernel
// (reference models/PointUtils/src/furthest_point_sampling_gpu.cu:84-206, :254-375).
// Not a translation: one workgroup per cloud keeps every point, its running
// minimum distance ("temp") and its weight in VGPRs for all m-1 dependent
// iterations (no HBM traffic inside the loop).
//
// The reference winner ("FPS tie rule"): with bs =
// opt_n_threads(n) "threads" (cuda_utils.h:22-26), reference thread r scans
// k = r, r+bs, ... keeping the first strictly larger d2 (.cu:132-133); the
// shared-memory tree keeps the lower slot on ties (.cu:75-80), so among equal
// maxima the thread with the smallest bit-reversed id wins, then the smallest
// k.  Here reference thread r = bitrev_L(r') is handled by our thread r'/G
// (slot g = r' % G) and its points k = r + i*bs sit in slots g*QT + i, so the
// order (thread, slot) is the reference order: "max value, then lowest lane,
// then lowest slot" reproduces the reference winner exactly.  A start value of
// -1 with fallback k = 0 reproduces the reference's (best=-1, besti=0) start
// (.cu:115-116).
//
// Per iteration: a packed (v_pk_*) distance update + running max, a DPP row
// reduction + ballot per wave (lowest lane wins ties), the wave winner's slot
// from a bit mask, its coordinates straight out of its registers (uniform slot
// index -> scalar branch tree + v_readlane), one double-buffered LDS slot per
// wave and ONE barrier that waits on LDS only (not on the per-iteration output
// stores), then a 16-lane DPP reduction over the waves.  (The reference
// re-reads dists_i[0] without a barrier: SURVEY.md 5, latent WAR race.)
#include "common.h"

#include <stdlib.h>

// The winner's coordinates by a uniform-index register read (r5): the slot coordinates live in
// one ext_vector per axis (a contiguous VGPR tuple), so VX[sl] with the wave-uniform slot sl
// is s_set_gpr_idx_on + v_mov + s_set_gpr_idx_off, then v_readlane -- instead of a log2(S)-deep
// tree of uniform branches (whose structurised Flow blocks were ~0.2-0.4 us of every
// iteration).  From FPS_MOVREL_MIN slots up (level 2's 16 and level 1's 32; the 4-slot level-2
// geometry measured slower with it, r5).
constexpr int FPS_MOVREL_MIN = 8;

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}

// The running-minimum update d2 = fminf(d, temp) (.cu:130) as one v_min_f32: IEEE minNum returns
// the non-NaN operand, so a NaN distance (a NaN coordinate, or inf - inf) keeps temp, as the
// reference's fminf does.  (fmin_nc's v_med3_f32 returns min3 when an input is NaN: temp became
// -inf, r6 non-finite test.)  Inline asm: fminf itself would add canonicalising v_max around a
// loop-carried value.
__device__ __forceinline__ float fmin_ref(float d, float t) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(d), "v"(t));
    return r;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Row / wave maxima with the DPP folded into the max itself (r5) -- v_max_f32_dpp, one VOP2 per
// step instead of v_mov_b32_dpp + v_med3_f32 (the VOP3 med3 takes no DPP on gfx9) -- and the wave
// max finished by row_bcast:15 / row_bcast:31 into lane 63 (one v_readlane instead of four +
// three maxima).  The values are never NaN (running minima, -inf for invalid slots); max returns
// one of its inputs, so the winners are the same bits.  gfx9 DPP reads a VGPR two wait states
// after its VALU write at the earliest: the s_nop 1s.

__device__ __forceinline__ float row_max16_dpp(float v) {
    float r;
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
        : "=&v"(r)
        : "v"(v));
    return r;
}

// the max of all 64 lanes in lane 63 (lanes 0-62 hold partial maxima)
__device__ __forceinline__ float wave_max_to63_dpp(float v) {
    float r = row_max16_dpp(v);
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(r));
    return r;
}

__device__ __forceinline__ float wave_max_uniform(float v) { return readlane_f(wave_max_to63_dpp(v), 63); }

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// Binary branch tree over a wave-uniform slot index -> three v_readlane (the cluster kernel:
// its coordinates as packed pairs, which keep it at 129 VGPRs; one tuple per axis took 159)
template <int LO, int HI, int N2>
__device__ __forceinline__ void pick_slot_pairs(int sl, int wl, const f2 (&PX)[N2], const f2 (&PY)[N2],
                                                const f2 (&PZ)[N2], float &x, float &y, float &z) {
    if constexpr (HI - LO == 1) {
        x = readlane_f(PX[LO / 2][LO % 2], wl);
        y = readlane_f(PY[LO / 2][LO % 2], wl);
        z = readlane_f(PZ[LO / 2][LO % 2], wl);
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (sl < MID) pick_slot_pairs<LO, MID>(sl, wl, PX, PY, PZ, x, y, z);
        else pick_slot_pairs<MID, HI>(sl, wl, PX, PY, PZ, x, y, z);
    }
}

// The lane's first slot of its maximum (r5), found over coarser maxima from these slot counts up
// (measured, bench lines on one box): pair maxima (16 compares at 32 slots instead of 32; level 1
// 1.567 -> 1.43 us per iteration; level 2's 4-slot geometry 0.545 -> 0.60, so the small geometries
// keep the per-slot search), then quad maxima (2 VALU per 4 slots, a select chain over S / 4
// entries, the winning lane's slot inside its quad by three indexed reads + ballots: level 1 252 ->
// 236 VALU per iteration, 1.251 -> 1.18 us; level 2 0.459 -> 0.468, so level 1 only).  Each lane's
// first maximal slot / pair / quad is a compare/select chain from the top (no bit mask, OR tree
// or find-first-set).
constexpr int FPS_PAIRMASK_MIN = 16, FPS_QUAD_MIN = 32;

// per-axis slot coordinates of a thread: one contiguous VGPR tuple
template <int N>
struct SlotVec {
    typedef float type __attribute__((ext_vector_type(N)));
};

// slot pair s of a coordinate tuple as a packed pair (subregisters: no moves)
template <class V>
__device__ __forceinline__ f2 pair_of(const V &v, int s) {
    return f2{v[2 * s], v[2 * s + 1]};
}

// The winner's coordinates: slot sl (wave-uniform) of lane wl.  FPS_MOVREL_MIN: one indexed
// register read per axis (s_set_gpr_idx_on) + v_readlane; else a binary tree of uniform
// branches down to the slot.
template <int LO, int HI, class V>
__device__ __forceinline__ void pick_slot(int sl, int wl, const V &VX, const V &VY, const V &VZ, float &x,
                                          float &y, float &z) {
    constexpr int N = sizeof(V) / sizeof(float);
    if constexpr (N >= FPS_MOVREL_MIN) {
        x = readlane_f(VX[sl], wl);
        y = readlane_f(VY[sl], wl);
        z = readlane_f(VZ[sl], wl);
    } else if constexpr (HI - LO == 1) {
        x = readlane_f(VX[LO], wl);
        y = readlane_f(VY[LO], wl);
        z = readlane_f(VZ[LO], wl);
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (sl < MID) pick_slot<LO, MID>(sl, wl, VX, VY, VZ, x, y, z);
        else pick_slot<MID, HI>(sl, wl, VX, VY, VZ, x, y, z);
    }
}

// T threads, G reference threads per thread, QT >= ceil(n/bs) points per
// reference thread (slots beyond n are invalid), S = G*QT slots per thread.
template <int T, int G, int QT, bool WEIGHTED, bool STAMP = false>
__global__ __launch_bounds__(T) void fps_reg_kernel(const float *__restrict__ xyz,
                                                    const float *__restrict__ wts,
                                                    float *__restrict__ temp_out,
                                                    int32_t *__restrict__ idx_out,
                                                    float *__restrict__ sampled_out, int n,
                                                    int m, int bs, int L, float inf,
                                                    uint64_t *stamps = nullptr) {
    constexpr int S = G * QT;
    constexpr int S2 = (S + 1) / 2;
    constexpr int NW = T / HREG_WAVE;
    constexpr bool PM = 2 * S2 >= FPS_PAIRMASK_MIN;
    // quad maxima (above): the pair-maxima search one level coarser
    constexpr bool QM = PM && 2 * S2 >= FPS_QUAD_MIN && S2 % 2 == 0;
    static_assert(NW <= 16, "block winner reduction uses one 16-lane row");
    static_assert(2 * S2 <= 32, "slot mask is 32 bits");
    __shared__ float4 s_cand[2][NW];
    __shared__ int s_k[2][NW];
    uint64_t acc0 = 0, acc1 = 0, acc2 = 0, acc3 = 0, r0 = 0, c0 = 0;

    const int cloud = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const float *P = xyz + (size_t)cloud * n * 3;
    const float *W = WEIGHTED ? wts + (size_t)cloud * n : nullptr;

    typename SlotVec<2 * S2>::type VX, VY, VZ;
    // the running minima ("temp"): one tuple when the pair-mask search reads them by a uniform
    // index (PM), else packed pairs (level 2's 4-slot geometry measured 0.545 vs 0.598 us per
    // iteration with the tuple)
    typename SlotVec<2 * S2>::type VT;
    f2 PT[S2];
    auto tget = [&](int s) -> float {
        if constexpr (PM) return VT[s];
        else return PT[s / 2][s % 2];
    };
    f2 PW[S2];
#pragma unroll
    for (int s = 0; s < 2 * S2; ++s) {
        const int g = s / QT, i = s % QT;
        const int rp = tid * G + g;  // position in bit-reversed thread order
        const int k = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
        const bool ok = (s < S) && (rp < bs) && (k < n);
        const int kk = ok ? k : 0;
        VX[s] = P[kk * 3 + 0];
        VY[s] = P[kk * 3 + 1];
        VZ[s] = P[kk * 3 + 2];
        PW[s / 2][s % 2] = WEIGHTED ? W[kk] : 1.0f;
        // the caller's temp is the initial running minimum, as the reference reads it (.cu:130:
        // d2 = min(d, temp[k]); models/utils.py:25 fills 1e10); without one, 1e10.  Invalid
        // slots can never be selected: d2 = -inf never reaches the max
        const float t0 = temp_out ? temp_out[(size_t)cloud * n + kk] : 1e10f;
        if constexpr (PM) VT[s] = ok ? t0 : -__builtin_huge_valf();
        else PT[s / 2][s % 2] = ok ? t0 : -__builtin_huge_valf();
    }
    // opaque: pick_slot must read its coordinates from these tuples, not from the loaded
    // scalars (otherwise every point stays live twice: +96 VGPRs at 32 slots)
    asm volatile("" : "+v"(VX), "+v"(VY), "+v"(VZ));

    float x1 = P[0], y1 = P[1], z1 = P[2];
    const float x0 = x1, y0 = y1, z0 = z1;  // (the reference's fallback point, .cu:115-116)
    if (tid == 0) {
        idx_out[(size_t)cloud * m] = 0;
        if (sampled_out) {
            float *o = sampled_out + (size_t)cloud * m * 3;
            o[0] = x1; o[1] = y1; o[2] = z1;
        }
    }
    if constexpr (STAMP) {
        r0 = __builtin_amdgcn_s_memrealtime();
        c0 = stamp();
    }

    for (int j = 1; j < m; ++j) {
        uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
        if constexpr (STAMP) t0 = stamp();
        const f2 X1 = {x1, x1}, Y1 = {y1, y1}, Z1 = {z1, z1};
        float best = -1.0f;
        float pmx[S2];  // (PM) the pair maxima; (QM) the quad maxima in pmx[0, S2 / 2)
#pragma unroll
        for (int s = 0; s < S2; ++s) {
            const f2 dx = pair_of(VX, s) - X1, dy = pair_of(VY, s) - Y1, dz = pair_of(VZ, s) - Z1;
            f2 d = (dx * dx + dy * dy) + dz * dz;
            if (WEIGHTED) d = PW[s] * d;
            f2 t;
            t.x = fmin_ref(d.x, tget(2 * s));
            t.y = fmin_ref(d.y, tget(2 * s + 1));
            if constexpr (PM) {
                VT[2 * s] = t.x;
                VT[2 * s + 1] = t.y;
            } else {
                PT[s] = t;
            }
            if constexpr (QM) {
                if (s & 1) {
                    const int q = s >> 1;
                    float m3;
                    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m3) : "v"(VT[2 * s - 2]), "v"(VT[2 * s - 1]), "v"(t.x));
                    pmx[q] = fmax_nc(m3, t.y, inf);
                    if (q & 1) asm("v_max3_f32 %0, %1, %2, %3" : "=v"(best) : "v"(best), "v"(pmx[q - 1]), "v"(pmx[q]));
                    else if (s + 1 == S2) best = fmax_nc(best, pmx[q], inf);
                }
            } else if constexpr (PM) {
                pmx[s] = fmax_nc(t.x, t.y, inf);
                if (s & 1) asm("v_max3_f32 %0, %1, %2, %3" : "=v"(best) : "v"(best), "v"(pmx[s - 1]), "v"(pmx[s]));
                else if (s + 1 == S2) best = fmax_nc(best, pmx[s], inf);
            } else {
                // one v_max3_f32 per pair instead of two v_med3 (t and best are never NaN):
                // level-1 FPS 1.634 -> 1.588 us per iteration, bench +0.7 % (A/B on one box, r4)
                asm("v_max3_f32 %0, %1, %2, %3" : "=v"(best) : "v"(best), "v"(t.x), "v"(t.y));
            }
        }
        (void)pmx;
        if constexpr (STAMP) t1 = stamp();
        // the lane's first quad (QM) / pair (PM) / slot holding its own maximum by a select chain
        // from the top: one compare + one select per entry
        int myslot = 0;
        if constexpr (QM) {
#pragma unroll
            for (int q = S2 / 2 - 1; q >= 0; --q) myslot = pmx[q] == best ? q : myslot;
        } else if constexpr (PM) {
#pragma unroll
            for (int s = S2 - 1; s >= 0; --s) myslot = pmx[s] == best ? s : myslot;
        } else {
#pragma unroll
            for (int s = 2 * S2 - 1; s >= 0; --s) myslot = tget(s) == best ? s : myslot;
        }
        const float wmax = wave_max_uniform(best);
        const uint64_t hit = __ballot(best == wmax);
        const int wl = (int)__builtin_ctzll(hit);  // lowest lane = lowest reference order
        int sl;
        if constexpr (QM) {
            // the winning lane's quad, then the first of its slots holding the max: three indexed
            // reads and ballots, each bit of lane wl tested on the scalar unit
            const int sq = __builtin_amdgcn_readlane(myslot, wl);
            const float v0 = VT[4 * sq], v1 = VT[4 * sq + 1], v2 = VT[4 * sq + 2];
            const uint64_t b0 = __ballot(v0 == wmax) >> wl, b1 = __ballot(v1 == wmax) >> wl,
                           b2 = __ballot(v2 == wmax) >> wl;
            sl = 4 * sq + ((b0 & 1) ? 0 : (b1 & 1) ? 1 : (b2 & 1) ? 2 : 3);
        } else if constexpr (PM) {
            // the winning lane's pair, then its x slot if that holds the max (ties: the lower slot)
            const int sp = __builtin_amdgcn_readlane(myslot, wl);
            // (every lane's x slot of pair sp by one indexed read; lane wl's compare bit from a
            // ballot, tested on the scalar unit -- no readlane / v_mov / select round trip)
            const float vtx = VT[2 * sp];
            sl = 2 * sp + (int)((~__ballot(vtx == wmax) >> wl) & 1);
        } else {
            sl = __builtin_amdgcn_readlane(myslot, wl);
        }
        const int rp = (wvu * 64 + wl) * G + sl / QT;  // (uniform: the index on the scalar unit)
        int kwin = (int)bitrev_bits((uint32_t)rp, L) + (sl % QT) * bs;
        asm volatile("" : "+s"(kwin));  // (kept scalar: else it is rebuilt per lane in the write below)
        // with several waves the winner's coordinates only go to LDS, so lane wl writes its own
        // slot sl (one indexed read per axis) instead of three v_readlane and four v_mov for a
        // lane-0 write (r5)
        constexpr bool LW = NW > 1;
        float wx = 0.f, wy = 0.f, wz = 0.f;
        if constexpr (LW) {
            wx = VX[sl];
            wy = VY[sl];
            wz = VZ[sl];
        } else {
            pick_slot<0, 2 * S2>(sl, wl, VX, VY, VZ, wx, wy, wz);
        }
        if constexpr (STAMP) t2 = stamp();
        int old;
        if constexpr (NW == 1) {
            // one wave: its winner is the block winner, no LDS round trip or barrier; no
            // d2 > -1 anywhere: the reference keeps (best=-1, besti=0) (selects, no branch)
            if constexpr (STAMP) t3 = t2;  // (no barrier phase)
            const bool any = wmax > -1.0f;
            old = any ? kwin : 0;
            x1 = any ? wx : x0;
            y1 = any ? wy : y0;
            z1 = any ? wz : z0;
        } else {
            const int buf = j & 1;
            if (lane == (LW ? wl : 0)) {
                s_cand[buf][wv] = make_float4(wx, wy, wz, wmax);
                s_k[buf][wv] = kwin;
            }
            lds_barrier();
            if constexpr (STAMP) t3 = stamp();
            // every lane reads candidate lane % NW (no exec mask, no fill values): the copies sit
            // at higher lanes, so the lowest lane holding the max is still the lowest wave
            const float4 c = s_cand[buf][lane & (NW - 1)];
            const int ck = s_k[buf][lane & (NW - 1)];
            // both loads issue before the reduction (else the compiler sinks x/y/z/k into the
            // branch below: a second LDS round trip on the dependent chain)
            asm volatile("" ::"v"(c.x), "v"(c.y), "v"(c.z), "v"(ck));
            const float gmax = readlane_f(row_max16_dpp(c.w), 0);
            const uint64_t ghit = __ballot(c.w == gmax);
            const int gw = (int)__builtin_ctzll(ghit);  // lowest wave = lowest reference order
            // (a uniform branch here: the selects of the one-wave path measured 0.26 vs 0.22 us
            // for this phase at level 2)
            if (gmax > -1.0f) {
                old = __builtin_amdgcn_readlane(ck, gw);
                x1 = readlane_f(c.x, gw);
                y1 = readlane_f(c.y, gw);
                z1 = readlane_f(c.z, gw);
            } else {  // no d2 > -1 anywhere: the reference keeps (best=-1, besti=0)
                old = 0;
                x1 = x0; y1 = y0; z1 = z0;
            }
        }
        if (tid == 0) {
            idx_out[(size_t)cloud * m + j] = old;
            if (sampled_out) {
                float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
        if constexpr (STAMP) {
            const uint64_t t4 = stamp();
            acc0 += t1 - t0; acc1 += t2 - t1; acc2 += t3 - t2; acc3 += t4 - t3;
        }
    }
    if constexpr (STAMP) {
        const uint64_t c1 = stamp();
        const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
        if (cloud == 0 && tid == 0) {
            stamps[0] = acc0; stamps[1] = acc1; stamps[2] = acc2; stamps[3] = acc3;
            stamps[4] = c1 - c0; stamps[5] = r1 - r0;
        }
    }

    if (temp_out) {
        // recompute the slot indices from an opaque copy of bs/L so the compiler
        // does not keep the prologue's S indices live across the whole loop
        int bs2 = bs, L2 = L;
        asm volatile("" : "+s"(bs2), "+s"(L2));
        float *tp = temp_out + (size_t)cloud * n;
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int g = s / QT, i = s % QT;
            const int rp = tid * G + g;
            const int k = (int)bitrev_bits((uint32_t)rp, L2) + i * bs2;
            if ((rp < bs2) && (k < n)) tp[k] = tget(s);
        }
    }
}

// Fallback for clouds too large for the register-resident path (n > 16384):
// temp lives in the caller's buffer (its contents are the initial running minima, as in the
// reference); same key, same winner.
template <bool WEIGHTED>
__global__ __launch_bounds__(1024) void fps_mem_kernel(const float *__restrict__ xyz,
                                                      const float *__restrict__ wts,
                                                      float *__restrict__ temp,
                                                      int32_t *__restrict__ idx_out,
                                                      float *__restrict__ sampled_out, int n,
                                                      int m, int bs, int L, int Q) {
    constexpr int T = 1024, NW = T / HREG_WAVE;
    __shared__ uint64_t red[2][NW];
    const int cloud = blockIdx.x;
    const int tid = threadIdx.x;
    const float *P = xyz + (size_t)cloud * n * 3;
    const float *W = WEIGHTED ? wts + (size_t)cloud * n : nullptr;
    float *tp = temp + (size_t)cloud * n;
    const int G = bs / T > 0 ? bs / T : 1;
    float x1 = P[0], y1 = P[1], z1 = P[2];
    if (tid == 0) {
        idx_out[(size_t)cloud * m] = 0;
        if (sampled_out) {
            float *o = sampled_out + (size_t)cloud * m * 3;
            o[0] = x1; o[1] = y1; o[2] = z1;
        }
    }
    for (int j = 1; j < m; ++j) {
        float best = -1.0f;
        uint32_t brank = 0;
        bool have = false;
        for (int g = 0; g < G; ++g) {
            const int rp = tid * G + g;
            if (rp >= bs) break;
            const int r = (int)bitrev_bits((uint32_t)rp, L);
            for (int i = 0; i < Q; ++i) {
                const int k = r + i * bs;
                if (k >= n) break;
                float d = sqdist3(P[k * 3], P[k * 3 + 1], P[k * 3 + 2], x1, y1, z1);
                if (WEIGHTED) d = fmul_rn(W[k], d);
                const float d2 = fminf(d, tp[k]);
                tp[k] = d2;
                if (d2 > best) { best = d2; brank = (uint32_t)(rp * Q + i); have = true; }
            }
        }
        if (!have) brank = 0;
        uint64_t key = ((uint64_t)float_orderable(best) << 32) | (uint64_t)(0xffffffffu - brank);
        key = wave_max_u64(key);
        const int buf = j & 1;
        if ((tid & (HREG_WAVE - 1)) == 0) red[buf][tid / HREG_WAVE] = key;
        __syncthreads();
        uint64_t k2 = red[buf][0];
        for (int w = 1; w < NW; ++w) { const uint64_t o = red[buf][w]; k2 = o > k2 ? o : k2; }
        const uint32_t wr = 0xffffffffu - (uint32_t)(k2 & 0xffffffffu);
        const int old = (int)bitrev_bits(wr / (uint32_t)Q, L) + (int)(wr % (uint32_t)Q) * bs;
        x1 = P[old * 3 + 0];
        y1 = P[old * 3 + 1];
        z1 = P[old * 3 + 2];
        if (tid == 0) {
            idx_out[(size_t)cloud * m + j] = old;
            if (sampled_out) {
                float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Large clouds (16384 < n <= 64 * 64 * 32): one cloud spread over NP <= 64
// single-wave workgroups ("participants"), every point still register-resident.
// Participant p's lane l owns the S consecutive reference ranks
// (p * 64 + l) * S + s, rank = rp * Q + i for point k = bitrev_L(rp) + i * bs
// (the fps_mem_kernel order), so "max d2, then lowest participant, lane, slot"
// is the reference winner.  Per iteration each participant publishes its
// candidate as four 64-bit words {d2 | rank | tag, x | j, y | j, z | j} with
// agent-scope relaxed atomic stores into a per-cloud, per-parity slot, then one
// lane per participant polls those slots (agent-scope atomic loads) until every
// word carries this iteration's tag: the data is its own flag, so there is no
// counter, fence or L2 write-back on the critical path.  A participant cannot
// reach iteration j + 2 (same parity slot) before every participant has
// published j + 1, i.e. finished reading j.  The slots live in the caller's
// temp buffer, zeroed by the launcher (tags 0 never match j >= 1).  Every
// poll loop is bounded; on expiry the wave sets HREG_STATUS_FPS_TIMEOUT in the
// library's device status word (read and cleared by hreg_device_status, which the
// host checks at its sync points) and leaves the kernel.  Only participant 0 writes
// idx / sampled, and the launcher zero-fills both first, so after a timeout every idx
// entry of the launch is a valid index (0 or a real selection) and every sampled row
// finite; their contents are otherwise undefined and the host raises.  Every other
// participant then times out within one poll budget too, so the grid drains.
// (measured alternatives, r2: four lanes publishing in one store instruction 2.45 vs
// 1.71 ms for 4 x 65536 points; a 128-byte slot stride and s_sleep between polls no
// faster)
struct SyncSlot {
    uint64_t w[4];
};
constexpr int FPS_CL_MAXP = 64;
constexpr uint32_t FPS_CL_POLLS = 1u << 22;

}  // namespace

// sticky error bits of asynchronous kernels (HREG_STATUS_*), hreg_device_status()
__device__ int g_hreg_status = 0;

namespace {

__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int S, bool WEIGHTED>
__global__ __launch_bounds__(64) void fps_cluster_kernel(const float *__restrict__ xyz,
                                                         const float *__restrict__ wts,
                                                         SyncSlot *__restrict__ slots,
                                                         int32_t *__restrict__ idx_out,
                                                         float *__restrict__ sampled_out, int b,
                                                         int n, int m, int bs, int L, int Q, int NP,
                                                         float inf, uint32_t polls_max, int stall) {
    constexpr int S2 = S / 2;
    static_assert(S % 2 == 0 && S <= 32, "slots");
    const int p = blockIdx.x;  // participant
    const int lane = threadIdx.x;
    for (int cloud = blockIdx.y; cloud < b; cloud += gridDim.y) {
        const float *P = xyz + (size_t)cloud * n * 3;
        const float *W = WEIGHTED ? wts + (size_t)cloud * n : nullptr;
        SyncSlot *sl = slots + (size_t)cloud * 2 * FPS_CL_MAXP;
        f2 PX[S2], PY[S2], PZ[S2], PT[S2], PW[S2];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int rank = (p * 64 + lane) * S + s;
            const int rp = rank / Q, i = rank - rp * Q;
            const int k = (int)bitrev_bits((uint32_t)rp, L) + i * bs;
            const bool ok = rp < bs && k < n;
            const int kk = ok ? k : 0;
            PX[s / 2][s % 2] = P[kk * 3 + 0];
            PY[s / 2][s % 2] = P[kk * 3 + 1];
            PZ[s / 2][s % 2] = P[kk * 3 + 2];
            PW[s / 2][s % 2] = WEIGHTED ? W[kk] : 1.0f;
            PT[s / 2][s % 2] = ok ? 1e10f : -__builtin_huge_valf();
        }
#pragma unroll
        for (int s = 0; s < S2; ++s) asm volatile("" : "+v"(PX[s]), "+v"(PY[s]), "+v"(PZ[s]));  // (fps_reg_kernel)
        float x1 = P[0], y1 = P[1], z1 = P[2];
        if (p == 0 && lane == 0) {
            idx_out[(size_t)cloud * m] = 0;
            if (sampled_out) {
                float *o = sampled_out + (size_t)cloud * m * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
        bool timed_out = false;
        for (int j = 1; j < m && !timed_out; ++j) {
            const f2 X1 = {x1, x1}, Y1 = {y1, y1}, Z1 = {z1, z1};
            float best = -1.0f;
#pragma unroll
            for (int s = 0; s < S2; ++s) {
                const f2 dx = PX[s] - X1, dy = PY[s] - Y1, dz = PZ[s] - Z1;
                f2 d = (dx * dx + dy * dy) + dz * dz;
                if (WEIGHTED) d = PW[s] * d;
                f2 t;
                t.x = fmin_ref(d.x, PT[s].x);
                t.y = fmin_ref(d.y, PT[s].y);
                PT[s] = t;
                best = fmax_nc(best, fmax_nc(t.x, t.y, inf), inf);
            }
            const float wmax = wave_max_uniform(best);
            uint32_t smask = 0;
#pragma unroll
            for (int s = 0; s < S; ++s) smask |= (PT[s / 2][s % 2] == wmax) ? (1u << s) : 0u;
            const int myslot = smask ? (int)__builtin_ctz(smask) : 0;
            const uint64_t hit = __ballot(best == wmax);
            const int wl = (int)__builtin_ctzll(hit);
            const int ws = __builtin_amdgcn_readlane(myslot, wl);
            float wx = 0.f, wy = 0.f, wz = 0.f;
            pick_slot_pairs<0, S>(ws, wl, PX, PY, PZ, wx, wy, wz);
            const uint32_t rank = (uint32_t)((p * 64 + wl) * S + ws);
            SyncSlot *cur = sl + (j & 1) * FPS_CL_MAXP;
            const uint64_t tag = (uint64_t)(uint32_t)j << 32;
            // lane 0 publishes; the coordinates first, the key word last (lanes 0..3
            // storing one word each in a single instruction let the polls start before the
            // stores are acknowledged and measured slower)
            if (lane == 0 && p != stall) {  // stall: hreg_debug_fps_cluster's forced-stall test
                st_agent(&cur[p].w[1], tag | __float_as_uint(wx));
                st_agent(&cur[p].w[2], tag | __float_as_uint(wy));
                st_agent(&cur[p].w[3], tag | __float_as_uint(wz));
                st_agent(&cur[p].w[0], ((uint64_t)__float_as_uint(wmax) << 32) |
                                           ((uint64_t)rank << 10) | (uint64_t)(j & 1023));
            }
            // wait for the store acknowledgement before polling: the r1 code got this wait
            // by accident of scheduling, and without it (the timeout rework of r2 let the
            // compiler drop it) a call took 3.0-3.9 instead of 1.7 ms for 4 x 65536 points
            // (Model_V2 bench 774 -> 617 pairs/s, tools/v2_bisect.sh)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // poll: lane q reads participant q's words until all carry tag j
            uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
            bool fresh = lane >= NP;
            uint32_t polls = 0;
            while (true) {
                if (!fresh) {
                    w0 = ld_agent(&cur[lane].w[0]);
                    w1 = ld_agent(&cur[lane].w[1]);
                    w2 = ld_agent(&cur[lane].w[2]);
                    w3 = ld_agent(&cur[lane].w[3]);
                    fresh = (w0 & 1023u) == (uint64_t)(j & 1023) && (w1 >> 32) == (uint64_t)j &&
                            (w2 >> 32) == (uint64_t)j && (w3 >> 32) == (uint64_t)j;
                }
                if (__all(fresh)) break;
                if (++polls > polls_max) {
                    timed_out = true;
                    break;
                }
            }
            if (timed_out) {
                // the launch's selections are lost: flag it and leave (idx / sampled hold
                // the launcher's zero fill where participant 0 has not written)
                if (lane == 0) atomicOr(&g_hreg_status, HREG_STATUS_FPS_TIMEOUT);
                return;
            }
            const float cd = lane < NP ? __uint_as_float((uint32_t)(w0 >> 32)) : -__builtin_huge_valf();
            const float gmax = wave_max_uniform(cd);
            const int gl = (int)__builtin_ctzll(__ballot(lane < NP && cd == gmax));
            int old;
            if (gmax > -1.0f) {
                const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w0, gl) >> 10;
                const uint32_t rp = r / (uint32_t)Q, i = r - rp * (uint32_t)Q;
                old = (int)bitrev_bits(rp, L) + (int)i * bs;
                x1 = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w1, gl));
                y1 = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w2, gl));
                z1 = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w3, gl));
            } else {  // the reference keeps (best=-1, besti=0)
                old = 0;
                x1 = P[0]; y1 = P[1]; z1 = P[2];
            }
            if (p == 0 && lane == 0) {
                idx_out[(size_t)cloud * m + j] = old;
                if (sampled_out) {
                    float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                    o[0] = x1; o[1] = y1; o[2] = z1;
                }
            }
        }
    }
}

template <bool WEIGHTED, bool STAMP = false>
bool launch_reg(int T, int G, int QT, int b, int n, int m, int bs, int L, const float *xyz,
                const float *w, float *temp, int32_t *idx, float *sampled, uint64_t *stamps,
                hipStream_t st) {
#define FPS_CASE(TT, GG, QQ)                                                              \
    if (T == TT && G == GG && QT == QQ) {                                                      \
        hipLaunchKernelGGL((fps_reg_kernel<TT, GG, QQ, WEIGHTED, STAMP>), dim3(b), dim3(TT), 0, \
                           st, xyz, w, temp, idx, sampled, n, m, bs, L, __builtin_huge_valf(), \
                           stamps);                                                            \
        return true;                                                                           \
    }
    FPS_CASE(1024, 1, 1) FPS_CASE(1024, 1, 2) FPS_CASE(1024, 1, 4)
    FPS_CASE(1024, 1, 8)
    // (512, 2, 16) unweighted only: the weighted form needs 32 more VGPRs and spills
    if constexpr (!WEIGHTED) { FPS_CASE(1024, 1, 16) FPS_CASE(512, 2, 16) }
    FPS_CASE(512, 1, 1) FPS_CASE(512, 1, 2)
    FPS_CASE(256, 4, 1) FPS_CASE(256, 1, 1) FPS_CASE(256, 1, 2)
    FPS_CASE(128, 4, 1) FPS_CASE(128, 1, 1) FPS_CASE(128, 1, 2)
    FPS_CASE(64, 16, 1) FPS_CASE(64, 8, 1) FPS_CASE(128, 8, 1)
    FPS_CASE(64, 4, 1) FPS_CASE(64, 1, 1) FPS_CASE(64, 1, 2)
#undef FPS_CASE
    return false;
}

// choose (T threads, G reference threads per thread, QT slots per reference thread)
void choose_geometry(int n, bool weighted, int &T, int &G, int &QT) {
    const int bs = hreg_opt_n_threads(n);
    const int Q = (n + bs - 1) / bs;
    QT = 1;
    while (QT < Q) QT <<= 1;
    if (Q == 1 && bs >= 256) {
        // one wave (no barrier) while its scan stays short; 4 waves at bs = 1024
        // (measured, 16 clouds: n=512 0.130 ms at 1 wave vs 0.150 at 2; n=1024 (r1) 0.300 ms
        // at 4 waves vs 0.331 at 1.  r5: with the pair-maxima slot search and the indexed
        // winner read, one wave x 16 weighted points per lane runs level 2 at 0.484 vs 0.564 us
        // per iteration, single-batch latency 3.26 vs 3.32 ms; two waves with the leaner
        // exchange measured 0.58 (level 2) / 0.47 (level 3) vs 0.46 / 0.38 -- one wave throughout)
        T = 64;
        G = bs / T;
        QT = 1;
        return;
    }
    if (bs >= 64) { T = bs; G = 1; }
    else { T = 64; G = 1; }
    // per-slot registers (x, y, z, temp[, w]) must fit the VGPR budget
    if (T == 1024 && QT > (weighted ? 8 : 16)) { T = 512; G = 2; }
    // n = 16384 (level 1): 8 waves x 32 slots rather than 16 waves x 16 -- the same VALU
    // work per SIMD, half the per-wave reduction/winner overhead; both fill a CU's VGPRs
    // (127 x 1024 vs 254 x 512).  768 clouds (the batched level-1 stage) 5.70 -> 5.19 ms,
    // identical indices (tools/micro/fps_l1_geom.py).
    // (1024 threads x 16 points measured 1.58 vs 1.43 us per iteration, r5)
    if (!weighted && T == 1024 && QT == 16) {
        T = 512; G = 2;
    }
}

// Co-residency of the cluster kernel's spinning participants.  A
// cluster makes progress once all its NP single-wave workgroups are resident; waves of
// other (finite) kernels always drain, so it can only stall if spinning waves alone fill
// every wave slot the kernel's registers allow.  This process runs at most
// GPU_MAX_HW_QUEUES kernels at once (HIP's hardware queues, default 4; kernels sharing a
// queue run in order), so a launch spins at most (resident waves of this kernel on the
// whole device) / queues waves -- every concurrent cluster launch together fits on the
// chip at once -- and never more than 256.  The budget is queried once per variant
// (occupancy API x CU count); if it cannot hold one cluster, the launch uses the
// non-spinning fps_mem_kernel.  The poll bound + HREG_STATUS_FPS_TIMEOUT stay the
// backstop (other processes on the same device are outside this bound).
//
// `concurrent` (hreg_fps_bounded): the caller guarantees at most that many cluster launches of
// this process run at once -- a graph whose ONE stage-1 stream runs every multi-workgroup FPS
// (Model_V2's batched stage 1) passes 1 -- so a launch may spin up to 3/4 of (resident waves) /
// concurrent (the quarter kept back is margin for the occupancy API's over-reports,
// MI355X_MICROARCH.md Residency: every other kernel's waves are finite and drain, so the
// spinning participants of one launch all become resident once they fit on the chip alone).
// 0: the hardware-queue bound above.
// The fewest slots per lane of a cluster participant (r5): 32 slots = 32 single-wave
// participants for a 65536-point cloud (253 VGPRs) instead of 64 x 16 slots (129 VGPRs).
// With the bounded budget of the batched Model_V2 stage 1 every lane's clouds then run at once
// (64 clouds of 32 waves): Model_V2 line 1410 -> 3279 pairs/s (merge 8, 2 lanes, one box;
// 16 slots with a 2048-wave cap: 1685).  (r6: Model_V2's clouds now run fps_blocks_kernel; the
// cluster kernel stays the boundary's path for hreg_furthest_point_sampling above 16384 points.)
constexpr int FPS_SPIN_CAP = 256, FPS_SPIN_CAP_BOUNDED = 4096, FPS_CL_S = 32;
int cluster_wave_budget(bool weighted, int concurrent = 0) {
    static int cache[2] = {-1, -1};  // resident waves of the variant
    int &c = cache[weighted ? 1 : 0];
    if (c < 0) {
        int dev = 0, cus = 0, per_cu = 0;
        const void *fn = weighted ? reinterpret_cast<const void *>(&fps_cluster_kernel<FPS_CL_S, true>)
                                  : reinterpret_cast<const void *>(&fps_cluster_kernel<FPS_CL_S, false>);
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, 0) != hipSuccess) {
            (void)hipGetLastError();
            c = 0;
        } else {
            c = per_cu * cus;
        }
    }
    if (c <= 0) return 0;
    if (concurrent > 0) {
        const long b = (long)c * 3 / 4 / concurrent;
        return (int)(b < FPS_SPIN_CAP_BOUNDED ? b : FPS_SPIN_CAP_BOUNDED);
    }
    const char *q = getenv("GPU_MAX_HW_QUEUES");
    int queues = q ? atoi(q) : 4;
    if (queues < 1) queues = 4;
    const long budget = (long)c / queues;
    return (int)(budget < FPS_SPIN_CAP ? budget : FPS_SPIN_CAP);
}

template <bool WEIGHTED>
int launch_fps(int b, int n, int m, const float *xyz, const float *w, float *temp, int32_t *idx,
               float *sampled, hipStream_t st, uint32_t polls_max = FPS_CL_POLLS, int stall = -1,
               bool force_cluster = false, int concurrent = 0) {
    if (b < 0 || n <= 0 || xyz == nullptr || idx == nullptr) return HREG_ERR_INVALID;
    if (WEIGHTED && w == nullptr) return HREG_ERR_INVALID;
    if (b == 0 || m <= 0) return HREG_OK;  // .cu:92: if (m <= 0) return;
    const int bs = hreg_opt_n_threads(n);
    const int L = hreg_ilog2(bs);
    const int Q = (n + bs - 1) / bs;
    int T, G, QT;
    choose_geometry(n, WEIGHTED, T, G, QT);
    if (!force_cluster &&
        launch_reg<WEIGHTED>(T, G, QT, b, n, m, bs, L, xyz, w, temp, idx, sampled, nullptr, st)) {
        HREG_CHECK_LAUNCH();
        return HREG_OK;
    }
    // large clouds: the caller's temp buffer is required (sync slots / running minima)
    if (temp == nullptr) return HREG_ERR_INVALID;
    const long ranks = (long)bs * Q;
    const int S = ranks <= (long)FPS_CL_MAXP * 64 * FPS_CL_S ? FPS_CL_S : 0;
    const size_t slot_bytes = (size_t)2 * FPS_CL_MAXP * sizeof(SyncSlot);
    const int NP = S ? (int)((ranks + 64L * S - 1) / (64L * S)) : 0;
    const int spin = S ? cluster_wave_budget(WEIGHTED, concurrent) : 0;
    if (S && (size_t)n * sizeof(float) >= slot_bytes && spin >= NP) {
        const int clusters = b < spin / NP ? b : spin / NP;
        SyncSlot *slots = reinterpret_cast<SyncSlot *>(temp);
        if (hipMemsetAsync(slots, 0, (size_t)b * slot_bytes, st) != hipSuccess) return HREG_ERR_LAUNCH;
        // valid outputs even if the exchange times out (participant 0 writes; see above)
        if (hipMemsetAsync(idx, 0, (size_t)b * m * sizeof(int32_t), st) != hipSuccess ||
            (sampled && hipMemsetAsync(sampled, 0, (size_t)b * m * 3 * sizeof(float), st) != hipSuccess))
            return HREG_ERR_LAUNCH;
        const dim3 grid(NP, clusters);
        hipLaunchKernelGGL((fps_cluster_kernel<FPS_CL_S, WEIGHTED>), grid, dim3(64), 0, st, xyz, w, slots, idx,
                           sampled, b, n, m, bs, L, Q, NP, __builtin_huge_valf(), polls_max, stall);
        HREG_CHECK_LAUNCH();
        return HREG_OK;
    }
    if (force_cluster) return HREG_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((fps_mem_kernel<WEIGHTED>), dim3(b), dim3(1024), 0, st, xyz, w, temp, idx,
                       sampled, n, m, bs, L, Q);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// ------------------------------------------------------------------------------------------------
// Level-1 FPS over the spatial index's Morton-sorted copy, with exact group pruning (r5).
//
// The same selections as fps_reg_kernel<512, 2, 16> (n = 16384): 8 waves x 32 slots per lane, but
// the slots hold hreg_spatial_index's Morton-sorted float4 (x, y, z, id) copy: group g (slots
// 4g..4g+3) of wave w is the 256-point Morton range 8g + w (slot 4g + q of lane l: sorted point
// (8g + w) * 256 + 64q + l), one bounding box per group.  Consecutive ranges sit in different
// waves: a new centre's few affected ranges are neighbours, so they spread over the waves instead
// of queueing in one (measured: ranges in wave order, w * 2048 + 64 s + l, ran 1.18 us per
// iteration, no faster than fps_reg_kernel).  Per iteration, group g is scanned only if the box lower bound of its squared
// distance to the new centre is below the group's largest running minimum: otherwise every point
// has d >= lb >= max T >= T and min(d, T) = T for all of them (lb and d are computed with the same
// rounded operations on coordinates the box orders, and rounding is monotone, so lb <= d holds
// in fp32 too).  A scanned group is updated with the reference arithmetic (two-rounding squared
// distance, min).  ~5 of 64 groups need a scan per iteration on KITTI-shape clouds (simulated).
//
// The reference's winner (max T, then the lowest reference thread in tree order, then its lowest
// k) no longer follows the register order, so every point carries its reference
// rank  rank(k) = bitrev_L(k mod bs) * Q + k div bs  (with its slot in the low 5 bits): a lane's
// candidate per group is (max T, min rank among its slots at that T), the wave's is (max T, min
// rank), and the workgroup's the same over the 8 waves.
constexpr int FS_T = 512, FS_NW = 8, FS_S = 32, FS_NG = 8, FS_N = FS_T * FS_S;
// (measured no faster, r5 gpurun_out/r5ag, and removed: the lane's candidate rank at the wave max
// as 8 independent selects + a v_min3_u32 tree, and the group scans laid out as unlikely)
__device__ __forceinline__ uint32_t row_min16_u32_dpp(uint32_t v) {
    uint32_t r;
    asm("s_nop 1\n\t"
        "v_min_u32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
        : "=&v"(r)
        : "v"(v));
    return r;
}

// the minimum of all 64 lanes in lane 63
__device__ __forceinline__ uint32_t wave_min_to63_u32_dpp(uint32_t v) {
    uint32_t r = row_min16_u32_dpp(v);
    asm("s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(r));
    return r;
}

__device__ __forceinline__ float wave_min_uniform_dpp(float v) {
    return -readlane_f(wave_max_to63_dpp(-v), 63);
}

__global__ __launch_bounds__(FS_T) void fps_sorted_kernel(const float4 *__restrict__ spts, int np,
                                                          const float *__restrict__ xyz,
                                                          float *__restrict__ temp_out,
                                                          int32_t *__restrict__ idx_out,
                                                          float *__restrict__ sampled_out, int m, int bs,
                                                          int L, int LQ, float inf) {
    typedef typename SlotVec<FS_S>::type V;
    __shared__ float4 s_cand[2][FS_NW];
    __shared__ uint32_t s_r[2][FS_NW];
    __shared__ int s_k[2][FS_NW];
    const int cloud = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    const float4 *SP = spts + (size_t)cloud * np + (size_t)wvu * 256;
    // slot s -> offset from SP: range 8 (s / 4) + w, row s % 4 of its 4 x 64
    auto soff = [&](int s) { return (s >> 2) * (FS_NW * 256) + (s & 3) * 64 + lane; };
    const float *P = xyz + (size_t)cloud * FS_N * 3;

    V VX, VY, VZ, VT;
    uint32_t VE[FS_S];  // rank << 5 | slot
#pragma unroll
    for (int s = 0; s < FS_S; ++s) {
        const float4 v = SP[soff(s)];
        VX[s] = v.x;
        VY[s] = v.y;
        VZ[s] = v.z;
        VT[s] = 1e10f;
        const uint32_t id = (uint32_t)__float_as_int(v.w);
        const uint32_t rank = (bitrev_bits(id & (uint32_t)(bs - 1), L) << LQ) + (id >> L);
        VE[s] = (rank << 5) | (uint32_t)s;
    }
    asm volatile("" : "+v"(VX), "+v"(VY), "+v"(VZ));

    // group boxes (wave-uniform) into lanes 0..7; per-lane group candidates
    float glx = 0.f, gly = 0.f, glz = 0.f, ghx = 0.f, ghy = 0.f, ghz = 0.f;
    float gm = -__builtin_huge_valf();  // lane g < 8: group g's largest running minimum
    float tg[FS_NG];
    uint32_t rg[FS_NG];
#pragma unroll
    for (int g = 0; g < FS_NG; ++g) {
        float lx = VX[4 * g], ly = VY[4 * g], lz = VZ[4 * g], hx = lx, hy = ly, hz = lz;
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            lx = fminf(lx, VX[4 * g + q]); hx = fmaxf(hx, VX[4 * g + q]);
            ly = fminf(ly, VY[4 * g + q]); hy = fmaxf(hy, VY[4 * g + q]);
            lz = fminf(lz, VZ[4 * g + q]); hz = fmaxf(hz, VZ[4 * g + q]);
        }
        lx = wave_min_uniform_dpp(lx); ly = wave_min_uniform_dpp(ly); lz = wave_min_uniform_dpp(lz);
        hx = readlane_f(wave_max_to63_dpp(hx), 63);
        hy = readlane_f(wave_max_to63_dpp(hy), 63);
        hz = readlane_f(wave_max_to63_dpp(hz), 63);
        if (lane == g) {
            glx = lx; gly = ly; glz = lz; ghx = hx; ghy = hy; ghz = hz;
            gm = 1e10f;
        }
        tg[g] = 1e10f;
        uint32_t r = VE[4 * g];
#pragma unroll
        for (int q = 1; q < 4; ++q) r = min(r, VE[4 * g + q]);
        rg[g] = r;
    }

    float x1 = P[0], y1 = P[1], z1 = P[2];
    if (tid == 0) {
        idx_out[(size_t)cloud * m] = 0;
        if (sampled_out) {
            float *o = sampled_out + (size_t)cloud * m * 3;
            o[0] = x1; o[1] = y1; o[2] = z1;
        }
    }

    for (int j = 1; j < m; ++j) {
        // which groups can change: box lower bound below the group's largest T (lanes 0..7)
        const float qx = fminf(fmaxf(x1, glx), ghx), qy = fminf(fmaxf(y1, gly), ghy), qz = fminf(fmaxf(z1, glz), ghz);
        const float lb = sqdist3(x1, y1, z1, qx, qy, qz);
        const uint32_t amask = (uint32_t)__ballot(lb < gm);
        const f2 X1 = {x1, x1}, Y1 = {y1, y1}, Z1 = {z1, z1};
#pragma unroll
        for (int g = 0; g < FS_NG; ++g) {
            if ((amask >> g) & 1u) {
#pragma unroll
                for (int s = 2 * g; s < 2 * g + 2; ++s) {
                    const f2 dx = pair_of(VX, s) - X1, dy = pair_of(VY, s) - Y1, dz = pair_of(VZ, s) - Z1;
                    const f2 d = (dx * dx + dy * dy) + dz * dz;
                    VT[2 * s] = fmin_ref(d.x, VT[2 * s]);
                    VT[2 * s + 1] = fmin_ref(d.y, VT[2 * s + 1]);
                }
                float m4;
                asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m4) : "v"(VT[4 * g]), "v"(VT[4 * g + 1]), "v"(VT[4 * g + 2]));
                m4 = fmax_nc(m4, VT[4 * g + 3], inf);
                uint32_t r = 0xffffffffu;
#pragma unroll
                for (int q = 0; q < 4; ++q) r = VT[4 * g + q] == m4 ? min(r, VE[4 * g + q]) : r;
                tg[g] = m4;
                rg[g] = r;
                const float gmx = readlane_f(wave_max_to63_dpp(m4), 63);
                gm = lane == g ? gmx : gm;
            }
        }
        // the wave's candidate: max T, then min rank (branch-free: skipping the min reductions when
        // one lane holds the max measured 1.04 vs 0.96 us per iteration)
        const float W = readlane_f(row_max16_dpp(gm), 0);
        uint32_t rl = 0xffffffffu;
#pragma unroll
        for (int g = 0; g < FS_NG; ++g) rl = tg[g] == W ? min(rl, rg[g]) : rl;
        const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)wave_min_to63_u32_dpp(rl), 63);
        const int wl = (int)__builtin_ctzll(__ballot(rl == R));
        const int sl = (int)(R & 31u);
        const uint32_t rank = R >> 5;
        int kwin = (int)bitrev_bits(rank >> LQ, L) + (int)(rank & ((1u << LQ) - 1u)) * bs;
        asm volatile("" : "+s"(kwin));
        const float wx = VX[sl], wy = VY[sl], wz = VZ[sl];
        const int buf = j & 1;
        if (lane == wl) {
            s_cand[buf][wv] = make_float4(wx, wy, wz, W);
            s_r[buf][wv] = R;
            s_k[buf][wv] = kwin;
        }
        lds_barrier();
        const float4 c = s_cand[buf][lane & (FS_NW - 1)];
        const uint32_t cr = s_r[buf][lane & (FS_NW - 1)];
        const int ck = s_k[buf][lane & (FS_NW - 1)];
        asm volatile("" ::"v"(c.x), "v"(c.y), "v"(c.z), "v"(cr), "v"(ck));
        const float gmax = readlane_f(row_max16_dpp(c.w), 0);
        const uint32_t rr = c.w == gmax ? cr : 0xffffffffu;
        const uint32_t rmin = (uint32_t)__builtin_amdgcn_readlane((int)row_min16_u32_dpp(rr), 0);
        const int gw = (int)__builtin_ctzll(__ballot(rr == rmin));
        const int old = __builtin_amdgcn_readlane(ck, gw);
        x1 = readlane_f(c.x, gw);
        y1 = readlane_f(c.y, gw);
        z1 = readlane_f(c.z, gw);
        if (tid == 0) {
            idx_out[(size_t)cloud * m + j] = old;
            if (sampled_out) {
                float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
    }
    if (temp_out) {
        float *tp = temp_out + (size_t)cloud * FS_N;
#pragma unroll
        for (int s = 0; s < FS_S; ++s) tp[__float_as_int(SP[soff(s)].w)] = VT[s];
    }
}

// ------------------------------------------------------------------------------------------------
// Level-1 FPS of large clouds (16384 < n <= 65536, n % 64 == 0: Model_V2's 65536-point clouds,
// configs[4]) on ONE workgroup, with exact pruning per 64-point block of the spatial index (r6).
//
// A 65536-point cloud's coordinates do not fit one CU's registers, which is why the cluster kernel
// above spreads it over 32 single-wave workgroups exchanging candidates through memory every
// iteration (~2 us per iteration in the Model_V2 step, with 32 spinning waves per cloud).  With
// pruning, an iteration only reads the few blocks its new centre can change (~28 of 1024 blocks
// on KITTI-shape clouds with the 15-bit index, knn.hip spatial_index_kernel<true>), so here the
// running minima T stay in registers (64 slots per lane) and the coordinates of the blocks to
// scan are read from the index's sorted float4 copy (L2-resident, 1 MB per cloud) each time:
//   * 16 waves; wave w's slot r of lane l is sorted point (16 r + w) * 64 + l, i.e. wave w owns
//     the index blocks 16 r + w (consecutive blocks in different waves: a centre's affected
//     blocks are spatial neighbours, so they spread over the waves), and lane r of wave w holds
//     block 16 r + w's box (the index's) and its candidate: the block's largest T and the
//     smallest reference rank R among its points at that T;
//   * per iteration a block is scanned only if its box lower bound to the new centre is below
//     the block's largest T (fps_sorted_kernel's exactness argument, per block), up to 4 blocks'
//     loads in flight per wave;
//   * the winner is max T, then min R over the blocks, waves (LDS, one barrier) -- R = the
//     reference rank (bitrev_L(k mod bs) * Q + k div bs, SURVEY.md 8a's tie rule) << 16 | the
//     sorted position -- and its coordinates and index come from the sorted copy.
// No spinning participants: one CU per cloud, ~100 VGPRs per lane, so the other lanes' level
// kernels share its CU.
// Measured (tools/fps_blocks_time.py, 8 / 64 KITTI-shape clouds, r6): up to 4 blocks' loads in
// flight per wave 1.53 / 1.87 us per iteration (2: 1.63 / 1.84; 8: 2.43 / 2.78, register
// pressure); skipping the block's min-rank reduction when one lane holds its maximum 1.73 ->
// 1.53; carrying the candidates' coordinates through the exchange instead of reading the
// winner's from the index after it 1.66 (no gain: three readlanes per scanned block).
// 64 clouds run slower than 8: their sorted copies (64 MB) exceed the L2s, so blocks come from
// the MALL.  The cluster kernel on the same clouds: 1.97 / 5.6 us per iteration.
// NW waves (a power of two <= 16): 16 for Model_V2's 65536-point clouds; r6, 4 for 16384-point
// clouds in the throughput executor's batched level-1 stage (fps_lean: 256 blocks, every lane one;
// 4 waves x 108 VGPRs leave the CU's other SIMD slots to the lanes' level kernels, where
// fps_sorted_kernel's 8 waves x 229 VGPRs hold the whole register file)
constexpr int FB_A = 4;

__device__ __forceinline__ uint32_t fb_rank(uint32_t id, int L, int Q) {
    return bitrev_bits(id & ((1u << L) - 1u), L) * (uint32_t)Q + (id >> L);
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void fps_blocks_kernel(const float4 *__restrict__ spts,
                                                          const float4 *__restrict__ boxes, int np,
                                                          const float *__restrict__ xyz,
                                                          float *__restrict__ temp_out,
                                                          int32_t *__restrict__ idx_out,
                                                          float *__restrict__ sampled_out, int n, int m,
                                                          int L, int Q, float inf) {
    typedef typename SlotVec<32>::type V;
    __shared__ float s_w[2][NW];  // the waves' candidates: max T, min R
    __shared__ uint32_t s_r[2][NW];
    const int cloud = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int w = __builtin_amdgcn_readfirstlane(wv);
    const int rows = n >> 6;
    const float4 *SP = spts + (size_t)cloud * np;
    const float4 *BX = boxes + (size_t)cloud * (np / 64) * 2;

    // this lane's block (NW lane + w): box and candidate; -inf: no block
    const int myrow = NW * lane + w;
    float lx = 0.f, ly = 0.f, lz = 0.f, hx = 0.f, hy = 0.f, hz = 0.f;
    float rmT = -__builtin_huge_valf();
    uint32_t rR = 0xffffffffu;
    if (myrow < rows) {
        const float4 a = BX[2 * myrow], b = BX[2 * myrow + 1];
        lx = a.x; ly = a.y; lz = a.z; hx = b.x; hy = b.y; hz = b.z;
        rmT = 1e10f;
    }
    // running minima: slot r in T0 (r < 32) / T1; the block's smallest rank into its lane
    V T0, T1;
#pragma unroll
    for (int r = 0; r < 64; ++r) {
        if (r < 32) T0[r] = 1e10f;
        else T1[r - 32] = 1e10f;
        if (NW * r + w < rows) {  // (uniform)
            const int pos = (NW * r + w) * 64 + lane;
            const uint32_t R = (fb_rank((uint32_t)__float_as_int(SP[pos].w), L, Q) << 16) | (uint32_t)pos;
            const uint32_t Rm = (uint32_t)__builtin_amdgcn_readlane((int)wave_min_to63_u32_dpp(R), 63);
            if (lane == r) rR = Rm;
        }
    }

    const float *P = xyz + (size_t)cloud * n * 3;
    float x1 = P[0], y1 = P[1], z1 = P[2];
    if (tid == 0) {
        idx_out[(size_t)cloud * m] = 0;
        if (sampled_out) {
            float *o = sampled_out + (size_t)cloud * m * 3;
            o[0] = x1; o[1] = y1; o[2] = z1;
        }
    }

    for (int j = 1; j < m; ++j) {
        // which of this wave's blocks can change: box lower bound below the block's largest T
        const float qx = fminf(fmaxf(x1, lx), hx), qy = fminf(fmaxf(y1, ly), hy), qz = fminf(fmaxf(z1, lz), hz);
        const float lb = sqdist3(x1, y1, z1, qx, qy, qz);
        const uint64_t act = __ballot(lb < rmT);
        // slots 0..31 (T0), then 32..63 (T1): a separate loop per register tuple, so every
        // access is one indexed register read / write (s_set_gpr_idx) with the slot in an SGPR
        auto scan = [&](V &T, uint32_t act32, int r0) {
            while (act32) {
                int ra[FB_A];
                float4 v[FB_A];
                int cnt = 0;
#pragma unroll
                for (int a = 0; a < FB_A; ++a) {
                    ra[a] = 0;
                    if (act32) {  // (uniform) the next block's points, loads in flight together
                        const int r = (int)__builtin_ctz(act32);
                        act32 &= act32 - 1;
                        ra[a] = r;
                        cnt = a + 1;
                        v[a] = SP[(NW * (r0 + r) + w) * 64 + lane];
                    }
                }
#pragma unroll
                for (int a = 0; a < FB_A; ++a) {
                    if (a < cnt) {
                        const int r = ra[a];
                        // the reference arithmetic (.cu:129-130): two-rounding squared distance, min
                        const float d = sqdist3(v[a].x, v[a].y, v[a].z, x1, y1, z1);
                        const float t = fmin_ref(d, T[r]);
                        T[r] = t;
                        const uint32_t pos = (uint32_t)((NW * (r0 + r) + w) * 64 + lane);
                        const uint32_t R = (fb_rank((uint32_t)__float_as_int(v[a].w), L, Q) << 16) | pos;
                        // the block's candidate: max T, then min R -- one lane at the max (the
                        // usual case) needs no second reduction
                        const float mx = readlane_f(wave_max_to63_dpp(t), 63);
                        const uint64_t at = __ballot(t == mx);
                        const uint32_t Rm =
                            __builtin_popcountll(at) == 1  // (uniform)
                                ? (uint32_t)__builtin_amdgcn_readlane((int)R, (int)__builtin_ctzll(at))
                                : (uint32_t)__builtin_amdgcn_readlane(
                                      (int)wave_min_to63_u32_dpp(t == mx ? R : 0xffffffffu), 63);
                        if (lane == r0 + r) {
                            rmT = mx;
                            rR = Rm;
                        }
                    }
                }
            }
        };
        scan(T0, (uint32_t)act, 0);
        scan(T1, (uint32_t)(act >> 32), 32);
        // the wave's candidate, then the workgroup's: max T, then min R
        const float W = readlane_f(wave_max_to63_dpp(rmT), 63);
        const uint32_t Rw =
            (uint32_t)__builtin_amdgcn_readlane((int)wave_min_to63_u32_dpp(rmT == W ? rR : 0xffffffffu), 63);
        const int buf = j & 1;
        if (lane == 0) {
            s_w[buf][wv] = W;
            s_r[buf][wv] = Rw;
        }
        lds_barrier();
        const float cw = s_w[buf][lane & (NW - 1)];
        const uint32_t cr = s_r[buf][lane & (NW - 1)];
        const float gmax = readlane_f(row_max16_dpp(cw), 0);
        const uint32_t Rg =
            (uint32_t)__builtin_amdgcn_readlane((int)row_min16_u32_dpp(cw == gmax ? cr : 0xffffffffu), 0);
        const float4 q = SP[Rg & 0xffffu];  // (uniform address: the winner from the sorted copy)
        x1 = q.x;
        y1 = q.y;
        z1 = q.z;
        if (tid == 0) {
            idx_out[(size_t)cloud * m + j] = __float_as_int(q.w);
            if (sampled_out) {
                float *o = sampled_out + ((size_t)cloud * m + j) * 3;
                o[0] = x1; o[1] = y1; o[2] = z1;
            }
        }
    }
    if (temp_out) {
        float *tp = temp_out + (size_t)cloud * n;
#pragma unroll
        for (int r = 0; r < 64; ++r)
            if (NW * r + w < rows) tp[__float_as_int(SP[(NW * r + w) * 64 + lane].w)] = r < 32 ? T0[r] : T1[r - 32];
    }
}

}  // namespace

// Diagnostic: per-phase cycle sums of block 0 / wave 0 of the register path
// (stamps[6] = scan, wave reduce + pick, LDS write + barrier, final reduce,
// total cycles, total 100 MHz ticks).  Not part of the product path.
extern "C" int hreg_debug_fps_stamps(int b, int n, int m, const float *points, const float *weights,
                                     int32_t *idx, uint64_t *stamps, void *stream) {
    if (b <= 0 || n <= 0 || m <= 0 || !points || !idx || !stamps) return HREG_ERR_INVALID;
    const int bs = hreg_opt_n_threads(n);
    int T, G, QT;
    choose_geometry(n, weights != nullptr, T, G, QT);
    const bool ok =
        weights ? launch_reg<true, true>(T, G, QT, b, n, m, bs, hreg_ilog2(bs), points, weights,
                                         nullptr, idx, nullptr, stamps, as_stream(stream))
                : launch_reg<false, true>(T, G, QT, b, n, m, bs, hreg_ilog2(bs), points, nullptr,
                                          nullptr, idx, nullptr, stamps, as_stream(stream));
    if (!ok) return HREG_ERR_UNSUPPORTED;
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// Diagnostic: the latency floor of the level-1 FPS geometry -- the same 512-thread,
// 8-wave workgroup, per-iteration exchange and barrier as the n = 16384 kernel
// (fps_reg_kernel<512, 2, 16>), but 2 points per thread (n = 1024), so an iteration is the
// dependent chain (wave max, winner pick, LDS hand-off + barrier, block max) with almost no
// scan.  stamps as hreg_debug_fps_stamps.  points [b][1024][3].
// stamps == nullptr: the same kernel without stamps (its launch time per iteration is the floor
// of an unstamped kernel).
extern "C" int hreg_debug_fps_floor(int b, int m, const float *points, int32_t *idx, uint64_t *stamps,
                                    void *stream) {
    if (b <= 0 || m <= 0 || !points || !idx) return HREG_ERR_INVALID;
    if (stamps)
        hipLaunchKernelGGL((fps_reg_kernel<512, 2, 1, false, true>), dim3(b), dim3(512), 0, as_stream(stream),
                           points, nullptr, nullptr, idx, nullptr, 1024, m, 1024, 10, __builtin_huge_valf(), stamps);
    else
        hipLaunchKernelGGL((fps_reg_kernel<512, 2, 1, false, false>), dim3(b), dim3(512), 0, as_stream(stream),
                           points, nullptr, nullptr, idx, nullptr, 1024, m, 1024, 10, __builtin_huge_valf(), nullptr);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// Diagnostic: the latency floor of a WFPS level's geometry -- T threads
// with one point each (n = T, bs = T, G = QT = 1: the same waves, per-iteration wave reduction,
// LDS hand-off + barrier (T > 64) and block reduction as the level's kernel, almost no scan and
// a one-slot pick), weighted.  T = 256: level 2's 4-wave workgroup (n = 1024 runs
// fps_reg_kernel<256, 4, 1, true>); T = 64: level 3's single wave (n = 512:
// fps_reg_kernel<64, 8, 1, true>).  points [b][T][3], weights [b][T]; stamps as
// hreg_debug_fps_stamps.
extern "C" int hreg_debug_wfps_floor(int b, int T, int m, const float *points, const float *weights,
                                     int32_t *idx, uint64_t *stamps, void *stream) {
    if (b <= 0 || m <= 0 || !points || !weights || !idx || !stamps) return HREG_ERR_INVALID;
    hipStream_t st = as_stream(stream);
    if (T == 256)
        hipLaunchKernelGGL((fps_reg_kernel<256, 1, 1, true, true>), dim3(b), dim3(256), 0, st, points, weights,
                           nullptr, idx, nullptr, 256, m, 256, 8, __builtin_huge_valf(), stamps);
    else if (T == 64)
        hipLaunchKernelGGL((fps_reg_kernel<64, 1, 1, true, true>), dim3(b), dim3(64), 0, st, points, weights,
                           nullptr, idx, nullptr, 64, m, 64, 6, __builtin_huge_valf(), stamps);
    else
        return HREG_ERR_UNSUPPORTED;
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_furthest_point_sampling(int b, int n, int m, const float *points,
                                            float *temp, int32_t *idx, float *sampled_xyz,
                                            void *stream) {
    return launch_fps<false>(b, n, m, points, nullptr, temp, idx, sampled_xyz, as_stream(stream));
}

// hreg_furthest_point_sampling whose caller guarantees that at most `concurrent` (>= 1)
// multi-workgroup FPS launches of this process run at once (one stream carries them all): the
// launch may then keep (resident waves) / concurrent participants spinning instead of
// (resident waves) / GPU_MAX_HW_QUEUES (cluster_wave_budget).  Same results.
extern "C" int hreg_fps_bounded(int b, int n, int m, const float *points, float *temp, int32_t *idx,
                                float *sampled_xyz, int concurrent, void *stream) {
    if (concurrent < 1) return HREG_ERR_INVALID;
    return launch_fps<false>(b, n, m, points, nullptr, temp, idx, sampled_xyz, as_stream(stream), FPS_CL_POLLS,
                             -1, false, concurrent);
}

// FPS of n = 16384-point clouds over the spatial index in ws (hreg_spatial_index of the same
// points, built before this call): fps_sorted_kernel, the selections of
// hreg_furthest_point_sampling bit for bit with most of each iteration's scan pruned.  Other
// sizes: hreg_furthest_point_sampling's kernels (ws unused).
extern "C" int hreg_fps_indexed(int b, int n, int m, const float *points, const void *ws, float *temp,
                                int32_t *idx, float *sampled_xyz, void *stream) {
    if (b < 0 || n <= 0 || !points || !idx || !ws) return HREG_ERR_INVALID;
    if (b == 0 || m <= 0) return HREG_OK;
    const int bs = hreg_opt_n_threads(n);
    if (n > FS_N && n <= 65536 && n % 64 == 0 && !(reinterpret_cast<uintptr_t>(ws) & 15)) {
        // large clouds: one workgroup, T in registers, blocks read from the index (above)
        size_t np = 64;
        while (np < (size_t)n) np <<= 1;
        const float4 *spts = static_cast<const float4 *>(ws);
        const int L = hreg_ilog2(bs), Q = (n + bs - 1) / bs;
        hipLaunchKernelGGL(fps_blocks_kernel<16>, dim3(b), dim3(16 * 64), 0, as_stream(stream), spts,
                           spts + (size_t)b * np, (int)np, points, temp, idx, sampled_xyz, n, m, L, Q,
                           __builtin_huge_valf());
        HREG_CHECK_LAUNCH();
        return HREG_OK;
    }
    if (n != FS_N || bs * (n / bs) != n || (n / bs) > 32 || (reinterpret_cast<uintptr_t>(ws) & 15))
        return launch_fps<false>(b, n, m, points, nullptr, temp, idx, sampled_xyz, as_stream(stream));
    const int L = hreg_ilog2(bs), LQ = hreg_ilog2(n / bs);
    hipLaunchKernelGGL(fps_sorted_kernel, dim3(b), dim3(FS_T), 0, as_stream(stream),
                       static_cast<const float4 *>(ws), FS_N, points, temp, idx, sampled_xyz, m, bs, L, LQ,
                       __builtin_huge_valf());
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

// hreg_fps_indexed for the throughput executor's batched level-1 stage (r6): 16384-point clouds on
// fps_blocks_kernel<4> (T in registers, block coordinates from the index's sorted copy: a small
// register footprint per cloud at a longer iteration) instead of fps_sorted_kernel; the same
// selections.  Other sizes: hreg_fps_indexed.
extern "C" int hreg_fps_indexed_lean(int b, int n, int m, const float *points, const void *ws, float *temp,
                                     int32_t *idx, float *sampled_xyz, void *stream) {
    if (b < 0 || n <= 0 || !points || !idx || !ws) return HREG_ERR_INVALID;
    if (b == 0 || m <= 0) return HREG_OK;
    if (n != FS_N || (reinterpret_cast<uintptr_t>(ws) & 15))
        return hreg_fps_indexed(b, n, m, points, ws, temp, idx, sampled_xyz, stream);
    const int bs = hreg_opt_n_threads(n);
    const float4 *spts = static_cast<const float4 *>(ws);
    const int L = hreg_ilog2(bs), Q = (n + bs - 1) / bs;
    hipLaunchKernelGGL(fps_blocks_kernel<4>, dim3(b), dim3(4 * 64), 0, as_stream(stream), spts,
                       spts + (size_t)b * n, n, points, temp, idx, sampled_xyz, n, m, L, Q, __builtin_huge_valf());
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_weighted_furthest_point_sampling(int b, int n, int m, const float *points,
                                                     const float *weights, float *temp,
                                                     int32_t *idx, float *sampled_xyz,
                                                     void *stream) {
    return launch_fps<true>(b, n, m, points, weights, temp, idx, sampled_xyz, as_stream(stream));
}

namespace {
__device__ int g_hreg_status_taken = 0;
// read-and-clear in one atomic step, so a bit raised by a kernel still running on
// another stream is either returned now or kept for the next call, never lost
__global__ void status_take_kernel() { g_hreg_status_taken = atomicExch(&g_hreg_status, 0); }
}  // namespace

// Synchronous: waits for every stream of the device first (the flagging kernels may run
// on any non-blocking stream), then reads (and with clear, atomically takes)
// the status word.
extern "C" int hreg_device_status(int *status, int clear) {
    if (!status) return HREG_ERR_INVALID;
    if (hipDeviceSynchronize() != hipSuccess) return HREG_ERR_LAUNCH;
    if (clear) {
        hipLaunchKernelGGL(status_take_kernel, dim3(1), dim3(1), 0, 0);
        if (hipGetLastError() != hipSuccess) return HREG_ERR_LAUNCH;
        if (hipMemcpyFromSymbol(status, HIP_SYMBOL(g_hreg_status_taken), sizeof(int)) != hipSuccess)
            return HREG_ERR_LAUNCH;
        return HREG_OK;
    }
    if (hipMemcpyFromSymbol(status, HIP_SYMBOL(g_hreg_status), sizeof(int)) != hipSuccess)
        return HREG_ERR_LAUNCH;
    return HREG_OK;
}

extern "C" int hreg_debug_fps_cluster(int b, int n, int m, const float *points, float *temp,
                                      int32_t *idx, float *sampled_xyz, int stall,
                                      unsigned polls_max, void *stream) {
    if (polls_max == 0) return HREG_ERR_INVALID;
    return launch_fps<false>(b, n, m, points, nullptr, temp, idx, sampled_xyz, as_stream(stream),
                             polls_max, stall, true);
}
