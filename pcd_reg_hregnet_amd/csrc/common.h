// common.h -- shared helpers for the HRegNet gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hregnet_amd.h"

#define HREG_WAVE 64

// Launch-check helper: every C-ABI entry returns a status code, never exits
// (the reference prints and calls exit(-1): furthest_point_sampling_gpu.cu:35-38).
#define HREG_CHECK_LAUNCH()                                       \
    do {                                                          \
        hipError_t _e = hipGetLastError();                        \
        if (_e != hipSuccess) return HREG_ERR_LAUNCH;             \
    } while (0)

static inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// cuda_utils.h:22-26: block size the reference picks for n points.
static inline int hreg_opt_n_threads(int work_size) {
    if (work_size < 1) return 1;
    const int pow_2 = (int)(__builtin_log((double)work_size) / __builtin_log(2.0));
    int v = 1 << pow_2;
    if (v > 1024) v = 1024;
    if (v < 1) v = 1;
    return v;
}

static inline int hreg_ilog2(int v) {
    int l = 0;
    while ((1 << (l + 1)) <= v) ++l;
    return l;
}

// ---------------------------------------------------------------- device --

// XCD-aware block order (MI355X_MICROARCH.md, workgroup dispatch; cdna_hip_programming.md
// T1): blocks are dealt round-robin over the 8 XCDs, each with its own L2, so block b and
// b + 8 share one.  The bijective remap below hands every XCD a CONTIGUOUS range of logical
// blocks; kernels whose neighbouring blocks read the same data (the queries of one cloud,
// which all read that cloud's points) then fetch it into one L2 instead of eight.  Speed only:
// the result never depends on the placement.  (Level-1 indexed kNN: 65.4 -> 7.8 MB read per
// launch, r4.)
__device__ __forceinline__ int xcd_block(int b, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// Non-contracted float arithmetic: the whole library builds with
// -ffp-contract=off; these make the intent explicit where order matters.
__device__ __forceinline__ float fmul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub_rn(float a, float b) { return __fsub_rn(a, b); }

// Train-mode BatchNorm apply (+ ReLU) of one value: act(gamma * ((y - mean) * invstd) + beta),
// the one arithmetic of hreg_bn_apply and of the GEMMs that apply it on load (train.hip,
// ts_gemm.hip)
__device__ __forceinline__ float bn_act(float y, float mu, float is, float ga, float be, int relu) {
    const float xh = fmul_rn(fsub_rn(y, mu), is);
    const float v = fadd_rn(fmul_rn(xh, ga), be);
    return relu ? fmaxf(v, 0.f) : v;
}

// Squared distance in the reference's order: (dx*dx + dy*dy) + dz*dz, two
// roundings per term (furthest_point_sampling_gpu.cu:129; pytorch3d knn loop).
__device__ __forceinline__ float sqdist3(float ax, float ay, float az, float bx, float by,
                                         float bz) {
    const float dx = fsub_rn(ax, bx), dy = fsub_rn(ay, by), dz = fsub_rn(az, bz);
    return fadd_rn(fadd_rn(fmul_rn(dx, dx), fmul_rn(dy, dy)), fmul_rn(dz, dz));
}

// min/max through v_med3_f32: one instruction, without the canonicalising
// v_max the compiler puts around fminf/fmaxf on loop-carried values.
// med3(a, b, -inf) = min(a, b), med3(a, b, +inf) = max(a, b) for non-NaN a, b.
// `inf` must be a runtime +infinity (e.g. a kernel argument): with a literal
// the compiler folds med3 back into minnum/maxnum.
__device__ __forceinline__ float fmin_nc(float a, float b, float inf) {
    return __builtin_amdgcn_fmed3f(a, b, -inf);
}
__device__ __forceinline__ float fmax_nc(float a, float b, float inf) {
    return __builtin_amdgcn_fmed3f(a, b, inf);
}

// IEEE float -> uint32 with the same total order (negative values included).
__device__ __forceinline__ uint32_t float_orderable(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float orderable_float(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ uint32_t bitrev_bits(uint32_t x, int L) {
    return L == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - L));
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt) but NOT for its outstanding global stores, unlike __syncthreads()
// whose release fence adds s_waitcnt vmcnt(0) -- in a loop that stores results
// every iteration that puts store-completion latency on the critical path.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wave-level LDS hand-off between lanes (rocPRIM's wave_barrier pattern):
// release fence + wave barrier + acquire fence, so the compiler cannot move
// one lane's LDS store past another lane's later LDS load.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((unsigned)(v & 0xffffffffu), m);
    const uint32_t hi = __shfl_xor((unsigned)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = shfl_xor_u64(v, m);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ float wave_max_f32(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
    return v;
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fadd_rn(v, __shfl_xor(v, m));
    return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}

// ------------------------------------------- half-wave (32-lane) reductions --
// Sum / max over the 32 lanes of each wave half on the VALU (DPP), instead of
// __shfl_xor's ds_bpermute round trips through the LDS crossbar: quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror and row_mirror reduce each 16-lane row,
// row_bcast:15 (rows 1 and 3 only) adds row 0 / row 2.  The result is valid in
// lanes 16..31 (half 0) and 48..63 (half 1); half_bcast() spreads it.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_mov(float v, float old) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL,
                                                      ROW_MASK, 0xf, false));
}
// full-mask DPP move within a 16-lane row (quad_perm / row_mirror / row_half_mirror: every
// lane has a valid source, so bound_ctrl and the old value never matter).  Written as
// update_dpp(old = 0, bound_ctrl = 1) the compiler folds it into the consuming
// v_add_f32_dpp / v_max_i32_dpp (one instruction per reduction step instead of a
// v_mov_b32_dpp + the op: the row reductions were ~30 % of the fused kernels' VALU)
template <int CTRL>
__device__ __forceinline__ float dpp_all(float v) {
    static_assert(CTRL <= 0xff || CTRL == 0x140 || CTRL == 0x141, "in-row controls only");
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ int dpp_all_i(int v) {
    static_assert(CTRL <= 0xff || CTRL == 0x140 || CTRL == 0x141, "in-row controls only");
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ float half_sum_hi(float v) {
    v = fadd_rn(v, dpp_all<0xb1>(v));
    v = fadd_rn(v, dpp_all<0x4e>(v));
    v = fadd_rn(v, dpp_all<0x141>(v));
    v = fadd_rn(v, dpp_all<0x140>(v));
    return fadd_rn(v, dpp_mov<0x142, 0xa>(v, 0.f));
}
// max of non-negative floats (ReLU outputs): their IEEE bit patterns order like
// signed integers, so the reduction runs on v_max_i32 (no NaN canonicalisation)
__device__ __forceinline__ float half_max_hi_nonneg(float f) {
    int v = __float_as_int(f);
    v = max(v, dpp_all_i<0xb1>(v));
    v = max(v, dpp_all_i<0x4e>(v));
    v = max(v, dpp_all_i<0x141>(v));
    v = max(v, dpp_all_i<0x140>(v));
    v = max(v, __builtin_amdgcn_update_dpp((int)0x80000000, v, 0x142, 0xa, 0xf, false));
    return __int_as_float(v);
}
// the half's reduced value (from lane 31 / 63) in every lane of that half
__device__ __forceinline__ float half_bcast(float v, int h) {
    const float lo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 31));
    const float hi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
    return h ? hi : lo;
}

// Sum / max over each 16-lane DPP row, result in every lane of the row.
__device__ __forceinline__ float row_sum16(float v) {
    v = fadd_rn(v, dpp_all<0xb1>(v));
    v = fadd_rn(v, dpp_all<0x4e>(v));
    v = fadd_rn(v, dpp_all<0x141>(v));
    return fadd_rn(v, dpp_all<0x140>(v));
}
__device__ __forceinline__ float row_max16_nonneg(float f) {
    int v = __float_as_int(f);
    v = max(v, dpp_all_i<0xb1>(v));
    v = max(v, dpp_all_i<0x4e>(v));
    v = max(v, dpp_all_i<0x141>(v));
    return __int_as_float(max(v, dpp_all_i<0x140>(v)));
}
