// group_l1.hip -- fused level-1 keypoint detector + descriptor for gfx950.
//
// One wave owns one keypoint group: its k = 64 neighbour rows (two 32-row
// MFMA column tiles).  Every layer of
//   KeypointDetector.convs 4->32->32->64   (layers.py:115-121, 150)
//   attention: max_c -> softmax_k -> keypoint / attentive feature (layers.py:151-159)
//   DescExtractor.convs   4->32->32->64    (layers.py:183-189, 201)
//   k-max, cat[x2, x1, att_map] -> mlp1 192->32 -> mlp2 32->64 -> k-max (layers.py:202-208)
// runs on v_mfma_f32_32x32x2_f32 with the activations kept in the MFMA
// accumulators: an output tile D[c_out][row] (lane = row, register q = channel
// (q&3) + 8(q>>2) + 4(lane>>5)) is directly the B operand of the next layer's
// k-step q, so activations never leave the registers.  The weight A-fragments
// were permuted to that channel order on the host and sit in LDS (shared by
// the workgroup's waves); BN(eval) is the per-channel epilogue
// y = relu(acc * alpha + beta).  Only the group outputs (keypoint 3, attentive
// feature 64, descriptor 64 floats) are written to HBM -- the reference
// materialises ~1 GB of [B,C,M,k] tensors per batch here.
#include "../common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVES = 4;
constexpr int KN = 64;  // neighbours per group (level 1)

// fragment table layout (floats), built by engine.L1Tables
constexpr int F_DC1 = 0;                       // det conv1: 1 co x 2 ksteps
constexpr int F_DC2 = F_DC1 + 2 * 64;          // det conv2: 1 co x 16
constexpr int F_DC3 = F_DC2 + 16 * 64;         // det conv3: 2 co x 16
constexpr int F_EC1 = F_DC3 + 32 * 64;         // desc conv1
constexpr int F_EC2 = F_EC1 + 2 * 64;
constexpr int F_EC3 = F_EC2 + 16 * 64;
constexpr int F_M1 = F_EC3 + 32 * 64;          // mlp1: 1 co x 6 ct x 16
constexpr int F_M2 = F_M1 + 96 * 64;           // mlp2: 2 co x 16
constexpr int F_END = F_M2 + 32 * 64;
// epilogue (alpha, beta) per layer, channel-indexed
constexpr int E_DC1 = F_END, E_DC2 = E_DC1 + 64, E_DC3 = E_DC2 + 64, E_EC1 = E_DC3 + 128,
              E_EC2 = E_EC1 + 64, E_EC3 = E_EC2 + 64, E_M1 = E_EC3 + 128, E_M2 = E_M1 + 64,
              TABLE_FLOATS = E_M2 + 128;

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int q = 0; q < 16; ++q) z[q] = 0.f;
    return z;
}

__device__ __forceinline__ int chan(int co, int q, int h) { return co * 32 + (q & 3) + 8 * (q >> 2) + 4 * h; }

// acc[co][jt] += W-fragments x in[ct][jt]  (in: accumulator-layout activations).
// Fragments are stored with 4 consecutive k-steps innermost per lane
// ([co][ct][q/4][lane][4], engine.l1_table): one ds_read_b128 per 4 MFMA k-steps.
template <int CIN_T, int COUT_T, int JT, int JT_IN>
__device__ __forceinline__ void mfma_accum(const float *__restrict__ wf, int lane,
                                           const f32x16 (&in)[CIN_T][JT_IN],
                                           f32x16 (&acc)[COUT_T][JT], const float *scale = nullptr) {
#pragma unroll
    for (int ct = 0; ct < CIN_T; ++ct)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            float4 a[COUT_T];
#pragma unroll
            for (int co = 0; co < COUT_T; ++co)
                a[co] = *reinterpret_cast<const float4 *>(wf + (((co * CIN_T + ct) * 4 + q4) * 64 + lane) * 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = q4 * 4 + i;
#pragma unroll
                for (int co = 0; co < COUT_T; ++co) {
#pragma unroll
                    for (int jt = 0; jt < JT; ++jt) {
                        float b = in[ct][JT_IN == 1 ? 0 : jt][q];
                        if (scale) b = fmul_rn(b, scale[jt]);
                        acc[co][jt] = __builtin_amdgcn_mfma_f32_32x32x2f32((&a[co].x)[i], b, acc[co][jt], 0, 0, 0);
                    }
                }
            }
            // bound the scheduler's look-ahead (LDS fragment loads, scaled B values) to
            // 4 k-steps so the live set stays in the register file
            __builtin_amdgcn_sched_barrier(0);
        }
}

template <int COUT_T, int JT>
__device__ __forceinline__ void epilogue(const float *__restrict__ ab, int lane,
                                         f32x16 (&acc)[COUT_T][JT]) {
    const int h = lane >> 5;
    constexpr int C = COUT_T * 32;
#pragma unroll
    for (int co = 0; co < COUT_T; ++co)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = chan(co, q, h);
            const float al = ab[c], be = ab[C + c];
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
                acc[co][jt][q] = fmaxf(fadd_rn(fmul_rn(acc[co][jt][q], al), be), 0.f);
        }
}

// first conv (Cin = 4 geometric channels): k-step s, lane half h -> channel 2h + s
template <int JT>
__device__ __forceinline__ void conv_geom(const float *__restrict__ wf, const float *__restrict__ ab,
                                          int lane, const float2 (&g)[JT], f32x16 (&acc)[1][JT]) {
#pragma unroll
    for (int jt = 0; jt < JT; ++jt) acc[0][jt] = zero16();
    const float2 a = *reinterpret_cast<const float2 *>(wf + lane * 2);  // [lane][2 k-steps]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int jt = 0; jt < JT; ++jt)
            acc[0][jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(s == 0 ? a.x : a.y, s == 0 ? g[jt].x : g[jt].y,
                                                               acc[0][jt], 0, 0, 0);
    }
    epilogue<1, JT>(ab, lane, acc);
}

// 3-layer conv stack 4 -> 32 -> 32 -> 64
__device__ __forceinline__ void conv_stack(const float *tb, int f1, int f2, int f3, int e1, int e2,
                                           int e3, int lane, const float2 (&g)[2],
                                           f32x16 (&out)[2][2]) {
    f32x16 h1[1][2], h2[1][2];
    conv_geom<2>(tb + f1, tb + e1, lane, g, h1);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) h2[0][jt] = zero16();
    mfma_accum<1, 1, 2, 2>(tb + f2, lane, h1, h2);
    epilogue<1, 2>(tb + e2, lane, h2);
#pragma unroll
    for (int co = 0; co < 2; ++co)
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) out[co][jt] = zero16();
    mfma_accum<1, 2, 2, 2>(tb + f3, lane, h2, out);
    epilogue<2, 2>(tb + e3, lane, out);
}

// one channel tile of a per-group result reduced over the rows (valid in lanes 31 /
// 63): channels co*32 + 8r + 4h + {0..3} for registers q = 4r..4r+3 -> 4 float4 stores
__device__ __forceinline__ void store_tile(float *out, int co, const f32x16 &v, int j, int h) {
    if (j == 31) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            *reinterpret_cast<float4 *>(out + co * 32 + 8 * r + 4 * h) =
                make_float4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
    }
}

__global__ __launch_bounds__(256, 2) void group_l1_kernel(
    const float *__restrict__ table, const float *__restrict__ geom, const float *__restrict__ knn_xyz,
    int G, float *__restrict__ kp, float *__restrict__ att_feat, float *__restrict__ desc) {
    __shared__ float tb[TABLE_FLOATS];
    for (int i = threadIdx.x; i < TABLE_FLOATS; i += blockDim.x) tb[i] = table[i];
    __syncthreads();

    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, j = lane & 31;
    for (int g = blockIdx.x * WAVES + w; g < G; g += gridDim.x * WAVES) {
        const size_t r0 = (size_t)g * KN;
        float2 gin[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
            gin[jt] = *reinterpret_cast<const float2 *>(geom + (r0 + jt * 32 + j) * 4 + 2 * h);

        // ---- detector convs -> emb [64 ch][64 rows]
        f32x16 emb[2][2];
        conv_stack(tb, F_DC1, F_DC2, F_DC3, E_DC1, E_DC2, E_DC3, lane, gin, emb);

        // ---- attention: x1 = max_c emb, a = softmax over the 64 rows (emb >= 0 after
        // ReLU: maxima on the integer bit patterns; DPP half-wave reductions)
        float x1[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            int mi = __float_as_int(emb[0][jt][0]);
#pragma unroll
            for (int co = 0; co < 2; ++co)
#pragma unroll
                for (int q = 0; q < 16; ++q) mi = max(mi, __float_as_int(emb[co][jt][q]));
            x1[jt] = __int_as_float(max(mi, __shfl_xor(mi, 32)));
        }
        const float mx = half_bcast(half_max_hi_nonneg(fmaxf(x1[0], x1[1])), h);
        const float e0 = expf(fsub_rn(x1[0], mx)), e1 = expf(fsub_rn(x1[1], mx));
        const float ssum = half_bcast(half_sum_hi(fadd_rn(e0, e1)), h);
        const float a[2] = {e0 / ssum, e1 / ssum};

        // keypoint = sum_rows a * knn_xyz
        float kx = 0.f, ky = 0.f, kz = 0.f;
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
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
        // attentive feature [64 ch] = sum_rows emb * a
#pragma unroll
        for (int co = 0; co < 2; ++co) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                v[q] = half_sum_hi(fadd_rn(fmul_rn(emb[co][0][q], a[0]), fmul_rn(emb[co][1][q], a[1])));
            store_tile(att_feat + (size_t)g * 64, co, v, j, h);
        }

        // ---- descriptor convs -> x1d [64][64]
        f32x16 x1d[2][2];
        conv_stack(tb, F_EC1, F_EC2, F_EC3, E_EC1, E_EC2, E_EC3, lane, gin, x1d);
        // x2 = max over rows (broadcast to every row = the repeat of layers.py:204)
        f32x16 x2[2][1];
#pragma unroll
        for (int co = 0; co < 2; ++co)
#pragma unroll
            for (int q = 0; q < 16; ++q)
                x2[co][0][q] = half_bcast(half_max_hi_nonneg(fmaxf(x1d[co][0][q], x1d[co][1][q])), h);

        // ---- mlp1: cat[x2 (64), x1d (64), emb * a (64)] -> 32
        f32x16 y1[1][2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) y1[0][jt] = zero16();
        mfma_accum<2, 1, 2, 1>(tb + F_M1, lane, x2, y1);
        mfma_accum<2, 1, 2, 2>(tb + F_M1 + 32 * 64, lane, x1d, y1);
        mfma_accum<2, 1, 2, 2>(tb + F_M1 + 64 * 64, lane, emb, y1, a);
        epilogue<1, 2>(tb + E_M1, lane, y1);
        // ---- mlp2: 32 -> 64, then max over rows
        f32x16 y2[2][2];
#pragma unroll
        for (int co = 0; co < 2; ++co)
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) y2[co][jt] = zero16();
        mfma_accum<1, 2, 2, 2>(tb + F_M2, lane, y1, y2);
        epilogue<2, 2>(tb + E_M2, lane, y2);
#pragma unroll
        for (int co = 0; co < 2; ++co) {
            f32x16 v;
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = half_max_hi_nonneg(fmaxf(y2[co][0][q], y2[co][1][q]));
            store_tile(desc + (size_t)g * 64, co, v, j, h);
        }
    }
}

}  // namespace

extern "C" int hreg_group_l1_table_floats(void) { return TABLE_FLOATS; }

extern "C" int hreg_group_l1(const float *table, const float *geom, const float *knn_xyz, int G,
                             float *kp, float *att_feat, float *desc, void *stream) {
    if (!table || !geom || !knn_xyz || !kp || !att_feat || !desc || G < 0) return HREG_ERR_INVALID;
    if (!G) return HREG_OK;
    int grid = (G + WAVES - 1) / WAVES;
    if (grid > 2048) grid = 2048;
    hipLaunchKernelGGL(group_l1_kernel, dim3(grid), dim3(256), 0, as_stream(stream), table, geom,
                       knn_xyz, G, kp, att_feat, desc);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}
