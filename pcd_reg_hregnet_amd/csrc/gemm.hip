// gemm.hip -- fp32 MFMA "NT" GEMM with fused BN/ReLU or cosine epilogue.
//
// Every 1x1 Conv1d/Conv2d + BatchNorm(eval) + ReLU of the HRegNet forward is
// out[r][n] = act(scale[n] * sum_k A[r][k] W[n][k] + shift[n]) over point rows
// r (layers.py:115-130, 183-198, 246-268, 417-431).  fp32 is required: a
// bf16-scale perturbation flips most level-2 kNN indices, and
// gfx950 has no xf32, so the contraction runs on v_mfma_f32_32x32x2_f32.
//
// The A operand is assembled on the fly from up to four K-segments (a plain
// row, a row gathered through a kNN index, a per-group row r/k, or a row scaled
// by an attention weight), so the reference's cat/repeat/knn_gather tensors
// (layers.py:23-27, 204-206, 364-380, 444-445) are never materialised.
//
// Layout: activations are point-major ([rows][channels]) in HBM.  A block
// computes a BM x BN tile; K is staged through LDS in BK = 16/32 chunks, double
// buffered with one barrier per chunk.  Inside each 16-deep sub-chunk lane half
// h takes k = h*8 + s for MFMA k-step s, so each lane's k-values are contiguous and
// come out of LDS with ds_read_b128 (rows padded by 4 floats: the 16 rows of a
// ds_read_b128 lane group hit 16 distinct 16-byte slots).
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float4 load_a4(const hreg_gemm_t &g, int b, int r, int k) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r >= g.R || k >= g.K) return v;
#pragma unroll
    for (int s = 0; s < HREG_MAX_SEGS; ++s) {
        if (s < g.nseg) {
            const hreg_seg_t &sg = g.seg[s];
            if (k >= sg.k0 && k < sg.k0 + sg.kc) {
                const int row = sg.gather ? sg.gather[r] : r / sg.row_div;
                const float *p = sg.base + (size_t)b * sg.batch_stride + (size_t)row * sg.ld +
                                 (k - sg.k0);
                v = *reinterpret_cast<const float4 *>(p);
                if (sg.rowscale) {
                    const float a = sg.rowscale[r];
                    v.x = fmul_rn(v.x, a); v.y = fmul_rn(v.y, a);
                    v.z = fmul_rn(v.z, a); v.w = fmul_rn(v.w, a);
                }
            }
        }
    }
    return v;
}

__device__ __forceinline__ float4 load_w4(const hreg_gemm_t &g, int b, int n, int k) {
    if (n >= g.N || k >= g.K) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float *p = g.W + (size_t)b * g.w_batch_stride + (size_t)n * g.ldw + k;
    return *reinterpret_cast<const float4 *>(p);
}


// one BM x BN output tile (r0, n0) of batch b (the body of gemm_nt_kernel and
// gemm_grouped_kernel)
template <int BM, int BN, int WM, int WN, int BK, bool ADD = false>
__device__ __forceinline__ void gemm_nt_tile(const hreg_gemm_t &g, const int b, const int r0, const int n0) {
    static_assert(WM * WN == 4, "4 waves");
    static_assert(BK == 16 || BK == 32, "BK");
    constexpr int LDS_STRIDE = BK + 4;          // pad: 16-row ds_read_b128 groups hit distinct slots
    constexpr int F4 = BK / 4;                  // float4 per row per chunk
    constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
    constexpr int TM = WTM / 32, TN = WTN / 32;  // 32x32 MFMA tiles per wave
    constexpr int A_LD = (BM * F4 + 255) / 256;  // float4 loads per thread per chunk
    constexpr int B_LD = (BN * F4 + 255) / 256;

    __shared__ __attribute__((aligned(16))) float As[2][BM * LDS_STRIDE];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDS_STRIDE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave / WN, wc = wave % WN;
    const int nchunks = (g.K + BK - 1) / BK;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

    float4 ra[A_LD], rb[B_LD];
    auto gload = [&](int c) {
#pragma unroll
        for (int i = 0; i < A_LD; ++i) {
            const int e = tid + i * 256;
            ra[i] = (e < BM * F4) ? load_a4(g, b, r0 + e / F4, c * BK + (e % F4) * 4)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) {
            const int e = tid + i * 256;
            rb[i] = (e < BN * F4) ? load_w4(g, b, n0 + e / F4, c * BK + (e % F4) * 4)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_LD; ++i) {
            const int e = tid + i * 256;
            if (e < BM * F4)
                *reinterpret_cast<float4 *>(&As[buf][(e / F4) * LDS_STRIDE + (e % F4) * 4]) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) {
            const int e = tid + i * 256;
            if (e < BN * F4)
                *reinterpret_cast<float4 *>(&Bs[buf][(e / F4) * LDS_STRIDE + (e % F4) * 4]) = rb[i];
        }
    };

    if (nchunks) {
        gload(0);
        lstore(0);
    }
    __syncthreads();

    const int h = lane >> 5, l32 = lane & 31;
    for (int c = 0; c < nchunks; ++c) {
        const int buf = c & 1;
        if (c + 1 < nchunks) gload(c + 1);
        // per 16-deep sub-chunk, lane half h takes k = sub*16 + h*8 + s for k-step s
        // (its 8 k-values are contiguous): the accumulation order of every output is
        // the same for every BK and tile shape, so results do not depend on R
#pragma unroll
        for (int s4 = 0; s4 < BK / 4 / 2; ++s4) {
            const int koff = (s4 >> 1) * 16 + h * 8 + (s4 & 1) * 4;
            float4 fa[TM], fb[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                fa[i] = *reinterpret_cast<const float4 *>(
                    &As[buf][(wr * WTM + i * 32 + l32) * LDS_STRIDE + koff]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                fb[j] = *reinterpret_cast<const float4 *>(
                    &Bs[buf][(wc * WTN + j * 32 + l32) * LDS_STRIDE + koff]);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32((&fa[i].x)[s], (&fb[j].x)[s],
                                                                         acc[i][j], 0, 0, 0);
        }
        if (c + 1 < nchunks) lstore(buf ^ 1);
        __syncthreads();
    }

    // epilogue: lane l, reg q -> row (q&3) + 8*(q>>2) + 4*h, col l&31
    // addends first, in a pass with no stores in it, so the (gathered) loads of a
    // lane's 16 * TM * TN outputs are all in flight together
    // (own instantiation: the plain kernels keep their register budget)
#pragma unroll
    for (int a = 0; a < (ADD ? 2 : 0); ++a) {
        if (a >= g.nadd) break;
        const hreg_seg_t &ad = g.add[a];
        const float *abase = ad.base + (size_t)b * ad.batch_stride;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = r0 + wr * WTM + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                const int rr = r < g.R ? r : g.R - 1;
                const float *arow = abase + (size_t)(ad.gather ? ad.gather[rr] : rr / ad.row_div) * ad.ld;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = n0 + wc * WTN + j * 32 + l32;
                    acc[i][j][q] = fadd_rn(acc[i][j][q], arow[n < g.N ? n : g.N - 1]);
                }
            }
    }
    float *out = g.out + (size_t)b * g.out_batch_stride;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wc * WTN + j * 32 + l32;
        if (n >= g.N) continue;
        float sc = 1.f, sh = 0.f, cn = 1.f;
        if (g.epi == HREG_EPI_AFFINE) {
            if (g.scale) sc = g.scale[n];
            if (g.shift) sh = g.shift[n];
        } else {
            cn = g.cnorm[(size_t)b * g.cnorm_batch_stride + n];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = r0 + wr * WTM + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (r < g.R) {
                    float y = acc[i][j][q];
                    if (g.epi == HREG_EPI_AFFINE) {
                        y = fadd_rn(fmul_rn(y, sc), sh);
                        if (g.relu) y = fmaxf(y, 0.f);
                    } else {
                        const float rn = g.rnorm[(size_t)b * g.rnorm_batch_stride + r];
                        y = y / fadd_rn(fmul_rn(rn, cn), 1e-6f);
                    }
                    out[(size_t)r * g.ldo + n] = y;
                }
            }
        }
    }
}

template <int BM, int BN, int WM, int WN, int BK, bool ADD = false>
__global__ __launch_bounds__(256) void gemm_nt_kernel(const hreg_gemm_t g) {
    gemm_nt_tile<BM, BN, WM, WN, BK, ADD>(g, blockIdx.z, blockIdx.x * BM, blockIdx.y * BN);
}

// Several independent GEMMs in one launch (hreg_gemm_grouped): a flat grid over every
// problem's 64 x 64 tiles, problem p owning blocks [start[p], start[p + 1]).  Each tile runs
// gemm_nt_kernel's body, so every output has the same bits as its own hreg_gemm launch (the
// accumulation order does not depend on the tile shape).
struct GemmGroup {
    hreg_gemm_t g[HREG_GEMM_GROUP_MAX];
    int start[HREG_GEMM_GROUP_MAX + 1];
    int tm[HREG_GEMM_GROUP_MAX];
    int tn[HREG_GEMM_GROUP_MAX];
    int n;
};

__global__ __launch_bounds__(256) void gemm_grouped_kernel(const GemmGroup gg) {
    const int bid = blockIdx.x;
    int p = 0;
    while (p + 1 < gg.n && bid >= gg.start[p + 1]) ++p;
    const int local = bid - gg.start[p];
    const int per_b = gg.tm[p] * gg.tn[p];
    const int b = local / per_b, rem = local - b * per_b;
    const int bx = rem % gg.tm[p], by = rem / gg.tm[p];
    gemm_nt_tile<64, 64, 2, 2, 32>(gg.g[p], b, bx * 64, by * 64);
}

// ------------------------------------------------------------------------
// The same GEMM with fp32-accurate products on the bf16 matrix cores (bf16x6,
// mfma_chain.h): every A and W value is split exactly into three bf16 pieces while it is
// staged into LDS (once per workgroup), and each 16-deep k sub-chunk of a 32x32 output
// tile is 6 v_mfma_f32_32x32x16_bf16 (a_h w_l, a_m w_m, a_l w_h, a_h w_m, a_m w_h, a_h w_h)
// instead of 8 v_mfma_f32_32x32x2_f32.  128 x 128 tiles, 4 waves of 64 x 64, K in 32-deep
// chunks: the next chunk is loaded into registers during this chunk's MFMAs, split and
// stored after a barrier (one LDS buffer of pieces, 60 KB: two workgroups per CU).  LDS
// rows of pieces are 32 bf16 + 8 pad (80 B: the 8-row groups of a ds_read_b128 hit
// distinct 16-byte bank quads).  Lane half h takes k = sub*16 + 8h + i of a sub-chunk,
// so the accumulation order of an output does not depend on R or the batch.
typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));

constexpr int G6_BM = 128, G6_BN = 128, G6_BK = 32, G6_LDR = G6_BK + 8;  // LDS row, in bf16

// x -> (hi, mid, lo) bf16 bit patterns: exact truncation split (mfma_chain.h split8)
__device__ __forceinline__ void split1(float v, uint32_t &hb, uint32_t &mb, uint32_t &lb) {
    const uint32_t xb = __float_as_uint(v);
    const float r = fsub_rn(v, __uint_as_float(xb & 0xffff0000u));
    const uint32_t rb = __float_as_uint(r);
    hb = xb >> 16;
    mb = rb >> 16;
    lb = __float_as_uint(fsub_rn(r, __uint_as_float(rb & 0xffff0000u))) >> 16;
}

// float4 of row `row`, k = k0..k0+3 -> three 8-byte piece stores
__device__ __forceinline__ void store_pieces(uint16_t *buf, int row, int k0, float4 v) {
    uint32_t h[4], m[4], l[4];
    split1(v.x, h[0], m[0], l[0]);
    split1(v.y, h[1], m[1], l[1]);
    split1(v.z, h[2], m[2], l[2]);
    split1(v.w, h[3], m[3], l[3]);
    constexpr int PS = 128 * G6_LDR;  // piece stride (bf16)
    uint16_t *p = buf + row * G6_LDR + k0;
    *reinterpret_cast<uint2 *>(p) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    *reinterpret_cast<uint2 *>(p + PS) = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
    *reinterpret_cast<uint2 *>(p + 2 * PS) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
}

__device__ __forceinline__ f32x16 mfma_b16(u32x4g a, u32x4g b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8g, a), __builtin_bit_cast(bf16x8g, b),
                                                   c, 0, 0, 0);
}

__global__ __launch_bounds__(256, 2) void gemm6_kernel(const hreg_gemm_t g) {
    constexpr int BM = G6_BM, BN = G6_BN, BK = G6_BK, LDR = G6_LDR, PS = 128 * LDR;
    constexpr int F4 = BK / 4, A_LD = BM * F4 / 256, B_LD = BN * F4 / 256;
    constexpr int TM = 2, TN = 2;  // 32x32 tiles per wave (64 x 64)
    __shared__ __attribute__((aligned(16))) uint16_t As[3 * PS];
    __shared__ __attribute__((aligned(16))) uint16_t Ws[3 * PS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int b = blockIdx.z, r0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int nchunks = (g.K + BK - 1) / BK;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

    float4 ra[A_LD], rb[B_LD];
    auto gload = [&](int c) {
#pragma unroll
        for (int i = 0; i < A_LD; ++i) {
            const int e = tid + i * 256;
            ra[i] = load_a4(g, b, r0 + e / F4, c * BK + (e % F4) * 4);
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) {
            const int e = tid + i * 256;
            rb[i] = load_w4(g, b, n0 + e / F4, c * BK + (e % F4) * 4);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int i = 0; i < A_LD; ++i) {
            const int e = tid + i * 256;
            store_pieces(As, e / F4, (e % F4) * 4, ra[i]);
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) {
            const int e = tid + i * 256;
            store_pieces(Ws, e / F4, (e % F4) * 4, rb[i]);
        }
    };

    gload(0);
    lstore();
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        if (c + 1 < nchunks) gload(c + 1);
#pragma unroll
        for (int sub = 0; sub < BK / 16; ++sub) {
            const int koff = sub * 16 + h * 8;
            u32x4g fa[TM][3], fw[TN][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    fa[i][p] = *reinterpret_cast<const u32x4g *>(&As[p * PS + (wr * 64 + i * 32 + l32) * LDR + koff]);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    fw[j][p] = *reinterpret_cast<const u32x4g *>(&Ws[p * PS + (wc * 64 + j * 32 + l32) * LDR + koff]);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    f32x16 c6 = acc[i][j];
                    c6 = mfma_b16(fa[i][0], fw[j][2], c6);
                    c6 = mfma_b16(fa[i][1], fw[j][1], c6);
                    c6 = mfma_b16(fa[i][2], fw[j][0], c6);
                    c6 = mfma_b16(fa[i][0], fw[j][1], c6);
                    c6 = mfma_b16(fa[i][1], fw[j][0], c6);
                    acc[i][j] = mfma_b16(fa[i][0], fw[j][0], c6);
                }
        }
        __syncthreads();  // every wave has read this chunk's pieces
        if (c + 1 < nchunks) {
            lstore();
            __syncthreads();
        }
    }

    // epilogue (gemm_nt_kernel's): lane l, reg q -> row (q&3) + 8*(q>>2) + 4*h, col l&31
    float *out = g.out + (size_t)b * g.out_batch_stride;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wc * 64 + j * 32 + l32;
        if (n >= g.N) continue;
        float sc = 1.f, sh = 0.f, cn = 1.f;
        if (g.epi == HREG_EPI_AFFINE) {
            if (g.scale) sc = g.scale[n];
            if (g.shift) sh = g.shift[n];
        } else {
            cn = g.cnorm[(size_t)b * g.cnorm_batch_stride + n];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = r0 + wr * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (r < g.R) {
                    float y = acc[i][j][q];
                    if (g.epi == HREG_EPI_AFFINE) {
                        y = fadd_rn(fmul_rn(y, sc), sh);
                        if (g.relu) y = fmaxf(y, 0.f);
                    } else {
                        const float rn = g.rnorm[(size_t)b * g.rnorm_batch_stride + r];
                        y = y / fadd_rn(fmul_rn(rn, cn), 1e-6f);
                    }
                    out[(size_t)r * g.ldo + n] = y;
                }
            }
        }
    }
}

bool seg_ok(const hreg_seg_t &s) {
    if (!s.base || s.ld <= 0 || (s.ld & 3) || (s.k0 & 3) || (s.kc & 3) || s.kc <= 0) return false;
    if (!s.gather && s.row_div < 1) return false;
    if (reinterpret_cast<uintptr_t>(s.base) & 15) return false;
    return true;
}

int gemm_check(const hreg_gemm_t &g) {
    if (g.R < 0 || g.N <= 0 || g.K <= 0 || g.batch < 1 || !g.W || !g.out) return HREG_ERR_INVALID;
    if (g.nseg < 1 || g.nseg > HREG_MAX_SEGS) return HREG_ERR_INVALID;
    if ((g.ldw & 3) || g.ldw < g.K || (reinterpret_cast<uintptr_t>(g.W) & 15)) return HREG_ERR_INVALID;
    if (g.ldo < g.N) return HREG_ERR_INVALID;
    if (g.epi == HREG_EPI_COSINE && (!g.rnorm || !g.cnorm)) return HREG_ERR_INVALID;
    for (int s = 0; s < g.nseg; ++s)
        if (!seg_ok(g.seg[s])) return HREG_ERR_INVALID;
    if (g.nadd < 0 || g.nadd > 2 || (g.nadd && g.epi != HREG_EPI_AFFINE)) return HREG_ERR_INVALID;
    for (int a = 0; a < g.nadd; ++a) {
        const hreg_seg_t &ad = g.add[a];
        if (!ad.base || ad.ld < g.N || (!ad.gather && ad.row_div < 1)) return HREG_ERR_INVALID;
    }
    return HREG_OK;
}

}  // namespace

extern "C" int hreg_gemm6(const hreg_gemm_t *gp, void *stream) {
    if (!gp) return HREG_ERR_INVALID;
    const hreg_gemm_t &g = *gp;
    if (const int rc = gemm_check(g)) return rc;
    if (g.nadd) return HREG_ERR_UNSUPPORTED;  // addends: hreg_gemm
    if (g.R == 0) return HREG_OK;
    dim3 grid((g.R + G6_BM - 1) / G6_BM, (g.N + G6_BN - 1) / G6_BN, g.batch);
    hipLaunchKernelGGL(gemm6_kernel, grid, dim3(256), 0, as_stream(stream), g);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_gemm(const hreg_gemm_t *gp, void *stream) {
    if (!gp) return HREG_ERR_INVALID;
    const hreg_gemm_t &g = *gp;
    if (const int rc = gemm_check(g)) return rc;
    if (g.R == 0) return HREG_OK;
    hipStream_t st = as_stream(stream);
    // tile choice: wide tiles (K in 16-deep chunks) for the big layers; 64x64 tiles
    // with 32-deep K chunks when a 128x128 grid would leave most of the 256 CUs idle
    // (the small mlp-head GEMMs: 2x fewer serial chunk round trips per block)
    const long tiles128 = (long)((g.R + 127) / 128) * ((g.N + 127) / 128) * g.batch;
    if (g.nadd) {
        // the addend GEMMs are short-K (memory-bound epilogue): small tiles, many blocks
        dim3 grid((g.R + 63) / 64, (g.N + 63) / 64, g.batch);
        hipLaunchKernelGGL((gemm_nt_kernel<64, 64, 2, 2, 32, true>), grid, dim3(256), 0, st, g);
    } else if (g.N <= 32) {
        dim3 grid((g.R + 255) / 256, (g.N + 31) / 32, g.batch);
        hipLaunchKernelGGL((gemm_nt_kernel<256, 32, 4, 1, 16>), grid, dim3(256), 0, st, g);
    } else if (g.N <= 64) {
        dim3 grid((g.R + 255) / 256, (g.N + 63) / 64, g.batch);
        hipLaunchKernelGGL((gemm_nt_kernel<256, 64, 4, 1, 16>), grid, dim3(256), 0, st, g);
    } else if (tiles128 < 256) {
        dim3 grid((g.R + 63) / 64, (g.N + 63) / 64, g.batch);
        hipLaunchKernelGGL((gemm_nt_kernel<64, 64, 2, 2, 32>), grid, dim3(256), 0, st, g);
    } else {
        // 128 x 128 tiles, K in 32-deep chunks (measured r1 against 16-deep chunks and
        // 128 x 256 tiles, tools/gemm_profile.py: half the barriers and load round trips per
        // MFMA; the same k-order in all three, bit-identical)
        dim3 grid((g.R + 127) / 128, (g.N + 127) / 128, g.batch);
        hipLaunchKernelGGL((gemm_nt_kernel<128, 128, 2, 2, 32>), grid, dim3(256), 0, st, g);
    }
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

extern "C" int hreg_gemm_grouped(const hreg_gemm_t *gs, int n, void *stream) {
    if (!gs || n < 1 || n > HREG_GEMM_GROUP_MAX) return HREG_ERR_INVALID;
    GemmGroup gg;
    int total = 0;
    for (int p = 0; p < n; ++p) {
        const hreg_gemm_t &g = gs[p];
        if (const int rc = gemm_check(g)) return rc;
        if (g.nadd) return HREG_ERR_UNSUPPORTED;  // addends: hreg_gemm
        gg.g[p] = g;
        gg.tm[p] = (g.R + 63) / 64;
        gg.tn[p] = (g.N + 63) / 64;
        gg.start[p] = total;
        total += gg.tm[p] * gg.tn[p] * g.batch;
    }
    gg.start[n] = total;
    gg.n = n;
    if (total == 0) return HREG_OK;
    hipLaunchKernelGGL(gemm_grouped_kernel, dim3(total), dim3(256), 0, as_stream(stream), gg);
    HREG_CHECK_LAUNCH();
    return HREG_OK;
}

