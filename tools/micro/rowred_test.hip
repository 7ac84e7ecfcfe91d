// Unit check of csrc/rowred.h on the GPU: butterfly row reductions (bfly32 / bfly16, max and
// sum), the broadcast back (bcast32) and the slot -> value mapping, against host loops.
// hipcc --offload-arch=gfx950 -O3 -I pcd_reg_hregnet_amd/csrc tools/micro/rowred_test.hip -o /tmp/rowred_test
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "rowred.h"

using namespace hreg_rowred;

constexpr int N = 16, N2 = 64;

// out layout per kernel: [lane][N] (slots / broadcast values)
__global__ void k_rowred(const float *in, const float *in2, float *mx32, float *sm32, float *bc32, float *mx16,
                         float *big32, float *st32, float *st16) {
    const int lane = threadIdx.x;
    float v[N], w[N], b[N], u[N], z[N2];
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = w[i] = b[i] = u[i] = in[lane * N + i];
#pragma unroll
    for (int i = 0; i < N2; ++i) z[i] = in2[lane * N2 + i];
    bfly32<MaxNN>(v, lane);
    bfly32<Sum>(w, lane);
    bfly32<MaxNN>(b, lane);
    bcast32(b, lane);
    bfly16<MaxNN>(u, lane);
    bfly32<MaxNN>(z, lane);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        mx32[lane * N + i] = i < N / 8 ? v[i] : -1.f;
        sm32[lane * N + i] = i < N / 8 ? w[i] : -1.f;
        bc32[lane * N + i] = b[i];
        mx16[lane * N + i] = i < N / 4 ? u[i] : -1.f;
    }
#pragma unroll
    for (int i = 0; i < N2; ++i) big32[lane * N2 + i] = i < N2 / 8 ? z[i] : -1.f;
    // tile layout store: one per-group row of 32 channels (h = lane >> 5 halves); st16: two groups
    store_slots<N, true>(st32, 0, v, lane);
    store_slots<N, false>(st16 + ((lane >> 4) & 1) * 32, 0, u, lane);
}

static int chan(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

int main() {
    std::vector<float> in(64 * N), in2(64 * N2);
    srand(7);
    for (auto &x : in) x = (float)(rand() % 100000) / 977.f;
    for (auto &x : in2) x = (float)(rand() % 100000) / 977.f;
    float *d[9];
    const size_t sz[9] = {in.size(), in2.size(), in.size(), in.size(), in.size(), in.size(), in2.size(), 64, 64};
    for (int i = 0; i < 9; ++i) {
        if (hipMalloc(&d[i], sz[i] * 4) != hipSuccess) return 2;
        hipMemset(d[i], 0, sz[i] * 4);
    }
    hipMemcpy(d[0], in.data(), in.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d[1], in2.data(), in2.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rowred, dim3(1), dim3(64), 0, 0, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8]);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<float> o[9];
    for (int i = 2; i < 9; ++i) {
        o[i].resize(sz[i]);
        hipMemcpy(o[i].data(), d[i], sz[i] * 4, hipMemcpyDeviceToHost);
    }
    int bad = 0;
    auto red = [&](const std::vector<float> &x, int n, int lane0, int nl, int val, bool sum) {
        double s = 0;
        float m = 0;
        for (int l = lane0; l < lane0 + nl; ++l) {
            s += x[l * n + val];
            m = fmaxf(m, x[l * n + val]);
        }
        return sum ? (float)s : m;
    };
    for (int lane = 0; lane < 64; ++lane) {
        const int h = lane >> 5, b = (lane >> 2) & 7, b16 = (lane >> 2) & 3, g16 = lane >> 4;
        for (int i = 0; i < N / 8; ++i) {
            const int val = i + (N / 8) * b;
            const float em = red(in, N, 32 * h, 32, val, false), es = red(in, N, 32 * h, 32, val, true);
            if (o[2][lane * N + i] != em) ++bad, printf("max32 lane %d slot %d: %g vs %g\n", lane, i, o[2][lane * N + i], em);
            if (fabsf(o[3][lane * N + i] - es) > 1e-5f * es) ++bad, printf("sum32 lane %d slot %d: %g vs %g\n", lane, i, o[3][lane * N + i], es);
        }
        for (int i = 0; i < N; ++i) {
            const float em = red(in, N, 32 * h, 32, i, false);
            if (o[4][lane * N + i] != em) ++bad, printf("bcast32 lane %d val %d: %g vs %g\n", lane, i, o[4][lane * N + i], em);
        }
        for (int i = 0; i < N / 4; ++i) {
            const int val = i + (N / 4) * b16;
            const float em = red(in, N, 16 * g16, 16, val, false);
            if (o[5][lane * N + i] != em) ++bad, printf("max16 lane %d slot %d: %g vs %g\n", lane, i, o[5][lane * N + i], em);
        }
        for (int i = 0; i < N2 / 8; ++i) {
            const int val = i + (N2 / 8) * b;
            const float em = red(in2, N2, 32 * h, 32, val, false);
            if (o[6][lane * N2 + i] != em) ++bad, printf("max32x64 lane %d slot %d: %g vs %g\n", lane, i, o[6][lane * N2 + i], em);
        }
    }
    for (int h = 0; h < 2; ++h)
        for (int q = 0; q < 16; ++q) {
            const float em = red(in, N, 32 * h, 32, q, false);
            if (o[7][chan(q, h)] != em) ++bad, printf("store32 h %d q %d: %g vs %g\n", h, q, o[7][chan(q, h)], em);
        }
    for (int g = 0; g < 4; ++g)
        for (int q = 0; q < 16; ++q) {
            // DPP row g: rows of group (g & 1) of half (g >> 1)
            const int h = g >> 1, grp = g & 1;
            const float em = red(in, N, 16 * g, 16, q, false);
            const float got = o[8][grp * 32 + chan(q, h)];
            if (got != em) ++bad, printf("store16 g %d q %d: %g vs %g\n", g, q, got, em);
        }
    printf(bad ? "rowred: %d mismatches\n" : "rowred: ok\n", bad);
    return bad ? 1 : 0;
}
