/*
 * hregnet_oracle.c -- CPU restatement of the reference's index/byte-exact ops.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline) -- never as the product path.
 *
 * What is restated (reference = /root/reference, read as text only):
 *   - opt_n_threads                    models/PointUtils/src/cuda_utils.h:22-26
 *   - furthest_point_sampling_kernel   models/PointUtils/src/furthest_point_sampling_gpu.cu:84-206
 *     emulated literally: bs "threads" each scan k = t, t+bs, ... keeping the
 *     first strictly larger d2 (.cu:122-134), then the shared-memory tree
 *     (__update .cu:75-80, tree .cu:140-199) that keeps the lower slot on ties.
 *   - weighted_furthest_point_sampling_kernel  .cu:254-375 (d = w2 * |p - p_old|^2, .cu:299)
 *   - gather_points_kernel_fast        .cu:7-21
 *   - gather_points_grad_kernel_fast   .cu:41-55 (sequential accumulation order)
 *   - pytorch3d.ops.knn_points (third-party, pinned pytorch3d==0.7.8,
 *     Dockerfile:44-46; not vendored): brute-force squared L2,
 *     dist = sum_d (p1_d - p2_d)^2 accumulated sequentially over d, K smallest
 *     returned ascending.  Tie order in pytorch3d is an unstable torch.sort,
 *     so the canonical order here is (dist, idx) ascending -- "parity
 *     unpinned" against pytorch3d itself.
 *   - the nearest-neighbour-within-radius search of open3d's registration_icp
 *     (third-party open3d, not vendored; caller test/test_v4.py:144-158): the
 *     nearest target point with dist^2 < r^2 strictly (dist in the order above),
 *     ties to the lowest index -- the choice of the GPU kernel (csrc/icp.hip);
 *     parity unpinned against open3d's kd-tree.
 *
 * Float policy: compiled with -ffp-contract=off, so every a*a+b*b is two
 * roundings, matching the non-contracted CPU/PyTorch reference path.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* cuda_utils.h:22-26 -- same double-precision log formula, truncated. */
int oracle_opt_n_threads(int work_size) {
    if (work_size < 1) return 1;
    const int pow_2 = (int)(log((double)work_size) / log(2.0));
    int v = 1 << pow_2;
    if (v > 1024) v = 1024;
    if (v < 1) v = 1;
    return v;
}

/* .cu:84-206 / .cu:254-375, one cloud.  weights may be NULL (plain FPS).
 * temp is scratch [n]: the initial running minima are temp0's (the caller's temp, .cu:130), or
 * 1e10 when temp0 is NULL (as models/utils.py:25 fills it). */
static void fps_one_cloud(const float *xyz, const float *w, const float *temp0, int n, int m,
                          float *temp, float *dists, int *dists_i, int32_t *idx) {
    const int bs = oracle_opt_n_threads(n);
    if (m <= 0) return;
    for (int k = 0; k < n; ++k) temp[k] = temp0 ? temp0[k] : 1e10f;
    int old = 0;
    idx[0] = old;
    for (int j = 1; j < m; ++j) {
        const float x1 = xyz[old * 3 + 0], y1 = xyz[old * 3 + 1], z1 = xyz[old * 3 + 2];
        for (int t = 0; t < bs; ++t) {
            int besti = 0;
            float best = -1.0f;
            for (int k = t; k < n; k += bs) {
                const float x2 = xyz[k * 3 + 0], y2 = xyz[k * 3 + 1], z2 = xyz[k * 3 + 2];
                float d = (x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1) + (z2 - z1) * (z2 - z1);
                if (w) d = w[k] * d;
                const float d2 = fminf(d, temp[k]);
                temp[k] = d2;
                besti = d2 > best ? k : besti;
                best = d2 > best ? d2 : best;
            }
            dists[t] = best;
            dists_i[t] = besti;
        }
        /* tree: for s = bs/2 .. 1: slot t < s merges t and t+s (.cu:140-199) */
        for (int s = bs / 2; s >= 1; s >>= 1) {
            for (int t = 0; t < s; ++t) {
                const float v1 = dists[t], v2 = dists[t + s];
                const int i1 = dists_i[t], i2 = dists_i[t + s];
                dists[t] = fmaxf(v1, v2);
                dists_i[t] = v2 > v1 ? i2 : i1;
            }
        }
        old = dists_i[0];
        idx[j] = old;
    }
}

/* furthest_point_sampling_wrapper (fps.cpp:33-43) semantics over b clouds; temp0 [b][n] the
 * caller's temp contents (NULL: 1e10). */
int oracle_fps_temp(const float *xyz, const float *weights, const float *temp0, int b, int n, int m,
                    int32_t *idx) {
    if (b <= 0 || n <= 0 || m <= 0) return 0;
    int rc = 0;
#pragma omp parallel for schedule(dynamic, 1)
    for (int c = 0; c < b; ++c) {
        float *temp = (float *)malloc(sizeof(float) * (size_t)n);
        float *dists = (float *)malloc(sizeof(float) * 1024);
        int *dists_i = (int *)malloc(sizeof(int) * 1024);
        if (!temp || !dists || !dists_i) {
            rc = -1;
        } else {
            fps_one_cloud(xyz + (size_t)c * n * 3, weights ? weights + (size_t)c * n : NULL,
                          temp0 ? temp0 + (size_t)c * n : NULL, n, m, temp, dists, dists_i,
                          idx + (size_t)c * m);
        }
        free(temp); free(dists); free(dists_i);
    }
    return rc;
}

int oracle_fps(const float *xyz, const float *weights, int b, int n, int m, int32_t *idx) {
    return oracle_fps_temp(xyz, weights, NULL, b, n, m, idx);
}

/* gather_points_kernel_fast (.cu:7-21): out[b,c,j] = points[b,c,idx[b,j]] */
void oracle_gather_points(const float *points, const int32_t *idx, int b, int c, int n, int m,
                          float *out) {
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (int j = 0; j < m; ++j)
                out[((size_t)bi * c + ci) * m + j] =
                    points[((size_t)bi * c + ci) * n + idx[(size_t)bi * m + j]];
}

/* gather_points_grad_kernel_fast (.cu:41-55); grad_points must be zeroed. */
void oracle_gather_points_grad(const float *grad_out, const int32_t *idx, int b, int c, int n,
                               int m, float *grad_points) {
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (int j = 0; j < m; ++j)
                grad_points[((size_t)bi * c + ci) * n + idx[(size_t)bi * m + j]] +=
                    grad_out[((size_t)bi * c + ci) * m + j];
}

/* ---- kNN (pytorch3d.ops.knn_points semantics, canonical tie order) ---- */

typedef struct { float d; int32_t i; } cand_t;

static inline int cand_less(cand_t a, cand_t b) {
    return a.d < b.d || (a.d == b.d && a.i < b.i);
}

/* Keep a sorted list of the K best (dist, idx); insertion for each db point. */
static void knn_one_query(const float *q, const float *db, int n2, int dim, int K,
                          cand_t *list, int32_t *out_idx, float *out_dist) {
    int size = 0;
    for (int p = 0; p < n2; ++p) {
        const float *x = db + (size_t)p * dim;
        float d = 0.0f;
        for (int e = 0; e < dim; ++e) {
            const float diff = q[e] - x[e];
            d = d + diff * diff;
        }
        cand_t c = {d, p};
        if (size < K) {
            int pos = size++;
            while (pos > 0 && cand_less(c, list[pos - 1])) { list[pos] = list[pos - 1]; --pos; }
            list[pos] = c;
        } else if (cand_less(c, list[K - 1])) {
            int pos = K - 1;
            while (pos > 0 && cand_less(c, list[pos - 1])) { list[pos] = list[pos - 1]; --pos; }
            list[pos] = c;
        }
    }
    for (int k = 0; k < K; ++k) {
        if (k < size) { out_idx[k] = list[k].i; out_dist[k] = list[k].d; }
        else { out_idx[k] = -1; out_dist[k] = 0.0f; }
    }
}

/* p1 [b, n1, dim], p2 [b, n2, dim] -> idx [b, n1, K] (int32), dist [b, n1, K] */
int oracle_knn(const float *p1, const float *p2, int b, int n1, int n2, int dim, int K,
               int32_t *idx, float *dist) {
    if (K <= 0) return 0;
    int rc = 0;
#pragma omp parallel
    {
        cand_t *list = (cand_t *)malloc(sizeof(cand_t) * (size_t)K);
        if (!list) rc = -1;
#pragma omp for schedule(static) collapse(2)
        for (int bi = 0; bi < b; ++bi)
            for (int qi = 0; qi < n1; ++qi) {
                if (!list) continue;
                const size_t qo = (size_t)bi * n1 + qi;
                knn_one_query(p1 + qo * dim, p2 + (size_t)bi * n2 * dim, n2, dim, K, list,
                              idx + qo * K, dist + qo * K);
            }
        free(list);
    }
    return rc;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* open3d registration_icp correspondence search, brute force: out[i] = argmin_j d2(q_i, p_j)
 * over d2 < r2 (ties: lowest j), -1 when none; OpenMP over queries. */
int oracle_nn_radius(const float *q, int nq, const float *p, int np, float r2, int32_t *out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nq; ++i) {
        const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
        float best = INFINITY;
        int bid = -1;
        for (int j = 0; j < np; ++j) {
            const float dx = qx - p[3 * j], dy = qy - p[3 * j + 1], dz = qz - p[3 * j + 2];
            const float d = (dx * dx + dy * dy) + dz * dz;
            if (d < best) { best = d; bid = j; }
        }
        out[i] = best < r2 ? bid : -1;
    }
    return 0;
}
