/*
 * hregnet_amd.h -- C ABI of the MI355X-native HRegNet forward path.
 *
 * Plain pointers and sizes only: every float/int pointer is a DEVICE pointer
 * (HBM), `stream` is a hipStream_t passed as void*.  Calls enqueue work on
 * that stream and return immediately (asynchronous, like the reference's
 * launches on at::cuda::getCurrentCUDAStream(), furthest_point_sampling.cpp:16).
 * Every entry returns a status code instead of printing and calling exit(-1)
 * as the reference launchers do (furthest_point_sampling_gpu.cu:35-38).
 * Callers allocate every buffer (reference models/utils.py:24-25,48-49,71,84).
 *
 * Reference interface replaced by each entry (reference = UpendraArun/pcd_reg_hregnet):
 *   hreg_furthest_point_sampling          <- point_utils_cuda.furthest_point_sampling_wrapper
 *                                            (models/PointUtils/src/furthest_point_sampling.cpp:33-43,
 *                                             point_utils_api.cpp:10)
 *   hreg_weighted_furthest_point_sampling <- point_utils_cuda.weighted_furthest_point_sampling_wrapper
 *                                            (furthest_point_sampling.cpp:45-55, point_utils_api.cpp:11)
 *   hreg_gather_points                    <- point_utils_cuda.gather_points_wrapper
 *                                            (furthest_point_sampling.cpp:10-19, point_utils_api.cpp:8)
 *   hreg_gather_points_grad               <- point_utils_cuda.gather_points_grad_wrapper
 *                                            (furthest_point_sampling.cpp:21-31, point_utils_api.cpp:9)
 *   hreg_knn_points                       <- pytorch3d.ops.knn_points (pytorch3d 0.7.8, Dockerfile:44-46;
 *                                            call sites models/HRegNet/layers.py:20,278,316,322,434)
 *   hreg_knn_gather                       <- pytorch3d.ops.knn_gather (layers.py:25,279,288,317,...)
 *   hreg_knn_group                        <- knn_group() (models/HRegNet/layers.py:9-27), fused
 *   hreg_gemm                             <- nn.Conv1d/Conv2d 1x1 + BatchNorm(eval) + ReLU stacks
 *                                            (layers.py:115-130,183-198,246-268,417-431) and the
 *                                            cosine-similarity contraction (layers.py:29-41,290-301)
 *   hreg_attend                           <- channel-max -> softmax_k -> attentive sums
 *                                            (layers.py:150-159, 329-337, 384-390, 446-450)
 *   hreg_group_max                        <- torch.max(x, dim=k) (layers.py:202, 208)
 *   hreg_head_out                         <- mlp3 + softplus(+0.001) / sigmoid (layers.py:161-163,393-394,451-452)
 *                                            and the sigma->weight normalisation (models/HRegNet/models.py:30-32)
 *   hreg_row_norms                        <- torch.norm(desc, dim=-1) inside calc_cosine_similarity (layers.py:38-39)
 *   hreg_sim_gather                       <- max-normalised similarity gathered at the desc kNN (layers.py:296-313,345-362)
 *   hreg_pair_feats                       <- geometric/weight/similarity feature rows (layers.py:279-288,364-370,437-445)
 *   hreg_weighted_svd                     <- WeightedSVDHead.forward (layers.py:469-504) + T = T_ @ T_prev
 *                                            composition (models/HRegNet/models.py:100-127)
 *   hreg_transform_points                 <- R @ xyz^T + t (models/HRegNet/models.py:91-92,113-114)
 *   hreg_bn_* / hreg_gemm_tn / hreg_adam_step <- train-mode BatchNorm, conv weight gradients and
 *                                            optim.Adam of the training step (train/train_reg_v0.py:241-296)
 *   hreg_copy_rows ... hreg_transformation_loss_bwd <- forward/backward of the training graph
 *                                            (train_reg_v0.py:241-296 over layers.py / models.py)
 *   hreg_transformation_loss              <- transformation_loss + calc_rot_rre_err + calc_tran_rte_err
 *                                            (losses/losses.py:97-164; callers train/train_reg_v1.py:101,252)
 *   hreg_calib_metrics                    <- CalibEval.add_batch / geodesic_distance
 *                                            (metrics/calibeval.py:72-113,197-214; caller test/test_v3.py:130-140)
 *   hreg_icp_init / _iterate / _result    <- open3d.pipelines.registration.registration_icp, point-to-point
 *                                            (test/test_v4.py:140-158; third-party, not vendored)
 */
#ifndef HREGNET_AMD_H
#define HREGNET_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    HREG_OK = 0,
    HREG_ERR_INVALID = 1,     /* bad argument (null pointer, negative size, unsupported shape) */
    HREG_ERR_LAUNCH = 2,      /* hipGetLastError() after a launch */
    HREG_ERR_UNSUPPORTED = 3  /* shape outside what the kernels implement (e.g. K > 64) */
};

/* Sticky error bits that asynchronous kernels raise on the device (no host round trip
 * at launch time); read (and optionally cleared) by hreg_device_status. */
enum {
    HREG_STATUS_FPS_TIMEOUT = 1  /* multi-workgroup FPS (n > 16384): a participant's
                                    exchange poll expired; that cloud's idx holds zeros */
};

/* ---------------- point_utils_cuda boundary ---------------- */

/* points [b,n,3] f32, temp [b,n] f32 (required for n > 16384, may be NULL below): for n <=
 * 16384 (weighted: 8192) its contents are the initial running minima, read as the reference's
 * kernel reads them (.cu:130, d2 = min(d, temp[k]); its callers fill 1e10, models/utils.py:25;
 * NULL: 1e10) and it receives the final running minima; above, the multi-workgroup kernel keeps
 * its exchange slots there (contents not read, unspecified after), and the single-workgroup
 * memory kernel (when the spin budget cannot hold a cluster) its running minima (read and
 * written as the reference's), idx [b,m] int32 (out), sampled_xyz [b,m,3] (optional out:
 * gathered coordinates of idx). */
/* hreg_furthest_point_sampling for a caller that guarantees at most `concurrent` (>= 1)
 * multi-workgroup FPS launches (clouds above 16384 points) of this process run at once -- e.g. a
 * graph whose one stage-1 stream carries all of them: such a launch may keep more clouds' worker
 * waves spinning at once: 3/4 of the kernel's resident waves on the device (occupancy API x CU
 * count) / concurrent, capped at 4096 waves, instead of resident waves / GPU_MAX_HW_QUEUES capped
 * at 256.  Same results as hreg_furthest_point_sampling. */
int hreg_fps_bounded(int b, int n, int m, const float *points, float *temp, int32_t *idx,
                     float *sampled_xyz, int concurrent, void *stream);
/* FPS over the clouds' spatial index (ws: hreg_spatial_index of the same points, enqueued
 * before), exact pruning: a point group whose box cannot hold a point nearer the new centre than
 * its largest running minimum is skipped (the same idx as hreg_furthest_point_sampling; temp, if
 * not NULL, receives the final running minima [b][n] as the reference leaves them).
 *   n == 16384: the sorted copy in registers, 256-point groups (one 512-thread workgroup per cloud);
 *   16384 < n <= 65536, n % 64 == 0 (Model_V2): one 1024-thread workgroup per cloud, running minima
 *   in registers, the index's 64-point blocks read from ws when their box passes;
 *   other sizes: hreg_furthest_point_sampling (temp then required above 16384 points).
 * Replaces furthest_point_sampling_kernel for level 1 (furthest_point_sampling_gpu.cu:84-206). */
int hreg_fps_indexed(int b, int n, int m, const float *points, const void *ws, float *temp,
                     int32_t *idx, float *sampled_xyz, void *stream);
/* hreg_fps_indexed for 16384-point clouds on the small-footprint pruned kernel (4 waves, running
 * minima in registers, block coordinates read from the index; the throughput executor's batched
 * level-1 stage); the same selections and temp.  Other sizes: hreg_fps_indexed. */
int hreg_fps_indexed_lean(int b, int n, int m, const float *points, const void *ws, float *temp,
                          int32_t *idx, float *sampled_xyz, void *stream);
int hreg_furthest_point_sampling(int b, int n, int m, const float *points, float *temp,
                                 int32_t *idx, float *sampled_xyz, void *stream);

/* as above with weights [b,n]: d = w_k * |p_k - p_old|^2 */
int hreg_weighted_furthest_point_sampling(int b, int n, int m, const float *points,
                                          const float *weights, float *temp, int32_t *idx,
                                          float *sampled_xyz, void *stream);

/* points [b,c,n], idx [b,npoints] -> out [b,c,npoints] */
int hreg_gather_points(int b, int c, int n, int npoints, const float *points, const int32_t *idx,
                       float *out, void *stream);

/* grad_out [b,c,npoints] scatter-added into grad_points [b,c,n] (caller zeroes it) */
int hreg_gather_points_grad(int b, int c, int n, int npoints, const float *grad_out,
                            const int32_t *idx, float *grad_points, void *stream);

/* ---------------- pytorch3d.ops boundary ---------------- */

/* p1 [b,n1,dim], p2 [b,n2,dim] -> K nearest of each p1 row in p2 by squared L2,
 * ascending (dist, idx).  dists [b,n1,k] f32; idx64 [b,n1,k] int64 and/or
 * idx32 [b,n1,k] int32 (either may be NULL); nn [b,n1,k,dim] optional.
 * k <= 64.  Rows beyond n2 (k > n2) get idx -1, dist 0, nn 0. */
int hreg_knn_points(const float *p1, const float *p2, int b, int n1, int n2, int dim, int k,
                    float *dists, int64_t *idx64, int32_t *idx32, float *nn, void *stream);

/* x [b,n,c], idx [b,m,k] int64 -> out [b,m,k,c]; idx < 0 gives zeros */
int hreg_knn_gather(const float *x, const int64_t *idx, int b, int n, int c, int m, int k,
                    float *out, void *stream);

/* ---------------- fused stages of the HRegNet forward ---------------- */

/* knn_group (layers.py:9-27) for nb clouds: query q [nb,m,3], database p [nb,n,3].
 * Outputs per (cloud, query, neighbour) row r = (c*m + i)*k + j:
 *   gidx [nb*m*k] int32 = c*n + idx (global row of the neighbour in p),
 *   geom [nb*m*k][4] = (p - q, |p - q|), knn_xyz [nb*m*k][3] (optional). */
int hreg_knn_group(const float *q, const float *p, int nb, int m, int n, int k, int32_t *gidx,
                   float *geom, float *knn_xyz, void *stream);

/* One K-segment of the GEMM's activation operand A (rows x K, row-major). */
typedef struct {
    const float *base;       /* [rows][ld] */
    const int32_t *gather;   /* optional: source row = gather[r] */
    const float *rowscale;   /* optional: value *= rowscale[r] (attentive map, layers.py:158) */
    int64_t batch_stride;    /* floats added per grid.z batch to base */
    int ld;                  /* row stride in floats, multiple of 4 */
    int k0;                  /* first K column of this segment, multiple of 4 */
    int kc;                  /* K columns in this segment, multiple of 4 */
    int row_div;             /* source row = r / row_div when gather == NULL (>= 1) */
} hreg_seg_t;

#define HREG_MAX_SEGS 4
#define HREG_EPI_AFFINE 0 /* y = acc * scale[n] + shift[n]; optional ReLU */
#define HREG_EPI_COSINE 1 /* y = acc / (rnorm[r] * cnorm[n] + 1e-6) */

/* out[r][n] = epi( sum_k A[r][k] * W[n][k] ), r < R, n < N, k < K, fp32 MFMA. */
typedef struct {
    hreg_seg_t seg[HREG_MAX_SEGS];
    int nseg;
    int R, N, K;
    int batch;               /* grid.z batches (>= 1) */
    int ldw;                 /* W row stride (>= K), multiple of 4 */
    int64_t w_batch_stride;
    const float *W;          /* [N][ldw] */
    const float *scale;      /* [N] or NULL (1) */
    const float *shift;      /* [N] or NULL (0) */
    int relu;
    int epi;
    const float *rnorm;      /* [R] per batch (EPI_COSINE) */
    const float *cnorm;      /* [N] per batch (EPI_COSINE) */
    int64_t rnorm_batch_stride, cnorm_batch_stride;
    float *out;              /* [R][ldo] */
    int ldo;
    int64_t out_batch_stride;
    /* optional pre-epilogue addends (EPI_AFFINE): acc = (acc + add[0][row0][n]) + add[1][row1][n],
     * row_i = add[i].gather ? add[i].gather[r] : r / add[i].row_div; k0/kc/rowscale unused.
     * A 1x1 conv over a concatenation [x_r | u_{r/k} | v_{idx[r]}] is W_x x_r + (W_u u)_{r/k} +
     * (W_v v)_{idx[r]}: the repeated / gathered parts are multiplied once per source row
     * (CoarseReg convs_1, layers.py:364-384) and added here. */
    hreg_seg_t add[2];
    int nadd;
} hreg_gemm_t;

int hreg_gemm(const hreg_gemm_t *g, void *stream);

/* n <= HREG_GEMM_GROUP_MAX independent hreg_gemm problems (no addends) in ONE launch: the
 * grid runs every problem's 64 x 64 tiles; each output has the bits its own hreg_gemm launch
 * gives (the per-output accumulation order does not depend on the tile shape).  For the
 * per-row products the registration heads precompute from the feature-extraction outputs
 * (engine.head_products). */
#define HREG_GEMM_GROUP_MAX 6
int hreg_gemm_grouped(const hreg_gemm_t *gs, int n, void *stream);

/* hreg_gemm with fp32-accurate products on the bf16 matrix cores (bf16x6: A and W split
 * exactly into three bf16 pieces while staged into LDS, 6 v_mfma_f32_32x32x16_bf16 per
 * 16-deep k sub-chunk; gemm.hip gemm6_kernel).  Same arguments; addends (nadd > 0) are
 * not supported (HREG_ERR_UNSUPPORTED).  Accumulation order independent of R / batch. */
int hreg_gemm6(const hreg_gemm_t *g, void *stream);

/* Attentive pooling over groups of k rows (layers.py:150-159 and siblings).
 * logits_src [G*k][C] : a = softmax_k(max_c logits_src[r][c])  -> attw [G*k] (optional)
 * values: att[g][c] = sum_j a[g,j] * V[row(g,j)][c], V = vals (row = g*k+j) or
 *         vals gathered by vgather[g*k+j]; att optional [G][ldatt]
 * xyz: kp[g][:] = sum_j a[g,j] * xyz_rows[g*k+j][:] (optional, [G*k][3] -> [G][3]) */
int hreg_attend(const float *logits_src, int C, int ldl, int G, int k, float *attw,
                const float *vals, const int32_t *vgather, int Cv, int ldv, float *att, int ldatt,
                const float *xyz_rows, float *kp, void *stream);

/* out[g][c] = max_j x[g*k+j][c] over groups of k rows, x [G*k][ldx] */
int hreg_group_max(const float *x, int G, int k, int C, int ldx, float *out, int ldo, void *stream);

#define HREG_HEAD_SOFTPLUS 0 /* sigma = softplus(z) + 0.001 (layers.py:162) */
#define HREG_HEAD_SIGMOID 1  /* w = sigmoid(z) (layers.py:394) */
/* z[r] = dot(x[r][:C], w3) + b3 for rows of nclouds x rows_per_cloud; writes
 * out[r]; if weights_out != NULL also w = 1/(sigma+1e-5) / mean_cloud(.) (models.py:30-32). */
int hreg_head_out(const float *x, int C, int ldx, int nclouds, int rows_per_cloud,
                  const float *w3, const float *b3, int mode, float *out, float *weights_out,
                  void *stream);

/* weights = (1/(sigma+1e-5)) / mean_cloud(1/(sigma+1e-5)) (models.py:30-32) over
 * nclouds x rows_per_cloud sigmas. */
int hreg_sigma_weights(const float *sigma, int nclouds, int rows_per_cloud, float *weights,
                       void *stream);

/* The whole mlp1 -> mlp2 -> mlp3 head of KeypointDetector (layers.py:124-132,161-163),
 * CoarseReg (layers.py:262-268,389-394) and FineReg (layers.py:425-431,451-452) in one
 * launch (mlp_head.hip): x [nclouds*rows_per_cloud][ldx] (first C columns, 16-byte
 * aligned rows, C in {64,128,256,512}, rows a multiple of 32) -> out [rows] =
 * softplus(z)+0.001 or sigmoid(z); weights_out as hreg_head_out.  table: engine.mlp_head_table
 * (hreg_mlp_head_table_floats(C) floats; -1 for an unsupported C). */
int hreg_mlp_head_table_floats(int C);
int hreg_mlp_head(const float *table, int C, const float *x, int ldx, int nclouds,
                  int rows_per_cloud, int mode, float *out, float *weights_out, void *stream);

/* hreg_mlp_head with fp32-accurate products on the bf16 matrix cores (bf16x6,
 * mlp_head.hip): same arguments and outputs, table = hreg_mlp_head6_table_floats(C)
 * floats (engine.mlp_head_table6), 16-byte aligned. */
int hreg_mlp_head6_table_floats(int C);
int hreg_mlp_head6(const float *table, int C, const float *x, int ldx, int nclouds,
                   int rows_per_cloud, int mode, float *out, float *weights_out, void *stream);
/* hreg_mlp_head6 with the row tiles per workgroup: 0 = the default (2-4: fewer weight bytes per
 * MFMA when launches share the chip), 1 = one 32-row tile per workgroup (more workgroups for a
 * small batch alone on the GPU).  Same outputs, bit for bit. */
int hreg_mlp_head6x(const float *table, int C, const float *x, int ldx, int nclouds,
                    int rows_per_cloud, int mode, float *out, float *weights_out, int row_tiles,
                    void *stream);

/* ---- data side in front of the path (perturb.hip) ----
 * Twists x = (w, v) [n][6], SE(3) matrices g [n][16] row-major. */
/* g = SE3.exp(x) (transform/rodrigues.py:526-553) */
int hreg_se3_exp(const float *x, int n, float *g, void *stream);
/* x = SE3.log(g) (transform/rodrigues.py:571-582 with SO3.log :330-370) */
int hreg_se3_log(const float *g, int n, float *x, void *stream);
#define HREG_TWIST_UNIFORM 0          /* dataset_transforms.py:96-98 */
#define HREG_TWIST_GAUSSIAN 1         /* dataset_transforms.py:100-105 */
#define HREG_TWIST_INVERSE_GAUSSIAN 2 /* dataset_transforms.py:107-122 */
/* UniformTransformSE3.generate_transform (transform/dataset_transforms.py:79-126) from
 * its random draws: samples [n][6] (w draw, t draw), amp_tran [n][2] (radians, metres)
 * -> x [n][6] = SE3.log([SO3.exp(w) | t]) */
int hreg_twists_from_samples(const float *samples, const float *amp_tran, int n, int distribution,
                             float *x, void *stream);
/* TruckScenesPerturbation.lidar_to_lidar (dataset/man_dataset.py:606-631) for nb
 * clouds: out[b] = SE3.transform(exp(x[b]), pts[b]), pts/out [nb][n][3]; igt [nb][16]
 * = exp(x[b]) and gt [nb][16] = igt^-1 (train/train_reg_v0.py:268-271), both optional. */
int hreg_perturb_clouds(const float *pts, const float *x, int nb, int n, float *out, float *igt,
                        float *gt, void *stream);
/* PointCloudFilter.remove_points_by_range (dataset/dataset_utils.py:113-127) for nb
 * clouds [nb][n][3] (+ intensity [nb][n], optional): the points with ||p|| < max_range,
 * in order, packed at the front of out[b] / out_intensity[b]; counts [nb] int32. */
int hreg_range_filter(const float *pts, const float *intensity, int nb, int n, float max_range,
                      float *out, float *out_intensity, int32_t *counts, void *stream);

/* ---- Model_V2 training losses (mi_loss.hip) ---- */
#define HREG_REDUCE_NONE 0
#define HREG_REDUCE_MEAN 1
#define HREG_REDUCE_SUM 2
/* ChamferDistanceLoss(scale, reduction) (losses/chamfer_loss.py:20-36) over the
 * chamfer_distance extension's nearest squared distances: p0 [nb][n][3], p1 [nb][m][3]
 * (divided by scale first) -> d01 [nb][n], d10 [nb][m] (+ argmin idx, optional),
 * per_pair [nb] = (mean sqrt d01 + mean sqrt d10) / 2 (optional), out [1] = mean / sum
 * of per_pair (reduction MEAN / SUM; NONE writes per_pair only). */
int hreg_chamfer(const float *p0, const float *p1, int nb, int n, int m, float scale, int reduction,
                 float *d01, float *d10, int32_t *idx01, int32_t *idx10, float *per_pair, float *out,
                 void *stream);
/* DeepMILoss Jensen-Shannon terms (losses/mi_loss_v2.py:56-64): out [3] = (0.5 (Em - Ej),
 * Ej, Em) from the discriminator outputs t_joint, t_marg [n]; g_joint / g_marg
 * (optional) = d out[0] / d t. */
int hreg_js_loss(const float *t_joint, const float *t_marg, int n, float *out, float *g_joint,
                 float *g_marg, void *stream);
/* t[r] = act(h[r] . w + b) (the 1-output conv3 / l0 of the discriminators,
 * mi_loss_v2.py:13,33); b optional, relu 0/1.  _bwd: dh = g' w^T, dw = g'^T h,
 * db = sum g' with g' = g [t > 0] when relu (each output optional). */
int hreg_rowdot(const float *h, int R, int C, const float *w, const float *b, int relu, float *t,
                void *stream);
int hreg_rowdot_bwd(const float *g, const float *t, int relu, const float *h, int R, int C,
                    const float *w, float *dh, float *dw, float *db, void *stream);
/* dx = dy [y > 0] */
int hreg_relu_bwd(const float *dy, const float *y, size_t n, float *dx, void *stream);

/* norms[r] = sqrt(sum_c x[r][c]^2), x [R][ldx] */
int hreg_row_norms(const float *x, int R, int C, int ldx, float *norms, void *stream);

/* S [nb][N1][N2]; kidx [nb][N1][k] int32 (local dst index) ->
 * sims[(b*N1+i)*k+j][2] = (S[i][n]/(rowmax_i + 1e-6), S[i][n]/(colmax_n + 1e-6)), n = kidx;
 * maxes [nb][N1+N2] receives (rowmax, colmax) (caller-allocated scratch/output). */
int hreg_sim_gather(const float *S, int nb, int N1, int N2, const int32_t *kidx, int k,
                    float *maxes, float *sims, int ld_sims, void *stream);

/* Small per-(query,neighbour) feature rows for CoarseReg/FineReg (16 floats):
 * [p-q (3), |p-q| (1), q (3), p (3), w_src (1), w_dst[n] (1), sims (ns: 0 or 4), pad].
 * q = src_xyz [nb][M][3], p = dst_xyz [nb][N][3] gathered by kidx (local), w from
 * src_w [nb][M], dst_w [nb][N]; sims [rows][2] x 2 (sim_a, sim_b) optional. */
int hreg_pair_feats(const float *src_xyz, const float *dst_xyz, const float *src_w,
                    const float *dst_w, const int32_t *kidx, int nb, int M, int N, int k,
                    const float *sims_a, const float *sims_b, float *feats, int ldf,
                    float *knn_xyz, int32_t *gidx, void *stream);

/* WeightedSVDHead (layers.py:469-504) for nb pairs of n points:
 * src, corres [nb][n][3], w [nb][n] -> R_ [nb][9], t_ [nb][3]; if prev_R/prev_t
 * are given, also R = R_ prev_R, t = R_ prev_t + t_ (models.py:100-127) into R/t.
 * A non-finite covariance anywhere in the batch gives R_ = I, t_ = 0 for the
 * whole batch (the reference's try/except, layers.py:485-493). */
int hreg_weighted_svd(const float *src, const float *corres, const float *w, int nb, int n,
                      const float *prev_R, const float *prev_t, float *R_, float *t_, float *R,
                      float *t, void *stream);
/* hreg_weighted_svd over nb pairs that are nb / group reference batches of `group` pairs each
 * (several batches merged into one launch set): the identity fallback of layers.py:485-493
 * applies per batch.  group = nb is hreg_weighted_svd. */
int hreg_weighted_svd_grouped(const float *src, const float *corres, const float *w, int nb, int group,
                              int n, const float *prev_R, const float *prev_t, float *R_, float *t_,
                              float *R, float *t, void *stream);
/* hreg_weighted_svd_grouped + hreg_transform_points of tr_xyz [nb][tr_n][3] by each pair's final
 * R, t (R / t when given, else R_ / t_) into tr_out, in the batch step's launch: the same bits as
 * the two calls (HRegNet.forward's src_xyz_{2,1} moves, models.py:100-127). */
int hreg_weighted_svd_tr(const float *src, const float *corres, const float *w, int nb, int group, int n,
                         const float *prev_R, const float *prev_t, float *R_, float *t_, float *R,
                         float *t, const float *tr_xyz, int tr_n, float *tr_out, void *stream);

/* out[b][i] = R[b] xyz[b][i] + t[b], xyz/out [nb][n][3] */
int hreg_transform_points(const float *xyz, const float *R, const float *t, int nb, int n,
                          float *out, void *stream);

/* transformation_loss (losses/losses.py:97-164) for one level of nb pairs, all device
 * pointers: pred_R/gt_R [nb][3][3], pred_t/gt_t [nb][3].  Outputs (each may be NULL):
 * scalars[3] = {alpha*loss_R + loss_t, loss_R, loss_t}; R_err[3] = batch-mean |Euler XYZ
 * angles| of pred_R^T gt_R in degrees; T_err[3] = batch-mean |pred_t - gt_t|;
 * geodesic[nb] (RRE, degrees); eucl[nb] (RTE).  Deterministic (fixed-order reduction).
 * Forward only (no gradient). */
int hreg_transformation_loss(const float *pred_R, const float *pred_t, const float *gt_R,
                             const float *gt_t, int nb, float alpha, float *scalars, float *R_err,
                             float *T_err, float *geodesic, float *eucl, void *stream);

/* CalibEval.add_batch (metrics/calibeval.py:72-113) for one layer's batch of nb pairs, all
 * device pointers: pred_tf/gt_tf [nb][4][4] row-major.  per_pair [nb][12] = {Euler XYZ
 * angles (deg) of E = pred_tf . gt_tf, E[:3,3], Euler XYZ (deg) of pred_tf, pred_tf[:3,3]};
 * batch_geo[2] = {mean geodesic angle of E (deg), mean ||E[:3,3]||} (calibeval.py:197-214). */
int hreg_calib_metrics(const float *pred_tf, const float *gt_tf, int nb, float *per_pair,
                       float *batch_geo, void *stream);

/* ---------------- point-to-point ICP refinement (csrc/icp.hip) ----------------
 * open3d registration_icp(source, target, max_correspondence_distance, init,
 * TransformationEstimationPointToPoint(), ICPConvergenceCriteria(relative_fitness,
 * relative_rmse, max_iteration)) as test/test_v4.py:140-158 calls it after the network,
 * for nb independent pairs.  source [nb][n_src][3], target [nb][n_dst][3] fp32, n <= 65536;
 * T0 [nb][4][4] fp32 row-major (null: identity).  ws: hreg_icp_ws_bytes, 256-byte aligned,
 * owned by the caller for the whole run.  hreg_icp_iterate enqueues `iters` iterations (pairs
 * already converged skip them); the caller polls hreg_icp_result's done flags between calls.
 * Results: T [nb][4][4], fitness = matches / n_src, inlier_rmse, iterations = updates applied. */
size_t hreg_icp_ws_bytes(int nb, int n_src, int n_dst);
int hreg_icp_init(const float *src, const float *dst, int nb, int n_src, int n_dst, const float *T0,
                  void *ws, void *stream);
int hreg_icp_iterate(const float *dst, int nb, int n_src, int n_dst, float max_corr_dist,
                     double rel_fitness, double rel_rmse, int max_iteration, int iters, void *ws,
                     void *stream);
int hreg_icp_result(const void *ws, int nb, int n_src, int n_dst, float *T_out, float *fitness,
                    float *inlier_rmse, int32_t *iterations, int32_t *done, void *stream);

/* ---------------- training-step building blocks (csrc/train.hip) ----------------
 * Train-mode BatchNorm after a 1x1 conv (layers.py:115-130 etc. in .train(); the
 * reference's train loop train/train_reg_v0.py:241-296), weight gradients and Adam
 * (train_reg_v0.py:246).  Row-major [R][C] tensors; every reduction over rows is
 * deterministic (split partials in ws, summed in a fixed order). */
size_t hreg_col_reduce_ws_bytes(int R, int C);
/* per channel of y [R][C]: mean, invstd = 1/sqrt(var_biased + eps), var_unbiased (may be NULL) */
int hreg_bn_stats(const float *y, int R, int C, float eps, void *ws, float *mean, float *invstd,
                  float *var_unbiased, void *stream);
/* Tall-skinny conv GEMM of the training step (csrc/ts_gemm.hip): out[r][n] = act(scale[n] *
 * sum_k A[r][k] W'[n][k] + shift[n]) with W' = W [N][K] (w_trans 0) or the transpose of
 * W [K][N] (w_trans 1); scale / shift may be NULL (1 / 0), act = ReLU if relu.  The same
 * fp32 sums as hreg_gemm (same k-order).  K, N, lda, ldo multiples of 4, 16-byte aligned
 * pointers; hreg_ts_gemm_supported(R, K, N, 0) != 0 when W' fits the kernel's LDS
 * (stats 1: with hreg_ts_gemm_bn's statistics buffers as well). */
int hreg_ts_gemm_supported(int R, int K, int N, int stats);
int hreg_ts_gemm(const float *A, int lda, int R, int K, const float *W, int w_trans, int N,
                 const float *scale, const float *shift, int relu, float *out, int ldo, void *stream);
/* hreg_ts_gemm (no scale / shift / activation) with its output [R][N] split by columns: [0, n1)
 * -> out0 (row stride ld0), [n1, n2) -> out1 (ld1), [n2, N) -> out2 (ld2; NULL when n2 = N); n1
 * and n2 multiples of 32 (n2 may equal N), 16-byte aligned outputs.  The same values as
 * hreg_ts_gemm's (r6: the descriptor tail's input gradient, layers.py:204-206, written straight
 * into its x2-block / x1 / att_map gradients). */
int hreg_ts_gemm_split_out(const float *A, int lda, int R, int K, const float *W, int w_trans, int N,
                           float *out0, int ld0, int n1, float *out1, int ld1, int n2, float *out2, int ld2,
                           void *stream);
/* hreg_ts_gemm (no scale / activation) with the output's train-mode BatchNorm statistics
 * computed in its epilogue (fp64 sums, fixed order; the hreg_bn_stats pass over out it
 * replaces): mean, invstd, var_unbiased as hreg_bn_stats (var_unbiased may be NULL without
 * running stats), and running_mean / running_var (both or neither) updated with momentum as
 * hreg_bn_running_update.  ws = hreg_ts_gemm_bn_ws_bytes(R, K, N) bytes. */
size_t hreg_ts_gemm_bn_ws_bytes(int R, int K, int N);
int hreg_ts_gemm_bn(const float *A, int lda, int R, int K, const float *W, int w_trans, int N,
                    const float *shift, float *out, int ldo, float eps, float momentum, void *ws,
                    float *mean, float *invstd, float *var_unbiased, float *running_mean,
                    float *running_var, void *stream);
/* hreg_ts_gemm_bn over the descriptor tail's rows without the concatenation (layers.py:204-206):
 * A = cat([x2 repeated over the k rows of each group, x1, att]), x2 [R/k][C1], x1 [R][C1],
 * att [R][Ca], C1 and Ca multiples of 16, W [N][2 C1 + Ca]; the same sums as hreg_ts_gemm_bn on
 * the materialised matrix.  ws = hreg_ts_gemm_bn_ws_bytes(R, 2 C1 + Ca, N) bytes. */
int hreg_ts_gemm_bn_tail(const float *x2, int k, const float *x1, int C1, const float *att, int Ca, int R,
                         const float *W, int N, const float *shift, float *out, int ldo, float eps,
                         float momentum, void *ws, float *mean, float *invstd, float *var_unbiased,
                         float *running_mean, float *running_var, void *stream);
/* hreg_ts_gemm_bn (w_trans 0) with A = the previous layer's pre-BatchNorm output [R][K]: every A
 * value enters as ReLU(pre_gamma * (A - pre_mean) * pre_invstd + pre_beta) (pre_relu must be 1,
 * else HREG_ERR_UNSUPPORTED; hreg_bn_apply's arithmetic, per column k), so out and the statistics are those of
 * hreg_bn_apply followed by hreg_ts_gemm_bn, without the activation materialised (the
 * train-mode Conv+BN+ReLU chains of layers.py:115-130, 183-198; r6).  hreg_ts_gemm_pre_supported
 * != 0 when the kernel takes the shape (K <= 512, up to 4 output tiles of 32 per workgroup).
 * ws = hreg_ts_gemm_bn_ws_bytes(R, K, N) bytes. */
int hreg_ts_gemm_pre_supported(int R, int K, int N);
int hreg_ts_gemm_bn_pre(const float *A, int lda, int R, int K, const float *W, int N, const float *shift,
                        float *out, int ldo, float eps, float momentum, void *ws, float *mean, float *invstd,
                        float *var_unbiased, float *running_mean, float *running_var, const float *pre_mean,
                        const float *pre_invstd, const float *pre_gamma, const float *pre_beta, int pre_relu,
                        void *stream);
/* out = act(gamma * (y - mean) * invstd + beta), act = ReLU if relu (out may alias y) */
int hreg_bn_apply(const float *y, int R, int C, const float *mean, const float *invstd,
                  const float *gamma, const float *beta, int relu, float *out, void *stream);
/* backward of hreg_bn_apply given dout: dgamma, dbeta [C], dy [R][C] (the
 * batch-statistics BN input gradient).  ReLU mask: out > 0 when out is given, else
 * recomputed bit-identically from y, gamma and beta (one fewer [R][C] stream).
 * accumulate != 0: dgamma / dbeta are added to (a parameter's .grad over its uses). */
int hreg_bn_backward(const float *dout, const float *out, const float *y, int R, int C,
                     const float *mean, const float *invstd, const float *gamma, const float *beta,
                     int relu, void *ws, float *dy, float *dgamma, float *dbeta, int accumulate,
                     void *stream);
/* running = (1 - momentum) * running + momentum * batch (nn.BatchNorm's momentum 0.1) */
int hreg_bn_running_update(const float *mean, const float *var_unbiased, int C, float momentum,
                           float *running_mean, float *running_var, void *stream);
/* out[c] = sum_r x[r][c] (conv bias gradients); accumulate != 0: out[c] += the sum */
int hreg_col_sum(const float *x, int R, int C, void *ws, float *out, int accumulate, void *stream);
/* out[n][k] = beta * out[n][k] + sum_r A[r][n] * B[r][k] (dW = dY^T X), fp32 MFMA,
 * ws = hreg_gemm_tn_ws_bytes(R, N, K) bytes */
size_t hreg_gemm_tn_ws_bytes(int R, int N, int K);
int hreg_gemm_tn(const float *A, int lda, const float *B, int ldb, int R, int N, int K, float beta,
                 void *ws, float *out, void *stream);
/* hreg_gemm_tn with B = cat([x2 repeated over the k rows of each group, x1, att]) read in place
 * (the descriptor tail's weight gradient): x2 [R/k][C1], x1 [R][C1], att [R][Ca], C1 and Ca
 * multiples of 64, out [N][2 C1 + Ca]; the same sums as hreg_gemm_tn on the materialised matrix.
 * ws = hreg_gemm_tn_ws_bytes(R, N, 2 C1 + Ca) bytes. */
int hreg_gemm_tn_tail(const float *A, int lda, const float *x2, int k, const float *x1, int C1,
                      const float *att, int Ca, int R, int N, float beta, void *ws, float *out, void *stream);
/* hreg_gemm_tn with B = the previous layer's pre-BatchNorm output [R][K]: B enters as
 * ReLU(pre_gamma * (B - pre_mean) * pre_invstd + pre_beta) per column (pre_relu must be 1;
 * hreg_bn_apply's arithmetic);
 * the same splits and sums as hreg_gemm_tn over the materialised activation (the weight gradient
 * of a Conv whose input is the previous Conv+BN+ReLU's output; r6).  lda, ldb multiples of 4,
 * 16-byte aligned A and B (else HREG_ERR_UNSUPPORTED).  ws = hreg_gemm_tn_ws_bytes(R, N, K). */
int hreg_gemm_tn_pre(const float *A, int lda, const float *B, int ldb, int R, int N, int K, float beta, void *ws,
                     float *out, const float *pre_mean, const float *pre_invstd, const float *pre_gamma,
                     const float *pre_beta, int pre_relu, void *stream);
/* out [C][R] = in [R][C]^T */
int hreg_transpose(const float *in, int R, int C, float *out, void *stream);
/* y[i] += x[i] (fp32, one rounding) over n floats: the second gradient bucket of the
 * two-stream training step added into the first */
int hreg_add_into(const float *x, float *y, size_t n, void *stream);
/* torch.optim.Adam step t (>= 1) over n floats, weight decay 0, amsgrad off */
int hreg_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, size_t n,
                   float lr, float beta1, float beta2, float eps, int step, void *stream);
/* the same update with scalars[2] = {lr / (1 - beta1^t), sqrt(1 - beta2^t)} (as hreg_adam_step
 * computes them) read from device memory when the kernel runs: a captured graph's replays */
int hreg_adam_step_dev(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, size_t n,
                       float lr, float beta1, float beta2, float eps, const float *scalars, void *stream);

/* ---------------- training graph ops (csrc/train_ops.hip) ----------------
 * Forward/backward of every non-GEMM op of the HRegNet training step
 * (train/train_reg_v0.py:241-296 through models/HRegNet/layers.py and models.py in
 * .train()), wired into autograd by pcd_reg_hregnet_amd/train_graph.py.  Rows are
 * point-major [rows][ld]; a group of k neighbours is k consecutive rows.  Backward
 * sums run in a fixed order (no float atomics): same bits every run. */
/* count (<= 16) device-to-device copies src[i] -> dst[i] of nbytes[i] bytes (multiples of 4; host
 * arrays, read at the call) in one launch */
int hreg_copy_many(int count, const void *const *src, void *const *dst, const size_t *nbytes, void *stream);
/* dst[r][c] (+)= src[r / row_div][c]  (torch.cat / repeat over k; accumulate != 0 adds) */
int hreg_copy_rows(const float *src, int lds, int row_div, int R, int C, float *dst, int ldd,
                   int accumulate, void *stream);
/* out[g][c] (+)= sum_{j<k} x[g*k+j][c]  (backward of a repeat over k; attentive sums) */
int hreg_group_sum(const float *x, int ldx, int G, int k, int C, float *out, int ldo,
                   int accumulate, void *stream);
/* out[m] = x[idx[m]]  (knn_gather layers.py:25,279,288,317,323,434,437; gather_operation
 * models/utils.py:60-78 with global row indices) */
int hreg_gather_rows(const float *x, int ldx, const int32_t *idx, int M, int C, float *out,
                     int ldo, void *stream);
/* out[b*m + j] = idx[b*m + j] + b*n (per-cloud indices -> global rows of the [nb*n] stack) */
int hreg_index_offset(const int32_t *idx, int nb, int m, int n, int32_t *out, void *stream);
/* inverse of an index (the scatter of a gather's backward): ws of hreg_csr_ws_bytes(M, n)
 * bytes gets, per source row s < n, the ascending list of m with idx[m] == s */
size_t hreg_csr_ws_bytes(int M, int n);
int hreg_csr_build(const int32_t *idx, int M, int n, void *ws, void *stream);
/* dx[s] (+)= sum_{m: idx[m] = s} dy[m] in ascending m (replaces the atomicAdd of
 * gather_points_grad_kernel, furthest_point_sampling_gpu.cu:41-73) */
int hreg_scatter_rows(const float *dy, int ldy, const void *ws, int M, int n, int C, float *dx,
                      int ldx, int accumulate, void *stream);
/* out[r] = [knn_xyz[r] - q[r/k], |knn_xyz[r] - q[r/k]|]  (layers.py:21-23, 284-285) */
int hreg_geom_rows(const float *q, const float *knn_xyz, int G, int k, float *out, int ldo,
                   void *stream);
/* backward: dq [G][3] = -sum_k drela, dknn [G*k][3] = drela (+ dknn_extra); either may be NULL */
int hreg_geom_rows_bwd(const float *geom, int ldg, const float *dgeom, int lddg,
                       const float *dknn_extra, int G, int k, float *dq, float *dknn,
                       void *stream);
/* a = softmax_k(max_c logits) (amax = argmax channel), kp = sum_k a knn_xyz,
 * vmap = vals * a, vsum = sum_k vmap  (layers.py:151-159, 340-343, 384-388, 447-450);
 * k <= 64, every output optional */
int hreg_attention_fwd(const float *logits, int ldl, int C, const float *vals, int ldv, int Cv,
                       const float *knn_xyz, int G, int k, float *a, int32_t *amax, float *kp,
                       float *vmap, int ldm, float *vsum, int lds, void *stream);
/* backward of hreg_attention_fwd: dlogits (written, every element), dvals, dknn;
 * same != 0: vals is logits, dlogits then holds both gradients */
int hreg_attention_bwd(const float *logits, int ldl, int C, const float *vals, int ldv, int Cv,
                       const float *knn_xyz, int G, int k, const float *a, const int32_t *amax,
                       const float *dkp, const float *dvmap, int lddm, const float *dvsum,
                       int ldds, int same, float *dlogits, int lddl, float *dvals, int lddv,
                       float *dknn, void *stream);
/* hreg_attention_fwd / _bwd with logits = vals = ReLU(gamma * (y - mean) * invstd + beta) of a
 * pre-BatchNorm y [G*k][C] (per channel; hreg_bn_apply's values, never materialised: the
 * detector's last Conv+BN+ReLU, layers.py:150-159; r6); the backward writes dact = the gradient
 * with respect to that activation (the BN backward follows) and dknn */
int hreg_attention_fwd_pre(const float *y, int ldy, int C, const float *mean, const float *invstd,
                           const float *gamma, const float *beta, const float *knn_xyz, int G, int k, float *a,
                           int32_t *amax, float *kp, float *vmap, int ldm, float *vsum, int lds, void *stream);
int hreg_attention_bwd_pre(const float *y, int ldy, int C, const float *mean, const float *invstd,
                           const float *gamma, const float *beta, const float *knn_xyz, int G, int k,
                           const float *a, const int32_t *amax, const float *dkp, const float *dvmap, int lddm,
                           const float *dvsum, int ldds, float *dact, int ldda, float *dknn, void *stream);
/* out[g][c] = max_j x[g*k+j][c], arg = first maximising j  (layers.py:202, 208) */
int hreg_group_max_arg(const float *x, int ldx, int G, int k, int C, float *out, int ldo,
                       int32_t *arg, void *stream);
/* hreg_group_max_arg over ReLU(gamma * (x - mean) * invstd + beta) (per column c; x the
 * pre-BatchNorm output, hreg_bn_apply's values): the maxima and arguments over the activation
 * without materialising it (r6, the descriptor's last k-max, train.py _BNActGroupMax) */
int hreg_group_max_arg_pre(const float *x, int ldx, int G, int k, int C, float *out, int ldo, int32_t *arg,
                           const float *mean, const float *invstd, const float *gamma, const float *beta,
                           void *stream);
int hreg_group_max_bwd(const float *dout, int ldd, const int32_t *arg, int G, int k, int C,
                       float *dx, int ldx, int accumulate, void *stream);
/* backward of hreg_head_out's activation: dz [G] = dy * act'(x.w3 + b3), dx = dz w3^T */
int hreg_head_out_bwd(const float *x, int ldx, int C, const float *w3, const float *b3,
                      const float *dy, int mode, int G, float *dz, float *dx, int lddx,
                      void *stream);
/* row maxima (over N2) / column maxima (over N1) of S [nb][N1][N2] with first argmax */
int hreg_sim_stats(const float *S, int nb, int N1, int N2, float *rmax, int32_t *rarg,
                   float *cmax, int32_t *carg, void *stream);
/* out[r] = [S[i][n] / (rmax_i + 1e-6), S[i][n] / (cmax_n + 1e-6)], n = kidx[r], r = (b,i,j)
 * (src_dst_cos, dst_src_cos: layers.py:290-313, 345-362) */
int hreg_sim_feats(const float *S, int nb, int N1, int N2, const int32_t *kidx, int k,
                   const float *rmax, const float *cmax, float *out, int ldo, void *stream);
/* backward through the gathers, the maxima and calc_cosine_similarity (layers.py:29-41)
 * to the descriptors a [nb][N1][C], b [nb][N2][C]; ws = hreg_sim_feats_bwd_ws_bytes */
size_t hreg_sim_feats_bwd_ws_bytes(int nb, int N1, int N2);
int hreg_sim_feats_bwd(const float *S, const float *a, const float *b, const float *na,
                       const float *nb_, int nb, int N1, int N2, int C, const int32_t *kidx,
                       int k, const float *rmax, const int32_t *rarg, const float *cmax,
                       const int32_t *carg, const float *dout, int ldd, void *ws, float *da,
                       float *db, void *stream);
/* WeightedSVDHead backward (layers.py:469-504; torch.svd + torch.det backward), fp64:
 * dR [nb][3][3], dt [nb][3] -> dsrc, dcorres [nb][n][3], dw [nb][n] */
int hreg_weighted_svd_bwd(const float *src, const float *corres, const float *w, int nb, int n,
                          const float *dR, const float *dt, float *dsrc, float *dcorres,
                          float *dw, void *stream);
/* backward of hreg_transform_points: dxyz (may be NULL), dR, dt (sums over the points) */
int hreg_transform_points_bwd(const float *xyz, const float *R, int nb, int n, const float *dy,
                              float *dxyz, float *dR, float *dt, void *stream);
/* (Ro, to) = (Ra Rb, Ra tb + ta): T = T_a @ T_b (models.py:100-110, 120-127) and backward */
int hreg_compose_se3(int nb, const float *Ra, const float *ta, const float *Rb, const float *tb,
                     float *Ro, float *to, void *stream);
int hreg_compose_se3_bwd(int nb, const float *Ra, const float *Rb, const float *tb,
                         const float *dRo, const float *dto, float *dRa, float *dta, float *dRb,
                         float *dtb, void *stream);
/* gradient of scale * dloss[0] * transformation_loss(...)[0] (losses.py:117-160) w.r.t.
 * pred R, t (dloss: device scalar, the upstream gradient; NULL = 1) */
int hreg_transformation_loss_bwd(const float *pred_R, const float *pred_t, const float *gt_R,
                                 const float *gt_t, int nb, float alpha, float scale,
                                 const float *dloss, float *dR, float *dt, void *stream);

/* Spatial index for exact culled kNN grouping (n <= 65536 points per cloud):
 * hreg_spatial_index sorts each cloud of p [nb][n][3] by Morton code (n <= 16384: an 18-bit
 * prefix, ties by index; larger clouds: the 12-bit cell) and records
 * the bounding box of every 64 sorted points into ws (16-byte aligned,
 * hreg_spatial_index_bytes(nb, n) bytes); hreg_knn_group_indexed is
 * hreg_knn_group over that index -- bit-identical results, visiting only the
 * point blocks whose box lower bound does not exceed the running K-th distance. */
size_t hreg_spatial_index_bytes(int nb, int n);
int hreg_spatial_index(const float *p, int nb, int n, void *ws, void *stream);
int hreg_knn_group_indexed(const float *q, const float *p, const void *ws, int nb, int m, int n,
                           int k, int32_t *gidx, float *geom, float *knn_xyz, void *stream);

/* Fused level-1 grouping stage (KeypointDetector.convs/mlp + attention + DescExtractor convs
 * + k-max + mlp, layers.py:115-130 and 183-198, with C = 64, nsample = 64): one wavefront per
 * group, every 1x1-conv+BN+ReLU layer chained through the MFMA accumulators, fp32-accurate
 * products on the bf16 matrix cores (bf16x6 split, group_l1_6.hip); geom [G][64] float4 and
 * knn_xyz [G][64][3] from hreg_knn_group(_indexed) -> kp [G][3], att_feat [G][64] (attentive
 * feature), desc [G][64].  (The fp32-MFMA twins hreg_group_l1 / _l2 / _l3 / _split_l{2,3} are
 * test checkers in libhregnet_checkers.so, include/hregnet_amd_checkers.h.)  table =
 * hreg_group_l1_6_table_floats() floats (engine.l1_table6), 16-byte aligned. */
int hreg_group_l1_6_table_floats(void);
int hreg_group_l1_6(const float *table, const float *geom, const float *knn_xyz, int G, float *kp,
                    float *att_feat, float *desc, void *stream);
/* The same with the weight table streamed from global memory instead of resident in LDS
 * (4-wave workgroups, no 92 KB LDS claim): for clouds whose FPS runs on the multi-workgroup
 * cluster kernel alongside (engine.L1_LDS_MAX_N); bitwise-equal outputs. */
int hreg_group_l1_6g(const float *table, const float *geom, const float *knn_xyz, int G, float *kp,
                     float *att_feat, float *desc, void *stream);

/* Fused level-2 / level-3 grouping stages (C_in = 4 + 64 / 4 + 128, convs 68->64->64->128 /
 * 132->128->128->256, mlp 384->64->128 / 768->128->256, nsample = 32 / 16), fp32-accurate
 * products on the bf16 matrix cores (bf16x6 split, group_fused6.hip): geom [G][k] float4 and
 * knn_xyz [G][k][3] from hreg_knn_group; gidx [G*k] rows of feats (the previous level's
 * attentive features, 16-byte aligned) -> kp [G][3], att_feat [G][2C], desc [G][2C]; pre
 * (optional): [*][2 * C1] = [W_det_f | W_desc_f] feats, the feature blocks of the two first
 * layers precomputed once per feature row.  table =
 * hreg_group6_l{2,3}_table_floats() floats (engine.l2_table6: bf16 piece fragments of
 * the same blocks, then the f32 epilogues), 16-byte aligned. */
int hreg_group6_l2_table_floats(void);
int hreg_group6_l2(const float *table, const float *geom, const float *knn_xyz,
                   const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                   float *desc, const float *pre, void *stream);
/* The channel-split stages (hreg_group_split_l{2,3}) with fp32-accurate products on the
 * bf16 matrix cores (bf16x6, group_split6.hip): same arguments and outputs, table =
 * hreg_group_split6_l{2,3}_table_floats() floats (engine.split_table6), 16-byte aligned. */
int hreg_group_split6_l2_table_floats(void);
int hreg_group_split6_l2(const float *table, const float *geom, const float *knn_xyz,
                         const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                         float *desc, const float *pre, void *stream);
int hreg_group_split6_l3_table_floats(void);
/* hreg_group_split6_l3 with two 32-row tiles per wave (each streamed weight piece feeds both
 * tiles' MFMAs; the same outputs bit for bit); pre (the precomputed feature block) required */
int hreg_group_split6j_l3(const float *table, const float *geom, const float *knn_xyz,
                          const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                          float *desc, const float *pre, void *stream);
int hreg_group_split6_l3(const float *table, const float *geom, const float *knn_xyz,
                         const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                         float *desc, const float *pre, void *stream);
int hreg_group6_l3_table_floats(void);
int hreg_group6_l3(const float *table, const float *geom, const float *knn_xyz,
                   const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                   float *desc, const float *pre, void *stream);

/* Fused FineReg head (layers.py:433-451) for C = 64 (fine_corres_1) or 128
 * (fine_corres_2): small [G*8][16] from hreg_pair_feats (ldf 16), src_desc [G][C]
 * (keypoint i's own descriptor), dst_desc [*][C] gathered by gidx [G*8],
 * knn_xyz [G*8][3] -> corres [G][3] (attention-weighted neighbour xyz) and
 * att [G][N1] (attentive feature, N1 = 2C), convs_1 + attention in one kernel.
 * table = hreg_fine_head_table_floats(C) floats (engine.fine_head_table).
 * pre_src [G][N1] = W_f src_desc, pre_dst [*][N1] = W_kf dst_desc (optional, both or
 * neither): the first layer's descriptor blocks precomputed once per point, so the
 * kernel multiplies only the 16 small columns per row (src_desc / dst_desc unread). */
int hreg_fine_head_table_floats(int C);
int hreg_fine_head(const float *table, int C, const float *small, const float *src_desc,
                   const float *dst_desc, const int32_t *gidx, const float *knn_xyz, int G,
                   float *corres, float *att, const float *pre_src, const float *pre_dst,
                   void *stream);

/* Fused CoarseReg neighbour branch (layers.py:315-337), C = 256: rows
 * [desc[gidx] C | geom 4] (geom [G*8] float4 from hreg_knn_group) through convs_2
 * (260 -> 256 x 3) and the attention over the 8 rows, applied to the gathered
 * descriptors: out [G][C] = sum_j a_j desc[gidx_j].  table =
 * hreg_nbr_head_table_floats() floats (engine.nbr_head_table).  pre [*][256] = W_d desc
 * (optional): the descriptor block of convs_2[0] precomputed once per point. */
int hreg_nbr_head_table_floats(void);
int hreg_nbr_head(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                  int G, float *out, const float *pre, void *stream);

/* The two heads above with fp32-accurate products on the bf16 matrix cores (bf16x6,
 * group_head.hip), precomputed-block form only (pre_src / pre_dst / pre required):
 * same outputs.  table = hreg_head6_table_floats(N1) floats, N1 = 2C for FineReg and
 * 256 for the neighbour branch (engine.head_table6: bf16 piece fragments of the narrow
 * first block, conv 2 and conv 3, then the f32 epilogues), 16-byte aligned. */
/* The correspondence-head kernel of hreg_coarse_head6 at conv width N1 in {128, 256, 512}
 * (channel split over N1/64 waves, activations through LDS, coarse6.hip): FineReg convs_1 +
 * attention with the precomputed descriptor blocks (ud0 = pre_src per keypoint, ud1 =
 * pre_dst per destination point gathered by gidx) -- the arguments of hreg_fine_head6 in
 * coarse6's order; table = hreg_corr_head6_table_floats(N1) floats (engine.fine_head_table6 /
 * coarse_head_table6, the same layout); -1 for an unsupported N1. */
int hreg_corr_head6_table_floats(int N1);
int hreg_corr_head6(const float *table, int N1, const float *small, const float *ud0, const float *ud1,
                    const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                    void *stream);
/* CoarseReg convs_1 + attention in one launch (coarse6.hip, bf16x6 products;
 * layers.py:364-390): G keypoints x 8 rows; small [G*8][16] packed small columns
 * (hreg_pair_feats), ud0 [G][512] = W_desc desc_src (per keypoint), ud1 [*][512] = W_knn_desc
 * desc_dst gathered by gidx [G*8], knn_xyz [G*8][3] -> corres [G][3], att [G][512] (the
 * attentive feature).  table = hreg_coarse_head6_table_floats() floats
 * (engine.coarse_head_table6), 16-byte aligned. */
int hreg_coarse_head6_table_floats(void);
int hreg_coarse_head6(const float *table, const float *small, const float *ud0, const float *ud1,
                      const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                      void *stream);

int hreg_head6_table_floats(int N1);
int hreg_fine_head6(const float *table, int C, const float *small, const int32_t *gidx,
                    const float *knn_xyz, int G, float *corres, float *att, const float *pre_src,
                    const float *pre_dst, void *stream);
int hreg_nbr_head6(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                   int G, float *out, const float *pre, void *stream);
/* hreg_nbr_head6 on the channel-split correspondence kernel (coarse6.hip: four waves of
 * 64 channels, activations through LDS): same arguments, table and outputs. */
int hreg_nbr_head6s(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                    int G, float *out, const float *pre, void *stream);
/* hreg_corr_head6 / hreg_nbr_head6s with the 32-row tiles per workgroup chosen: row_tiles 0 =
 * the default (2 at N1 <= 256: every streamed weight piece feeds both tiles; 1 at 512),
 * 1 or 2 (2 only at N1 <= 256); the same outputs bit for bit. */
int hreg_corr_head6x(const float *table, int N1, const float *small, const float *ud0, const float *ud1,
                     const int32_t *gidx, const float *knn_xyz, int G, float *corres, float *att,
                     int row_tiles, void *stream);
int hreg_nbr_head6sx(const float *table, const float *desc, const int32_t *gidx, const float *geom,
                     int G, float *out, const float *pre, int row_tiles, void *stream);

/* Diagnostic: the register FPS kernel (weights optional) with per-iteration clock
 * stamps [b][m] (tools/op_bench.py stamps) -- same selection as the two FPS entries. */
int hreg_debug_fps_stamps(int b, int n, int m, const float *points, const float *weights,
                          int32_t *idx, uint64_t *stamps, void *stream);
/* Latency floor of the level-1 FPS geometry: the same 8-wave workgroup and per-iteration
 * exchange, 2 points per thread (n = 1024); points [b][1024][3], stamps[6] as above, or NULL for
 * the unstamped kernel (its launch time is the floor of an unstamped level-1 kernel). */
/* Diagnostic: the latency floor of the level-2 (T = 256) / level-3 (T = 64) WFPS geometry: T
 * threads, one weighted point each (n = T); stamps as hreg_debug_fps_stamps. */
int hreg_debug_wfps_floor(int b, int T, int m, const float *points, const float *weights,
                          int32_t *idx, uint64_t *stamps, void *stream);
int hreg_debug_fps_floor(int b, int m, const float *points, int32_t *idx, uint64_t *stamps,
                         void *stream);

/* Reads the device status word (HREG_STATUS_* bits raised by kernels since the last
 * clear) into *status; clear != 0 takes it atomically (read and reset in one step).
 * Synchronous: waits for all work on the device (every stream) first. */
int hreg_device_status(int *status, int clear);

/* Diagnostic: the multi-workgroup FPS kernel forced on any n with at most polls_max
 * exchange polls per iteration, participant `stall` never publishing (-1: none) --
 * the timeout path of hreg_furthest_point_sampling (tests/test_gpu_ops.py). */
int hreg_debug_fps_cluster(int b, int n, int m, const float *points, float *temp,
                           int32_t *idx, float *sampled_xyz, int stall, unsigned polls_max,
                           void *stream);

/* Diagnostic: hreg_gemm_tn with S row splits instead of its own choice (ws: S * N * K
 * floats) -- tools/tn_split_sweep.py. */
int hreg_debug_gemm_tn_s(const float *A, int lda, const float *B, int ldb, int R, int N, int K,
                         float beta, void *ws, float *out, void *stream, int S);

/* library build id (for the loaded-.so audit) */
const char *hreg_version(void);

#ifdef __cplusplus
}
#endif

#endif /* HREGNET_AMD_H */
