/* hregnet_amd_checkers.h -- TEST-ONLY fp32-MFMA twins of the fused level kernels.
 *
 * The product library (libhregnet_amd.so, include/hregnet_amd.h) runs the level stages on
 * the bf16 matrix cores with fp32-accurate split products (bf16x6).  These kernels compute
 * the same stages on v_mfma_f32_32x32x2_f32 and serve only as independent checkers in
 * tests/ (and the engine's debug switches B6_L1 / B6_L2 / B6_L3 = 0); they are built into
 * libhregnet_checkers.so (csrc/checkers/), which the product path never loads.
 */
#ifndef HREGNET_AMD_CHECKERS_H
#define HREGNET_AMD_CHECKERS_H

#include "hregnet_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fused level-1 grouping stage (KeypointDetector.convs/mlp + attention + DescExtractor
 * convs + k-max + mlp, layers.py:115-130 and 183-198, with C=64, nsample=32):
 * one wavefront per group of 32 neighbours, every 1x1-conv+BN+ReLU layer chained
 * through MFMA accumulators.  table = the folded, fragment-permuted weights
 * (hreg_group_l1_table_floats() floats, built by engine.l1_table);
 * geom [G][32] float4 and knn_xyz [G][32][3] from hreg_knn_group ->
 * kp [G][3], att_feat [G][64] (attentive feature), desc [G][64]. */
int hreg_group_l1_table_floats(void);
int hreg_group_l1(const float *table, const float *geom, const float *knn_xyz, int G,
                  float *kp, float *att_feat, float *desc, void *stream);

/* Fused level-2 grouping stage (same layers as hreg_group_l1 with C_in = 4 + 64,
 * convs 68->64->64->128, mlp 384->64->128, nsample = 32): one wavefront per group.
 * table = hreg_group_l2_table_floats() floats (engine.l2_table); geom [G][32] float4
 * and knn_xyz [G][32][3] from hreg_knn_group; gidx [G*32] rows of feats
 * [*][64] (the level-1 attentive features, 16-byte aligned) ->
 * kp [G][3], att_feat [G][128], desc [G][128].  pre (optional, levels 2 and 3, both
 * kernels): [*][2 * C1] = [W_det_f | W_desc_f] feats, the feature blocks of the two
 * first layers precomputed once per feature row (same gidx): then only the 4 geometry
 * columns of those layers run per grouped row. */
int hreg_group_l2_table_floats(void);
int hreg_group_l2(const float *table, const float *geom, const float *knn_xyz,
                  const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                  float *desc, const float *pre, void *stream);

/* Fused level-3 grouping stage: C_in = 4 + 128, convs 132->128->128->256,
 * mlp 768->128->256, nsample = 16 (two groups per 32-row tile, G even);
 * feats [*][128] (the level-2 attentive features) -> kp [G][3],
 * att_feat [G][256], desc [G][256]. */
int hreg_group_l3_table_floats(void);
int hreg_group_l3(const float *table, const float *geom, const float *knn_xyz,
                  const int32_t *gidx, const float *feats, int G, float *kp, float *att_feat,
                  float *desc, const float *pre, void *stream);

/* The level-2 / level-3 stages above on the channel-split kernel (group_split.hip):
 * same arguments and outputs, table = hreg_group_split_l{2,3}_table_floats() floats
 * (engine.split_table: the same blocks, fragments grouped 4 k-steps per lane); geom
 * must be 16-byte aligned. */
int hreg_group_split_l2_table_floats(void);
int hreg_group_split_l2(const float *table, const float *geom, const float *knn_xyz,
                        const int32_t *gidx, const float *feats, int G, float *kp,
                        float *att_feat, float *desc, const float *pre, void *stream);
int hreg_group_split_l3_table_floats(void);
int hreg_group_split_l3(const float *table, const float *geom, const float *knn_xyz,
                        const int32_t *gidx, const float *feats, int G, float *kp,
                        float *att_feat, float *desc, const float *pre, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HREGNET_AMD_CHECKERS_H */
