/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. CPU restatement of the per-frame tracking matchers
 * (Frame::isInFrustum, both ORBmatcher::SearchByProjection overloads used by Tracking) and
 * glibc logf (see track_oracle.c). Uses the orbt_* POD types of the C-ABI header (types
 * only; nothing of the product library is linked).
 */
#ifndef TRACK_ORACLE_H
#define TRACK_ORACLE_H
#include "../include/orbslam2_amd.h"
#ifdef __cplusplus
extern "C" {
#endif
float orc_logf(float x);
void orc_is_in_frustum(const orbt_frame *F, const orbt_mappoints *M, int i, float viewingCosLimit,
                       uint8_t *in_view, float *px, float *py, float *pxr, float *vcos, int *lvl);
int orc_search_local_points(const orbt_frame *F, const orbt_mappoints *M, float viewCosLimit, float th,
                            float nnratio, const uint8_t *kp_blocked, orbt_view *view, int32_t *owner);
int orc_search_by_projection_frame(const orbt_frame *cur, const orbt_frame *last, const int32_t *last_mp,
                                   const uint8_t *last_outlier, const orbt_mappoints *M, float th, int bMono,
                                   int checkOri, const uint8_t *kp_blocked, int32_t *owner);
int orc_search_by_projection_kf(const orbt_frame *cur, const orbt_frame *kf, const int32_t *kf_mp,
                                const orbt_mappoints *M, float th, int ORBdist, int checkOri,
                                const uint8_t *kp_blocked, int32_t *owner);
int orc_search_by_bow(const orbb_keyframe *kf, const orbb_keyframe *F, float nnratio, int checkOri, int32_t *matches);
void orc_sim3_unscale(const float Scw[16], float Tcw[12], float Ow[3]);
int orc_search_by_projection_sim3(const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M, int th,
                                  int32_t *matched);
void orc_fuse_sim3_candidates(const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M, float th,
                              int32_t *best_idx, int32_t *best_dist);
void orc_sim3_relative(float s12, const float R12[9], const float t12[3], float sR12[9], float sR21[9], float t21[3]);
int orc_search_by_sim3(const orbt_frame *kf1, const int32_t *mp1, const orbt_frame *kf2, const int32_t *mp2,
                       const orbt_mappoints *M, float s12, const float R12[9], const float t12[3], float th,
                       int32_t *matches12);
int orc_search_by_bow_kf(const orbb_keyframe *k1, const orbb_keyframe *k2, float nnratio, int checkOri,
                         int32_t *matches12);
int orc_search_for_triangulation(const orbb_keyframe *kf1, const orbb_keyframe *kf2, const float F12[9],
                                 const float Cw[3], const float T2w[12], int bOnlyStereo, int checkOri,
                                 int32_t *pairs);
void orc_fuse_candidates(const orbt_frame *kf, const orbt_mappoints *M, float th, int32_t *best_idx,
                         int32_t *best_dist);
#ifdef __cplusplus
}
#endif
#endif
