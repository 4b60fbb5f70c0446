/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.h). Never linked into the product.
 *
 * Single-threaded C restatement of the per-frame tracking matchers of ORB-SLAM2-noted:
 *   Frame::isInFrustum            src/Frame.cc:490-578
 *   MapPoint::PredictScale        src/MapPoint.cc:612-626 (Frame overload)
 *   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)
 *                                 src/ORBmatcher.cc:78-176 (+ RadiusByViewingCos :179-191)
 *   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
 *                                 src/ORBmatcher.cc:1741-1904
 *   Tracking::SearchLocalPoints   src/Tracking.cc:1745-1810 (the in-view selection)
 *
 * Float semantics pinned (SURVEY.md Appendix A + A.8 in DESIGN.md):
 *   - cv::Mat float products R*X + t (3x3 * 3x1 + 3x1): OpenCV's small-matrix gemm path,
 *     float products summed left to right in float, then the float add of t;
 *   - cv::norm(float 3-vector): double sum of squares, sqrt in double, stored as float;
 *   - Mat::dot(float 3-vectors): double products summed left to right;
 *   - log(float) resolves to std::log(float) = glibc logf (`using namespace std` from
 *     DBoW2/TemplatedVocabulary.h:36); restated here as glibc 2.35's table algorithm and
 *     pinned exhaustively by oracle/tools/check_logf.c (0 mismatches over every positive
 *     float);
 *   - `1.0 / z` with float z is a double division rounded to float (ORBmatcher.cc:1794);
 *   - round(float) = roundf (half away from zero), ceil(float) = ceilf.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"
#include "track_oracle.h"

/* ---- glibc 2.35 logf (sysdeps/ieee754/flt-32/e_logf.c, e_logf_data.c), restated ---- */
static const double LOGF_INVC[16] = {
    0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
    0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
    0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
    0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
static const double LOGF_LOGC[16] = {
    -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
    -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3,   -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4,
    -0x1.252f438e10c1ep-5, 0x0p+0,                0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
    0x1.526e57720db08p-3,  0x1.bc2860d22477p-3,   0x1.1058bc8a07ee1p-2,  0x1.4043057b6ee09p-2};
static const double LOGF_A[3] = {-0x1.00ea348b88334p-2, 0x1.5575b0be00b6ap-2, -0x1.ffffef20a4123p-2};
static const double LOGF_LN2 = 0x1.62e42fefa39efp-1;

float orc_logf(float x) {
    uint32_t ix;
    memcpy(&ix, &x, 4);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;
        float y = x * 0x1p23f;               /* subnormal: normalise */
        memcpy(&ix, &y, 4);
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    float zf;
    memcpy(&zf, &iz, 4);
    const double z = zf;
    const double r = z * LOGF_INVC[i] - 1;
    const double y0 = LOGF_LOGC[i] + (double)k * LOGF_LN2;
    const double r2 = r * r;
    double y = LOGF_A[1] * r + LOGF_A[2];
    y = LOGF_A[0] * r2 + y;
    y = y * r2 + (y0 + r);
    return (float)y;
}

/* R * X + t as cv::Mat CV_32F expressions evaluate it (pinned, see header) */
static void mat_rx_t(const float T[12], const float X[3], float o[3]) {
    for (int i = 0; i < 3; i++) {
        const float *R = T + 4 * i;
        float s = R[0] * X[0];
        s = s + R[1] * X[1];
        s = s + R[2] * X[2];
        o[i] = s + R[3];
    }
}

void orc_is_in_frustum(const orbt_frame *F, const orbt_mappoints *M, int i, float viewingCosLimit,
                       uint8_t *in_view, float *px, float *py, float *pxr, float *vcos, int *lvl) {
    *in_view = 0;
    const float *P = M->Xw + 3 * i;
    float Pc[3];
    mat_rx_t(F->Tcw, P, Pc);
    const float PcX = Pc[0], PcY = Pc[1], PcZ = Pc[2];
    if (PcZ < 0.0f) return;                                        /* Frame.cc:509 */
    const float invz = 1.0f / PcZ;
    const float u = F->fx * PcX * invz + F->cx;
    const float v = F->fy * PcY * invz + F->cy;
    if (u < F->min_x || u > F->max_x) return;
    if (v < F->min_y || v > F->max_y) return;
    const float maxDistance = 1.2f * M->max_dist[i];               /* MapPoint.cc:555-559 */
    const float minDistance = 0.8f * M->min_dist[i];
    const float PO[3] = {P[0] - F->Ow[0], P[1] - F->Ow[1], P[2] - F->Ow[2]};
    double ss = 0;
    for (int k = 0; k < 3; k++) { const double t = PO[k]; ss += t * t; }
    const float dist = (float)sqrt(ss);                           /* cv::norm */
    if (dist < minDistance || dist > maxDistance) return;
    const float *Pn = M->normal + 3 * i;
    double dot = 0;
    for (int k = 0; k < 3; k++) dot += (double)PO[k] * Pn[k];     /* Mat::dot */
    const float viewCos = (float)(dot / dist);
    if (viewCos < viewingCosLimit) return;
    /* MapPoint::PredictScale(dist, Frame*) */
    const float ratio = M->max_dist[i] / dist;
    int nScale = (int)ceilf(orc_logf(ratio) / F->log_scale_factor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= F->nlevels) nScale = F->nlevels - 1;
    *in_view = 1;
    *px = u;
    *pxr = u - F->mbf * invz;
    *py = v;
    *lvl = nScale;
    *vcos = viewCos;
}

static int frame_grid(const orbt_frame *F, orc_frame_grid *g) {
    return orc_grid_build(g, (const orc_kp *)F->keys_un, F->desc, F->n, F->min_x, F->max_x, F->min_y,
                          F->max_y);
}

int orc_search_local_points(const orbt_frame *F, const orbt_mappoints *M, float viewCosLimit, float th,
                            float nnratio, const uint8_t *kp_blocked, orbt_view *view, int32_t *owner) {
    const int TH_HIGH = 100;
    const int N = F->n;
    orc_frame_grid g;
    frame_grid(F, &g);
    uint8_t *blocked = (uint8_t *)calloc((size_t)N + 1, 1);
    if (kp_blocked) memcpy(blocked, kp_blocked, (size_t)N);
    int *cand = (int *)malloc(sizeof(int) * ((size_t)N + 1));
    for (int k = 0; k < N; k++) owner[k] = -1;
    const int bFactor = th != 1.0f;
    int nmatches = 0;
    for (int m = 0; m < M->n; m++) {
        uint8_t inv = 0;
        float px = 0, py = 0, pxr = 0, vc = 0;
        int lvl = 0;
        /* Tracking::SearchLocalPoints: points matched in this frame keep mbTrackInView
         * false, bad points are skipped, the rest go through isInFrustum(pMP, 0.5) */
        if (!(M->flags[m] & (ORBT_MP_BAD | ORBT_MP_IN_FRAME)))
            orc_is_in_frustum(F, M, m, viewCosLimit, &inv, &px, &py, &pxr, &vc, &lvl);
        if (view) {
            if (view->in_view) view->in_view[m] = inv;
            if (view->proj_x) view->proj_x[m] = inv ? px : 0;
            if (view->proj_y) view->proj_y[m] = inv ? py : 0;
            if (view->proj_xr) view->proj_xr[m] = inv ? pxr : 0;
            if (view->view_cos) view->view_cos[m] = inv ? vc : 0;
            if (view->level) view->level[m] = inv ? lvl : 0;
        }
        if (!inv) continue;
        if (M->flags[m] & ORBT_MP_BAD) continue;
        /* ORBmatcher::SearchByProjection(F, vpMapPoints, th), ORBmatcher.cc:78-176 */
        float r = (vc > 0.998) ? 2.5f : 4.0f;                      /* RadiusByViewingCos */
        if (bFactor) r *= th;
        const float rs = r * F->scale_factors[lvl];
        const int nc = orc_features_in_area(&g, px, py, rs, lvl - 1, lvl, cand, N + 1);
        if (nc == 0) continue;
        const uint8_t *dMP = M->desc + 32 * (size_t)m;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            if (blocked[idx]) continue;
            if (F->u_right[idx] > 0) {
                const float er = fabsf(pxr - F->u_right[idx]);
                if (er > rs) continue;
            }
            const int dist = orc_descriptor_distance(dMP, F->desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist;
                bestLevel2 = bestLevel; bestLevel = F->keys_un[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F->keys_un[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2) continue;
            owner[bestIdx] = m;
            blocked[bestIdx] = (M->flags[m] & ORBT_MP_HAS_OBS) ? 1 : 0;
            nmatches++;
        }
    }
    free(cand); free(blocked);
    orc_grid_free(&g);
    return nmatches;
}

static void three_maxima30(const int *counts, int *ind1, int *ind2, int *ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < 30; i++) {
        const int s = counts[i];
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; *ind3 = *ind2; *ind2 = *ind1; *ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; *ind3 = *ind2; *ind2 = i; }
        else if (s > max3) { max3 = s; *ind3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { *ind2 = -1; *ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { *ind3 = -1; }
}

int orc_search_by_projection_frame(const orbt_frame *cur, const orbt_frame *last, const int32_t *last_mp,
                                   const uint8_t *last_outlier, const orbt_mappoints *M, float th, int bMono,
                                   int checkOri, const uint8_t *kp_blocked, int32_t *owner) {
    const int TH_HIGH = 100, HISTO_LENGTH = 30;
    const int N = cur->n;
    orc_frame_grid g;
    frame_grid(cur, &g);
    uint8_t *blocked = (uint8_t *)calloc((size_t)N + 1, 1);
    if (kp_blocked) memcpy(blocked, kp_blocked, (size_t)N);
    int *cand = (int *)malloc(sizeof(int) * ((size_t)N + 1));
    int *hist_bin = (int *)malloc(sizeof(int) * ((size_t)last->n + 1));
    int *hist_idx = (int *)malloc(sizeof(int) * ((size_t)last->n + 1));
    int nhist = 0;
    for (int k = 0; k < N; k++) owner[k] = -1;
    const float factor = HISTO_LENGTH / 360.0f;
    /* twc = -Rcw^T tcw (small-matrix gemm with GEMM_1_T, alpha -1); tlc = Rlw twc + tlw */
    float twc[3];
    for (int i = 0; i < 3; i++) {
        float s = cur->Tcw[i] * cur->Tcw[3];
        s = s + cur->Tcw[4 + i] * cur->Tcw[7];
        s = s + cur->Tcw[8 + i] * cur->Tcw[11];
        twc[i] = -s;
    }
    float tlc[3];
    mat_rx_t(last->Tcw, twc, tlc);
    const int bForward = tlc[2] > cur->mb && !bMono;
    const int bBackward = -tlc[2] > cur->mb && !bMono;
    int nmatches = 0;
    for (int i = 0; i < last->n; i++) {
        const int m = last_mp[i];
        if (m < 0) continue;
        if (last_outlier && last_outlier[i]) continue;
        float x3Dc[3];
        mat_rx_t(cur->Tcw, M->Xw + 3 * (size_t)m, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0) continue;
        const float u = cur->fx * xc * invzc + cur->cx;
        const float v = cur->fy * yc * invzc + cur->cy;
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        const int nLastOctave = last->keys_un[i].octave;
        const float radius = th * cur->scale_factors[nLastOctave];
        int nc;
        if (bForward) nc = orc_features_in_area(&g, u, v, radius, nLastOctave, -1, cand, N + 1);
        else if (bBackward) nc = orc_features_in_area(&g, u, v, radius, 0, nLastOctave, cand, N + 1);
        else nc = orc_features_in_area(&g, u, v, radius, nLastOctave - 1, nLastOctave + 1, cand, N + 1);
        if (nc == 0) continue;
        const uint8_t *dMP = M->desc + 32 * (size_t)m;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (blocked[i2]) continue;
            if (cur->u_right[i2] > 0) {
                const float ur = u - cur->mbf * invzc;
                const float er = fabsf(ur - cur->u_right[i2]);
                if (er > radius) continue;
            }
            const int dist = orc_descriptor_distance(dMP, cur->desc + 32 * (size_t)i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= TH_HIGH) {
            owner[bestIdx2] = m;
            blocked[bestIdx2] = (M->flags[m] & ORBT_MP_HAS_OBS) ? 1 : 0;
            nmatches++;
            if (checkOri) {
                float rot = last->keys_un[i].angle - cur->keys_un[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                hist_bin[nhist] = bin;
                hist_idx[nhist] = bestIdx2;
                nhist++;
            }
        }
    }
    if (checkOri) {
        int counts[30] = {0};
        for (int k = 0; k < nhist; k++) counts[hist_bin[k]]++;
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima30(counts, &ind1, &ind2, &ind3);
        for (int k = 0; k < nhist; k++) {
            const int b = hist_bin[k];
            if (b == ind1 || b == ind2 || b == ind3) continue;
            owner[hist_idx[k]] = -2;                            /* mvpMapPoints[..] = NULL */
            nmatches--;
        }
    }
    free(cand); free(blocked); free(hist_bin); free(hist_idx);
    orc_grid_free(&g);
    return nmatches;
}

/* ORBmatcher::SearchByProjection(Frame &CurrentFrame, KeyFrame *pKF, const set<MapPoint*>
 * &sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1922-2066; Tracking::Relocalization). kf_mp[i] =
 * index into M of pKF->GetMapPointMatches()[i] (-1 = NULL); ORBT_MP_FOUND marks sAlreadyFound.
 * kp_blocked = CurrentFrame.mvpMapPoints[i2] != NULL on entry; every claim blocks the keypoint
 * for later points (:2007-2008). No depth-sign test (:1959-1968). */
int orc_search_by_projection_kf(const orbt_frame *cur, const orbt_frame *kf, const int32_t *kf_mp,
                                const orbt_mappoints *M, float th, int ORBdist, int checkOri,
                                const uint8_t *kp_blocked, int32_t *owner) {
    const int HISTO_LENGTH = 30;
    const int N = cur->n;
    orc_frame_grid g;
    frame_grid(cur, &g);
    uint8_t *blocked = (uint8_t *)calloc((size_t)N + 1, 1);
    if (kp_blocked) memcpy(blocked, kp_blocked, (size_t)N);
    int *cand = (int *)malloc(sizeof(int) * ((size_t)N + 1));
    int *hist_bin = (int *)malloc(sizeof(int) * ((size_t)kf->n + 1));
    int *hist_idx = (int *)malloc(sizeof(int) * ((size_t)kf->n + 1));
    int nhist = 0, nmatches = 0;
    for (int k = 0; k < N; k++) owner[k] = -1;
    const float factor = HISTO_LENGTH / 360.0f;
    for (int i = 0; i < kf->n; i++) {
        const int m = kf_mp[i];
        if (m < 0) continue;
        if (M->flags[m] & (ORBT_MP_BAD | ORBT_MP_FOUND)) continue;   /* isBad() || sAlreadyFound.count */
        const float *P = M->Xw + 3 * (size_t)m;
        float x3Dc[3];
        mat_rx_t(cur->Tcw, P, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        const float u = cur->fx * xc * invzc + cur->cx;
        const float v = cur->fy * yc * invzc + cur->cy;
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        const float PO[3] = {P[0] - cur->Ow[0], P[1] - cur->Ow[1], P[2] - cur->Ow[2]};
        double ss = 0;
        for (int k = 0; k < 3; k++) { const double t = PO[k]; ss += t * t; }
        const float dist3D = (float)sqrt(ss);                         /* cv::norm */
        const float maxDistance = 1.2f * M->max_dist[m], minDistance = 0.8f * M->min_dist[m];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float ratio = M->max_dist[m] / dist3D;                  /* PredictScale(dist3D, &F) */
        int nPredictedLevel = (int)ceilf(orc_logf(ratio) / cur->log_scale_factor);
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= cur->nlevels) nPredictedLevel = cur->nlevels - 1;
        const float radius = th * cur->scale_factors[nPredictedLevel];
        const int nc = orc_features_in_area(&g, u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1, cand, N + 1);
        if (nc == 0) continue;
        const uint8_t *dMP = M->desc + 32 * (size_t)m;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (blocked[i2]) continue;
            const int dist = orc_descriptor_distance(dMP, cur->desc + 32 * (size_t)i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= ORBdist && bestIdx2 >= 0) {
            owner[bestIdx2] = m;
            blocked[bestIdx2] = 1;
            nmatches++;
            if (checkOri) {
                float rot = kf->keys_un[i].angle - cur->keys_un[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                hist_bin[nhist] = bin;
                hist_idx[nhist] = bestIdx2;
                nhist++;
            }
        }
    }
    if (checkOri) {
        int counts[30] = {0};
        for (int k = 0; k < nhist; k++) counts[hist_bin[k]]++;
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima30(counts, &ind1, &ind2, &ind3);
        for (int k = 0; k < nhist; k++) {
            const int b = hist_bin[k];
            if (b == ind1 || b == ind2 || b == ind3) continue;
            owner[hist_idx[k]] = -2;
            nmatches--;
        }
    }
    free(cand); free(blocked); free(hist_bin); free(hist_idx);
    orc_grid_free(&g);
    return nmatches;
}

/* LoopClosing's SearchByProjection(KeyFrame* pKF, cv::Mat Scw, vpPoints, vpMatched, th)
 * (src/ORBmatcher.cc:431-560). The Sim3 pose is unscaled as cv::Mat evaluates it:
 * scw = (float)sqrt(row0 . row0) (Mat::dot in double), sRcw / scw and st / scw through
 * convertTo(alpha = 1.0 / scw) in float (cvtScale_<float, float, float>), Ow = -Rcw^T tcw (float
 * gemm). matched[kf->n] in/out = vpMatched as indices into M (-1 = NULL, <= -2 = a point outside
 * vpPoints). Returns nmatches. */
void orc_sim3_unscale(const float Scw[16], float Tcw[12], float Ow[3]) {
    double d = 0;
    for (int k = 0; k < 3; k++) d += (double)Scw[k] * Scw[k];
    const float scw = (float)sqrt(d);
    const float a = (float)(1.0 / (double)scw);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) Tcw[4 * r + c] = Scw[4 * r + c] * a + 0.0f;
    for (int i = 0; i < 3; i++) {
        float t = Tcw[i] * Tcw[3];
        t = t + Tcw[4 + i] * Tcw[7];
        t = t + Tcw[8 + i] * Tcw[11];
        Ow[i] = -t;
    }
}

int orc_search_by_projection_sim3(const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M, int th,
                                  int32_t *matched) {
    const int TH_LOW = 50;
    const int N = kf->n;
    orbt_frame K = *kf;
    orc_sim3_unscale(Scw, K.Tcw, K.Ow);
    orc_frame_grid g;
    frame_grid(&K, &g);
    uint8_t *found = (uint8_t *)calloc((size_t)M->n + 1, 1);   /* spAlreadyFound */
    for (int i = 0; i < N; i++)
        if (matched[i] >= 0 && matched[i] < M->n) found[matched[i]] = 1;
    int *cand = (int *)malloc(sizeof(int) * ((size_t)N + 1));
    int nmatches = 0;
    for (int m = 0; m < M->n; m++) {
        if ((M->flags[m] & ORBT_MP_BAD) || found[m]) continue;                 /* :463 */
        const float *P = M->Xw + 3 * (size_t)m;
        float p3Dc[3];
        mat_rx_t(K.Tcw, P, p3Dc);                                                /* :471 */
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = K.fx * x + K.cx, v = K.fy * y + K.cy;
        if (!(u >= K.min_x && u < K.max_x && v >= K.min_y && v < K.max_y)) continue;   /* KeyFrame::IsInImage */
        const float maxDistance = 1.2f * M->max_dist[m], minDistance = 0.8f * M->min_dist[m];
        const float PO[3] = {P[0] - K.Ow[0], P[1] - K.Ow[1], P[2] - K.Ow[2]};
        double ss = 0;
        for (int k = 0; k < 3; k++) { const double t = PO[k]; ss += t * t; }
        const float dist = (float)sqrt(ss);
        if (dist < minDistance || dist > maxDistance) continue;                 /* :499 */
        const float *Pn = M->normal + 3 * (size_t)m;
        double dot = 0;
        for (int k = 0; k < 3; k++) dot += (double)PO[k] * Pn[k];
        if (dot < 0.5 * (double)dist) continue;                                 /* :506 */
        const float ratio = M->max_dist[m] / dist;                               /* PredictScale(dist, pKF) */
        int nPredictedLevel = (int)ceilf(orc_logf(ratio) / K.log_scale_factor);
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= K.nlevels) nPredictedLevel = K.nlevels - 1;
        const float radius = th * K.scale_factors[nPredictedLevel];
        const int nc = orc_features_in_area(&g, u, v, radius, -1, -1, cand, N + 1);   /* KeyFrame version */
        if (nc == 0) continue;
        const uint8_t *dMP = M->desc + 32 * (size_t)m;
        int bestDist = 256, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            if (matched[idx] != -1) continue;                                   /* :531 vpMatched[idx] */
            const int kpLevel = K.keys_un[idx].octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int d = orc_descriptor_distance(dMP, K.desc + 32 * (size_t)idx);
            if (d < bestDist) { bestDist = d; bestIdx = idx; }
        }
        if (bestDist <= TH_LOW) {                                                /* :552-556 */
            matched[bestIdx] = m;
            nmatches++;
        }
    }
    free(cand); free(found);
    orc_grid_free(&g);
    return nmatches;
}

/* LoopClosing's Fuse(KeyFrame* pKF, cv::Mat Scw, vpPoints, th, vpReplacePoint) search half
 * (src/ORBmatcher.cc:1321-1437): per point the first minimum Hamming distance in the window
 * (bestDist starts at INT_MAX, :1414), levels [l - 1, l], no chi2 gate; invz = 1.0 / z in double
 * (:1369). flags ORBT_MP_IN_FRAME = in pKF->GetMapPoints() (spAlreadyFound, :1339). */
void orc_fuse_sim3_candidates(const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M, float th,
                              int32_t *best_idx, int32_t *best_dist) {
    const int N = kf->n;
    orbt_frame K = *kf;
    orc_sim3_unscale(Scw, K.Tcw, K.Ow);
    orc_frame_grid g;
    frame_grid(&K, &g);
    int *cand = (int *)malloc(sizeof(int) * ((size_t)N + 1));
    for (int m = 0; m < M->n; m++) {
        best_idx[m] = -1;
        best_dist[m] = INT_MAX;
        if (M->flags[m] & (ORBT_MP_BAD | ORBT_MP_IN_FRAME)) continue;          /* :1353 */
        const float *P = M->Xw + 3 * (size_t)m;
        float p3Dc[3];
        mat_rx_t(K.Tcw, P, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = (float)(1.0 / (double)p3Dc[2]);
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = K.fx * x + K.cx, v = K.fy * y + K.cy;
        if (!(u >= K.min_x && u < K.max_x && v >= K.min_y && v < K.max_y)) continue;
        const float maxDistance = 1.2f * M->max_dist[m], minDistance = 0.8f * M->min_dist[m];
        const float PO[3] = {P[0] - K.Ow[0], P[1] - K.Ow[1], P[2] - K.Ow[2]};
        double ss = 0;
        for (int k = 0; k < 3; k++) { const double t = PO[k]; ss += t * t; }
        const float dist3D = (float)sqrt(ss);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float *Pn = M->normal + 3 * (size_t)m;
        double dot = 0;
        for (int k = 0; k < 3; k++) dot += (double)PO[k] * Pn[k];
        if (dot < 0.5 * (double)dist3D) continue;
        int lvl = (int)ceilf(orc_logf(M->max_dist[m] / dist3D) / K.log_scale_factor);
        if (lvl < 0) lvl = 0;
        else if (lvl >= K.nlevels) lvl = K.nlevels - 1;
        const float radius = th * K.scale_factors[lvl];
        const int nc = orc_features_in_area(&g, u, v, radius, -1, -1, cand, N + 1);
        const uint8_t *dMP = M->desc + 32 * (size_t)m;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            const int kpLevel = K.keys_un[idx].octave;
            if (kpLevel < lvl - 1 || kpLevel > lvl) continue;
            const int d = orc_descriptor_distance(dMP, K.desc + 32 * (size_t)idx);
            if (d < bestDist) { bestDist = d; bestIdx = idx; }
        }
        best_idx[m] = bestIdx;
        best_dist[m] = bestDist;
    }
    free(cand);
    orc_grid_free(&g);
}

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (src/ORBmatcher.cc:1472-1723).
 * Both keyframes' GetMapPointMatches() as indices into M; matches12[kf1->n] in/out (-1 = NULL).
 * sR12 = s12 * R12, sR21 = (1.0 / s12) * R12.t() (MatExpr scale -> convertTo in float),
 * t21 = -sR21 * t12 (float gemm). pKF1's intrinsics project in both directions (:1476-1479). */
static int sim3_pass(const orbt_frame *src, const int32_t *mp_src, const uint8_t *already, const orbt_frame *dst,
                     const orbt_frame *k1, const float sR[9], const float st[3], const orbt_mappoints *M, float th,
                     orc_frame_grid *g, int *cand, int *vnMatch) {
    const int TH_HIGH = 100;
    float T[12];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) T[4 * r + c] = sR[3 * r + c];
        T[4 * r + 3] = st[r];
    }
    for (int i = 0; i < src->n; i++) {
        vnMatch[i] = -1;
        const int m = mp_src[i];
        if (m < 0 || already[i]) continue;                                     /* :1535 */
        if (M->flags[m] & ORBT_MP_BAD) continue;
        const float *P = M->Xw + 3 * (size_t)m;
        float pc1[3], pc2[3];
        mat_rx_t(src->Tcw, P, pc1);                                              /* :1544 */
        mat_rx_t(T, pc1, pc2);                                                   /* :1546 */
        if (pc2[2] < 0.0f) continue;
        const float invz = (float)(1.0 / (double)pc2[2]);
        const float x = pc2[0] * invz, y = pc2[1] * invz;
        const float u = k1->fx * x + k1->cx, v = k1->fy * y + k1->cy;
        if (!(u >= dst->min_x && u < dst->max_x && v >= dst->min_y && v < dst->max_y)) continue;
        const float maxDistance = 1.2f * M->max_dist[m], minDistance = 0.8f * M->min_dist[m];
        double ss = 0;
        for (int k = 0; k < 3; k++) { const double t = pc2[k]; ss += t * t; }
        const float dist3D = (float)sqrt(ss);                                    /* cv::norm(p3Dc2) */
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        int lvl = (int)ceilf(orc_logf(M->max_dist[m] / dist3D) / dst->log_scale_factor);
        if (lvl < 0) lvl = 0;
        else if (lvl >= dst->nlevels) lvl = dst->nlevels - 1;
        const float radius = th * dst->scale_factors[lvl];
        const int nc = orc_features_in_area(g, u, v, radius, -1, -1, cand, dst->n + 1);
        const uint8_t *dMP = M->desc + 32 * (size_t)m;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            const int o = dst->keys_un[idx].octave;
            if (o < lvl - 1 || o > lvl) continue;
            const int d = orc_descriptor_distance(dMP, dst->desc + 32 * (size_t)idx);
            if (d < bestDist) { bestDist = d; bestIdx = idx; }
        }
        if (bestDist <= TH_HIGH) vnMatch[i] = bestIdx;
    }
    return 0;
}

void orc_sim3_relative(float s12, const float R12[9], const float t12[3], float sR12[9], float sR21[9], float t21[3]) {
    for (int k = 0; k < 9; k++) sR12[k] = R12[k] * s12 + 0.0f;
    const float a = (float)(1.0 / (double)s12);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) sR21[3 * i + j] = R12[3 * j + i] * a + 0.0f;
    for (int i = 0; i < 3; i++) {
        float t = sR21[3 * i] * t12[0];
        t = t + sR21[3 * i + 1] * t12[1];
        t = t + sR21[3 * i + 2] * t12[2];
        t21[i] = -t;
    }
}

int orc_search_by_sim3(const orbt_frame *kf1, const int32_t *mp1, const orbt_frame *kf2, const int32_t *mp2,
                       const orbt_mappoints *M, float s12, const float R12[9], const float t12[3], float th,
                       int32_t *matches12) {
    const int N1 = kf1->n, N2 = kf2->n;
    float sR12[9], sR21[9], t21[3];
    orc_sim3_relative(s12, R12, t12, sR12, sR21, t21);
    uint8_t *am1 = (uint8_t *)calloc((size_t)N1 + 1, 1), *am2 = (uint8_t *)calloc((size_t)N2 + 1, 1);
    for (int i = 0; i < N1; i++) {
        const int m = matches12[i];
        if (m < 0) continue;
        am1[i] = 1;
        for (int j = 0; j < N2; j++)   /* pMP->GetIndexInKeyFrame(pKF2) */
            if (mp2[j] == m) { am2[j] = 1; break; }
    }
    int *v1 = (int *)malloc(sizeof(int) * ((size_t)N1 + 1)), *v2 = (int *)malloc(sizeof(int) * ((size_t)N2 + 1));
    int *cand = (int *)malloc(sizeof(int) * ((size_t)(N1 > N2 ? N1 : N2) + 1));
    orc_frame_grid g1, g2;
    frame_grid(kf1, &g1);
    frame_grid(kf2, &g2);
    sim3_pass(kf1, mp1, am1, kf2, kf1, sR21, t21, M, th, &g2, cand, v1);
    sim3_pass(kf2, mp2, am2, kf1, kf1, sR12, t12, M, th, &g1, cand, v2);
    int nFound = 0;
    for (int i1 = 0; i1 < N1; i1++) {                                            /* :1706-1720 */
        const int idx2 = v1[i1];
        if (idx2 >= 0 && v2[idx2] == i1) {
            matches12[i1] = mp2[idx2];
            nFound++;
        }
    }
    orc_grid_free(&g1); orc_grid_free(&g2);
    free(am1); free(am2); free(v1); free(v2); free(cand);
    return nFound;
}

/* ==========================================================================================
 * BoW-guided matchers: ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
 * (ORBmatcher.cc:236-353) and ORBmatcher::SearchForTriangulation (ORBmatcher.cc:915-1089,
 * CheckDistEpipolarLine :211-231). FeatureVector = sorted node arrays; the reference's
 * while loop with lower_bound visits exactly the nodes present in both.
 * ========================================================================================*/
static int fv_find(const orbb_keyframe *k, uint32_t node) {
    int lo = 0, hi = k->n_fv;
    while (lo < hi) { const int m = (lo + hi) >> 1; if (k->fv_nodes[m] < node) lo = m + 1; else hi = m; }
    return (lo < k->n_fv && k->fv_nodes[lo] == node) ? lo : -1;
}

static void three_maxima_n(const int *counts, int *ind1, int *ind2, int *ind3) { three_maxima30(counts, ind1, ind2, ind3); }

int orc_search_by_bow(const orbb_keyframe *kf, const orbb_keyframe *F, float nnratio, int checkOri, int32_t *matches) {
    const int TH_LOW = 50, HISTO_LENGTH = 30;
    const float factor = HISTO_LENGTH / 360.0f;
    for (int i = 0; i < F->n; i++) matches[i] = -1;
    int *hb = (int *)malloc(sizeof(int) * ((size_t)F->n + 1)), *hi = (int *)malloc(sizeof(int) * ((size_t)F->n + 1));
    int nh = 0, nmatches = 0;
    for (int a = 0; a < kf->n_fv; a++) {
        const int b = fv_find(F, kf->fv_nodes[a]);
        if (b < 0) continue;
        for (int u = kf->fv_start[a]; u < kf->fv_start[a + 1]; u++) {
            const int realIdxKF = kf->fv_features[u];
            const int pMP = kf->mp[realIdxKF];
            if (pMP < 0) continue;
            if (kf->mp_bad && kf->mp_bad[realIdxKF]) continue;
            const uint8_t *dKF = kf->desc + 32 * (size_t)realIdxKF;
            int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
            for (int w = F->fv_start[b]; w < F->fv_start[b + 1]; w++) {
                const int realIdxF = F->fv_features[w];
                if (matches[realIdxF] >= 0) continue;
                const int dist = orc_descriptor_distance(dKF, F->desc + 32 * (size_t)realIdxF);
                if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = realIdxF; }
                else if (dist < bestDist2) bestDist2 = dist;
            }
            if (bestDist1 <= TH_LOW) {
                if ((float)bestDist1 < nnratio * (float)bestDist2) {
                    matches[bestIdxF] = pMP;
                    if (checkOri) {
                        float rot = kf->keys_un[realIdxKF].angle - F->keys_un[bestIdxF].angle;
                        if (rot < 0.0) rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        hb[nh] = bin; hi[nh] = bestIdxF; nh++;
                    }
                    nmatches++;
                }
            }
        }
    }
    if (checkOri) {
        int counts[30] = {0};
        for (int k = 0; k < nh; k++) counts[hb[k]]++;
        int i1 = -1, i2 = -1, i3 = -1;
        three_maxima_n(counts, &i1, &i2, &i3);
        for (int k = 0; k < nh; k++) {
            if (hb[k] == i1 || hb[k] == i2 || hb[k] == i3) continue;
            matches[hi[k]] = -1;
            nmatches--;
        }
    }
    free(hb); free(hi);
    return nmatches;
}

/* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
 * (src/ORBmatcher.cc:760-903; LoopClosing::ComputeSim3 with ORBmatcher(0.75, true)):
 * matches12[idx1] = map point index of pKF2 matched to keypoint idx1 of pKF1, -1 = NULL.
 * Differences to the (KF, F) overload: both sides need a non-bad map point, vbMatched2
 * marks claimed KF2 keypoints, the distance gate is strict (bestDist1 < TH_LOW, :845) and the
 * rotation histogram holds idx1. */
int orc_search_by_bow_kf(const orbb_keyframe *k1, const orbb_keyframe *k2, float nnratio, int checkOri,
                         int32_t *matches12) {
    const int TH_LOW = 50, HISTO_LENGTH = 30;
    const float factor = HISTO_LENGTH / 360.0f;
    for (int i = 0; i < k1->n; i++) matches12[i] = -1;
    uint8_t *matched2 = (uint8_t *)calloc((size_t)k2->n + 1, 1);
    int *hb = (int *)malloc(sizeof(int) * ((size_t)k1->n + 1)), *hi = (int *)malloc(sizeof(int) * ((size_t)k1->n + 1));
    int nh = 0, nmatches = 0;
    for (int a = 0; a < k1->n_fv; a++) {
        const int b = fv_find(k2, k1->fv_nodes[a]);
        if (b < 0) continue;
        for (int u = k1->fv_start[a]; u < k1->fv_start[a + 1]; u++) {
            const int idx1 = k1->fv_features[u];
            if (k1->mp[idx1] < 0) continue;                                     /* :802-806 */
            if (k1->mp_bad && k1->mp_bad[idx1]) continue;
            const uint8_t *d1 = k1->desc + 32 * (size_t)idx1;
            int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
            for (int w = k2->fv_start[b]; w < k2->fv_start[b + 1]; w++) {
                const int idx2 = k2->fv_features[w];
                if (matched2[idx2] || k2->mp[idx2] < 0) continue;                /* :822-826 */
                if (k2->mp_bad && k2->mp_bad[idx2]) continue;
                const int dist = orc_descriptor_distance(d1, k2->desc + 32 * (size_t)idx2);
                if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdx2 = idx2; }
                else if (dist < bestDist2) bestDist2 = dist;
            }
            if (bestDist1 < TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {   /* :845-864 */
                matches12[idx1] = k2->mp[bestIdx2];
                matched2[bestIdx2] = 1;
                if (checkOri) {
                    float rot = k1->keys_un[idx1].angle - k2->keys_un[bestIdx2].angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == HISTO_LENGTH) bin = 0;
                    hb[nh] = bin; hi[nh] = idx1; nh++;
                }
                nmatches++;
            }
        }
    }
    if (checkOri) {                                                              /* :882-900 */
        int counts[30] = {0};
        for (int k = 0; k < nh; k++) counts[hb[k]]++;
        int i1 = -1, i2 = -1, i3 = -1;
        three_maxima_n(counts, &i1, &i2, &i3);
        for (int k = 0; k < nh; k++) {
            if (hb[k] == i1 || hb[k] == i2 || hb[k] == i3) continue;
            matches12[hi[k]] = -1;
            nmatches--;
        }
    }
    free(matched2); free(hb); free(hi);
    return nmatches;
}

static int check_dist_epipolar(const orc_kp *kp1, const orc_kp *kp2, const float F12[9], const orbb_keyframe *kf2) {
    const float a = kp1->x * F12[0] + kp1->y * F12[3] + F12[6];
    const float b = kp1->x * F12[1] + kp1->y * F12[4] + F12[7];
    const float c = kp1->x * F12[2] + kp1->y * F12[5] + F12[8];
    const float num = a * kp2->x + b * kp2->y + c;
    const float den = a * a + b * b;
    if (den == 0) return 0;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * kf2->level_sigma2[kp2->octave];
}

int orc_search_for_triangulation(const orbb_keyframe *kf1, const orbb_keyframe *kf2, const float F12[9],
                                 const float Cw[3], const float T2w[12], int bOnlyStereo, int checkOri,
                                 int32_t *pairs) {
    const int TH_LOW = 50, HISTO_LENGTH = 30;
    const float factor = HISTO_LENGTH / 360.0f;
    float C2[3];
    mat_rx_t(T2w, Cw, C2);
    const float invz = 1.0f / C2[2];
    const float ex = kf2->fx * C2[0] * invz + kf2->cx;
    const float ey = kf2->fy * C2[1] * invz + kf2->cy;
    uint8_t *matched2 = (uint8_t *)calloc((size_t)kf2->n + 1, 1);
    int *m12 = (int *)malloc(sizeof(int) * ((size_t)kf1->n + 1));
    for (int i = 0; i < kf1->n; i++) m12[i] = -1;
    int *hb = (int *)malloc(sizeof(int) * ((size_t)kf1->n + 1)), *hi = (int *)malloc(sizeof(int) * ((size_t)kf1->n + 1));
    int nh = 0, nmatches = 0;
    for (int a = 0; a < kf1->n_fv; a++) {
        const int b = fv_find(kf2, kf1->fv_nodes[a]);
        if (b < 0) continue;
        for (int u = kf1->fv_start[a]; u < kf1->fv_start[a + 1]; u++) {
            const int idx1 = kf1->fv_features[u];
            if (kf1->mp[idx1] >= 0) continue;                     /* GetMapPoint(idx1) != NULL */
            const int bStereo1 = kf1->u_right[idx1] >= 0;
            if (bOnlyStereo && !bStereo1) continue;
            const orc_kp *kp1 = (const orc_kp *)&kf1->keys_un[idx1];
            const uint8_t *d1 = kf1->desc + 32 * (size_t)idx1;
            int bestDist = TH_LOW, bestIdx2 = -1;
            for (int w = kf2->fv_start[b]; w < kf2->fv_start[b + 1]; w++) {
                const int idx2 = kf2->fv_features[w];
                if (matched2[idx2] || kf2->mp[idx2] >= 0) continue;
                const int bStereo2 = kf2->u_right[idx2] >= 0;
                if (bOnlyStereo && !bStereo2) continue;
                const int dist = orc_descriptor_distance(d1, kf2->desc + 32 * (size_t)idx2);
                if (dist > TH_LOW || dist > bestDist) continue;
                const orc_kp *kp2 = (const orc_kp *)&kf2->keys_un[idx2];
                if (!bStereo1 && !bStereo2) {
                    const float distex = ex - kp2->x, distey = ey - kp2->y;
                    if (distex * distex + distey * distey < 100 * kf2->scale_factors[kp2->octave]) continue;
                }
                if (check_dist_epipolar(kp1, kp2, F12, kf2)) { bestIdx2 = idx2; bestDist = dist; }
            }
            if (bestIdx2 >= 0) {
                m12[idx1] = bestIdx2;
                matched2[bestIdx2] = 1;
                nmatches++;
                if (checkOri) {
                    float rot = kp1->angle - kf2->keys_un[bestIdx2].angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == HISTO_LENGTH) bin = 0;
                    hb[nh] = bin; hi[nh] = idx1; nh++;
                }
            }
        }
    }
    if (checkOri) {
        int counts[30] = {0};
        for (int k = 0; k < nh; k++) counts[hb[k]]++;
        int i1 = -1, i2 = -1, i3 = -1;
        three_maxima_n(counts, &i1, &i2, &i3);
        for (int k = 0; k < nh; k++) {
            if (hb[k] == i1 || hb[k] == i2 || hb[k] == i3) continue;
            matched2[m12[hi[k]]] = 0;
            m12[hi[k]] = -1;
            nmatches--;
        }
    }
    int np = 0;
    for (int i = 0; i < kf1->n; i++)
        if (m12[i] >= 0) { pairs[2 * np] = i; pairs[2 * np + 1] = m12[i]; np++; }
    free(matched2); free(m12); free(hb); free(hi);
    return np;
}

/* ==========================================================================================
 * ORBmatcher::Fuse(KeyFrame*, const vector<MapPoint*>&, th), search half (ORBmatcher.cc:
 * 1139-1240; KeyFrame::IsInImage KeyFrame.cc:841-844, KeyFrame::GetFeaturesInArea :794-838,
 * MapPoint::PredictScale(dist, KeyFrame*) MapPoint.cc:584-606).
 * ========================================================================================*/
void orc_fuse_candidates(const orbt_frame *kf, const orbt_mappoints *M, float th, int32_t *best_idx,
                         int32_t *best_dist) {
    orc_frame_grid g;
    frame_grid(kf, &g);
    int *cand = (int *)malloc(sizeof(int) * ((size_t)kf->n + 1));
    for (int i = 0; i < M->n; i++) {
        best_idx[i] = -1;
        best_dist[i] = 256;
        if (M->flags[i] & (ORBT_MP_BAD | ORBT_MP_IN_FRAME)) continue;   /* isBad() || IsInKeyFrame(pKF) */
        const float *P = M->Xw + 3 * (size_t)i;
        float p3Dc[3];
        mat_rx_t(kf->Tcw, P, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = kf->fx * x + kf->cx, v = kf->fy * y + kf->cy;
        if (!(u >= kf->min_x && u < kf->max_x && v >= kf->min_y && v < kf->max_y)) continue;   /* IsInImage */
        const float ur = u - kf->mbf * invz;
        const float maxDistance = 1.2f * M->max_dist[i], minDistance = 0.8f * M->min_dist[i];
        const float PO[3] = {P[0] - kf->Ow[0], P[1] - kf->Ow[1], P[2] - kf->Ow[2]};
        double ss = 0;
        for (int k = 0; k < 3; k++) { const double t = PO[k]; ss += t * t; }
        const float dist3D = (float)sqrt(ss);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float *Pn = M->normal + 3 * (size_t)i;
        double dot = 0;
        for (int k = 0; k < 3; k++) dot += (double)PO[k] * Pn[k];
        if (dot < 0.5 * dist3D) continue;
        const float ratio = M->max_dist[i] / dist3D;
        int nPredictedLevel = (int)ceilf(orc_logf(ratio) / kf->log_scale_factor);
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= kf->nlevels) nPredictedLevel = kf->nlevels - 1;
        const float radius = th * kf->scale_factors[nPredictedLevel];
        const int nc = orc_features_in_area(&g, u, v, radius, -1, -1, cand, kf->n + 1);
        const uint8_t *dMP = M->desc + 32 * (size_t)i;
        int bestDist = 256, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            const orbx_kp *kp = &kf->keys_un[idx];
            const int kpLevel = kp->octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            if (kf->u_right[idx] >= 0) {
                const float ex = u - kp->x, ey = v - kp->y, er = ur - kf->u_right[idx];
                const float e2 = ex * ex + ey * ey + er * er;
                if (e2 * kf->inv_level_sigma2[kpLevel] > 7.8) continue;
            } else {
                const float ex = u - kp->x, ey = v - kp->y;
                const float e2 = ex * ex + ey * ey;
                if (e2 * kf->inv_level_sigma2[kpLevel] > 5.99) continue;
            }
            const int dist = orc_descriptor_distance(dMP, kf->desc + 32 * (size_t)idx);
            if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
        }
        best_idx[i] = bestIdx;
        best_dist[i] = bestDist;
    }
    free(cand);
    orc_grid_free(&g);
}
