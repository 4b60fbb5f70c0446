/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.h). Never linked into the product.
 *
 * Single-threaded C restatement of the per-match triangulation loop of
 * LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:396-600) and of the OpenCV 3.2 pieces it
 * calls, with the float semantics each cv::Mat expression evaluates in:
 *   - Rwc * xn (3x3 * 3x1 CV_32F): small-matrix gemm, float products summed left to right
 *     (SURVEY A.8 / DESIGN.md §3);
 *   - Mat::dot: double products summed left to right; cv::norm: double sum of squares, sqrt
 *     in double (A.8);
 *   - s * Tcw.row(2) - Tcw.row(0): one MatExpr AddEx -> addWeighted_<float, double>:
 *     float(double(a) * s + double(b) * -1 + 0) (OpenCV arithm.cpp);
 *   - x3D.rowRange(0,3) / w: MatExpr AddEx alpha = 1.0 / w -> convertTo(scale) ->
 *     cvtScale_<float, float, float>: float(v * (float)(1.0 / w) + 0.0f);
 *   - cv::SVD::compute(A, w, u, vt, MODIFY_A | FULL_UV) on 4x4 CV_32F: transpose(A), then
 *     JacobiSVDImpl_<float>(At, .., W, Vt, .., m = n = 4, n1 = 4, FLT_MIN, 2 * FLT_EPSILON)
 *     (OpenCV lapack.cpp): one-sided Jacobi over the rows of At with double norms / dots,
 *     hypot, float rotations, up to max(m, 30) sweeps, then a descending selection sort of the
 *     singular values that swaps the rows of At and Vt; vt = Vt. The random completion of U
 *     for zero singular values touches At only, not Vt;
 *   - cos(2 * atan2(mb / 2, depth)) with float arguments resolves to cosf / atan2f
 *     (`using namespace std` from DBoW2's headers, as for logf in track_oracle.c): the live
 *     libm is called here, i.e. the reference's own calls; hypot likewise.
 * These OpenCV internals cannot be checked without OpenCV (absent here): parity
 * of this restatement to the real reference is unpinned; the libm calls are the reference's.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "newpts_oracle.h"

/* JacobiSVDImpl_<float> on At (rows = columns of A), m = n = 4 */
static void jacobi_svd4(float At[4][4], double W[4], float Vt[4][4]) {
    const int m = 4, n = 4, max_iter = 30;   /* std::max(m, 30) */
    const float eps = FLT_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const float t = At[i][k];
            sd += (double)t * t;
        }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i][k] = 0;
        Vt[i][i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                float *Ai = At[i], *Aj = At[j];
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += (double)Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt((double)a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = hypot(p, beta);
                float c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = (float)sqrt(delta / gamma);
                    c = (float)(p / (gamma * s * 2));
                } else {
                    c = (float)sqrt((gamma + beta) / (gamma * 2));
                    s = (float)(p / (gamma * c * 2));
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    const float t0 = c * Ai[k] + s * Aj[k];
                    const float t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += (double)t0 * t0;
                    b += (double)t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                float *Vi = Vt[i], *Vj = Vt[j];
                for (int k = 0; k < n; k++) {   /* VBLAS<float>::givens: same float ops */
                    const float t0 = c * Vi[k] + s * Vj[k];
                    const float t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const float t = At[i][k];
            sd += (double)t * t;
        }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            const double tw = W[i];
            W[i] = W[j];
            W[j] = tw;
            for (int k = 0; k < m; k++) {
                const float t = At[i][k];
                At[i][k] = At[j][k];
                At[j][k] = t;
            }
            for (int k = 0; k < n; k++) {
                const float t = Vt[i][k];
                Vt[i][k] = Vt[j][k];
                Vt[j][k] = t;
            }
        }
    }
}

void orc_svd4_vt(const float A[16], float vt[16], float w[4]) {
    float At[4][4], Vt[4][4];
    double W[4];
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 4; k++) At[i][k] = A[4 * k + i];   /* transpose(src, temp_a) */
    jacobi_svd4(At, W, Vt);
    for (int i = 0; i < 4; i++) {
        w[i] = (float)W[i];
        for (int k = 0; k < 4; k++) vt[4 * i + k] = Vt[i][k];
    }
}

static double dot3d(const float *a, const float *b) {   /* Mat::dot */
    double r = 0;
    for (int k = 0; k < 3; k++) r += (double)a[k] * b[k];
    return r;
}

static double norm3d(const float *a) {   /* cv::norm(NORM_L2) */
    double r = 0;
    for (int k = 0; k < 3; k++) r += (double)a[k] * a[k];
    return sqrt(r);
}

/* Rwc * x with Rwc = Rcw^T (materialised by Rcw.t()): float gemm, left to right */
static void rwc_mul(const float T[12], const float x[3], float o[3]) {
    for (int r = 0; r < 3; r++) {
        float s = T[r] * x[0];
        s = s + T[4 + r] * x[1];
        s = s + T[8 + r] * x[2];
        o[r] = s;
    }
}

int orc_triangulate(const orbn_keyframe *k1, const orbn_keyframe *k2, const int32_t *pairs, int npairs,
                    float ratio_factor, float *x3d, uint8_t *ok) {
    int nnew = 0;
    for (int ikp = 0; ikp < npairs; ikp++) {
        ok[ikp] = 0;
        x3d[3 * ikp] = x3d[3 * ikp + 1] = x3d[3 * ikp + 2] = 0;
        const int idx1 = pairs[2 * ikp], idx2 = pairs[2 * ikp + 1];
        const orbx_kp kp1 = k1->keys_un[idx1], kp2 = k2->keys_un[idx2];
        const float kp1_ur = k1->u_right[idx1], kp2_ur = k2->u_right[idx2];
        const int bStereo1 = kp1_ur >= 0, bStereo2 = kp2_ur >= 0;               /* :418-423 */
        const float xn1[3] = {(kp1.x - k1->cx) * k1->invfx, (kp1.y - k1->cy) * k1->invfy, 1.0f};   /* :424 */
        const float xn2[3] = {(kp2.x - k2->cx) * k2->invfx, (kp2.y - k2->cy) * k2->invfy, 1.0f};
        float ray1[3], ray2[3];
        rwc_mul(k1->Tcw, xn1, ray1);                                             /* :428-429 */
        rwc_mul(k2->Tcw, xn2, ray2);
        const float cosParallaxRays = (float)(dot3d(ray1, ray2) / (norm3d(ray1) * norm3d(ray2)));   /* :432 */
        float cosParallaxStereo = cosParallaxRays + 1;
        float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
        if (bStereo1)                                                            /* :442-447 */
            cosParallaxStereo1 = cosf(2 * atan2f(k1->mb / 2, k1->depth[idx1]));
        else if (bStereo2)
            cosParallaxStereo2 = cosf(2 * atan2f(k2->mb / 2, k2->depth[idx2]));
        cosParallaxStereo = cosParallaxStereo2 < cosParallaxStereo1 ? cosParallaxStereo2 : cosParallaxStereo1;   /* std::min */
        float x3D[3];
        if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
            (bStereo1 || bStereo2 || (double)cosParallaxRays < 0.9998)) {          /* :455 */
            float A[16];                                                         /* :462-466 */
            for (int c = 0; c < 4; c++) {
                A[c] = (float)((double)k1->Tcw[8 + c] * (double)xn1[0] + (double)k1->Tcw[c] * -1.0 + 0.0);
                A[4 + c] = (float)((double)k1->Tcw[8 + c] * (double)xn1[1] + (double)k1->Tcw[4 + c] * -1.0 + 0.0);
                A[8 + c] = (float)((double)k2->Tcw[8 + c] * (double)xn2[0] + (double)k2->Tcw[c] * -1.0 + 0.0);
                A[12 + c] = (float)((double)k2->Tcw[8 + c] * (double)xn2[1] + (double)k2->Tcw[4 + c] * -1.0 + 0.0);
            }
            float vt[16], w[4];
            orc_svd4_vt(A, vt, w);                                               /* :469 */
            const float w3 = vt[15];
            if (w3 == 0) continue;                                               /* :473-474 */
            const float sc = (float)(1.0 / (double)w3);                          /* :476 */
            for (int k = 0; k < 3; k++) x3D[k] = vt[12 + k] * sc + 0.0f;
        } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {        /* :479-483 */
            const float z = k1->depth[idx1];                                     /* KeyFrame::UnprojectStereo */
            if (!(z > 0)) continue;   /* empty Mat: the reference would fault on x3D.t(); not reached */
            const float u = k1->keys[idx1].x, v = k1->keys[idx1].y;
            const float xc[3] = {(u - k1->cx) * z * k1->invfx, (v - k1->cy) * z * k1->invfy, z};
            rwc_mul(k1->Tcw, xc, x3D);
            for (int k = 0; k < 3; k++) x3D[k] = x3D[k] + k1->Ow[k];
        } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {        /* :484-488 */
            const float z = k2->depth[idx2];
            if (!(z > 0)) continue;
            const float u = k2->keys[idx2].x, v = k2->keys[idx2].y;
            const float xc[3] = {(u - k2->cx) * z * k2->invfx, (v - k2->cy) * z * k2->invfy, z};
            rwc_mul(k2->Tcw, xc, x3D);
            for (int k = 0; k < 3; k++) x3D[k] = x3D[k] + k2->Ow[k];
        } else {
            continue;                                                            /* :489-490 */
        }
        /* Rcw.row(r).dot(x3Dt) + tcw(r): double dot + float -> float (:496-506) */
        const float z1 = (float)(dot3d(k1->Tcw + 8, x3D) + (double)k1->Tcw[11]);
        if (z1 <= 0) continue;
        const float z2 = (float)(dot3d(k2->Tcw + 8, x3D) + (double)k2->Tcw[11]);
        if (z2 <= 0) continue;
        const float sigmaSquare1 = k1->level_sigma2[kp1.octave];                 /* :509-531 */
        const float x1 = (float)(dot3d(k1->Tcw, x3D) + (double)k1->Tcw[3]);
        const float y1 = (float)(dot3d(k1->Tcw + 4, x3D) + (double)k1->Tcw[7]);
        const float invz1 = (float)(1.0 / (double)z1);
        if (!bStereo1) {
            const float u1 = k1->fx * x1 * invz1 + k1->cx, v1 = k1->fy * y1 * invz1 + k1->cy;
            const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y;
            if ((double)(errX1 * errX1 + errY1 * errY1) > 5.991 * (double)sigmaSquare1) continue;
        } else {
            const float u1 = k1->fx * x1 * invz1 + k1->cx;
            const float u1_r = u1 - k1->mbf * invz1;
            const float v1 = k1->fy * y1 * invz1 + k1->cy;
            const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y, errX1_r = u1_r - kp1_ur;
            if ((double)(errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * (double)sigmaSquare1) continue;
        }
        const float sigmaSquare2 = k2->level_sigma2[kp2.octave];                 /* :534-561 */
        const float x2 = (float)(dot3d(k2->Tcw, x3D) + (double)k2->Tcw[3]);
        const float y2 = (float)(dot3d(k2->Tcw + 4, x3D) + (double)k2->Tcw[7]);
        const float invz2 = (float)(1.0 / (double)z2);
        if (!bStereo2) {
            const float u2 = k2->fx * x2 * invz2 + k2->cx, v2 = k2->fy * y2 * invz2 + k2->cy;
            const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y;
            if ((double)(errX2 * errX2 + errY2 * errY2) > 5.991 * (double)sigmaSquare2) continue;
        } else {
            const float u2 = k2->fx * x2 * invz2 + k2->cx;
            const float u2_r = u2 - k1->mbf * invz2;   /* mpCurrentKeyFrame->mbf (:553), as written */
            const float v2 = k2->fy * y2 * invz2 + k2->cy;
            const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y, errX2_r = u2_r - kp2_ur;
            if ((double)(errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * (double)sigmaSquare2) continue;
        }
        float normal1[3], normal2[3];                                            /* :566-575 */
        for (int k = 0; k < 3; k++) {
            normal1[k] = x3D[k] - k1->Ow[k];
            normal2[k] = x3D[k] - k2->Ow[k];
        }
        const float dist1 = (float)norm3d(normal1), dist2 = (float)norm3d(normal2);
        if (dist1 == 0 || dist2 == 0) continue;
        const float ratioDist = dist2 / dist1;                                   /* :578-587 */
        const float ratioOctave = k1->scale_factors[kp1.octave] / k2->scale_factors[kp2.octave];
        if (ratioDist * ratio_factor < ratioOctave || ratioDist > ratioOctave * ratio_factor) continue;
        ok[ikp] = 1;                                                             /* :589-600 */
        memcpy(x3d + 3 * ikp, x3D, sizeof x3D);
        nnew++;
    }
    return nnew;
}
