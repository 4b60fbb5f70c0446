// MI355X-native triangulation of new map points: the per-match body of
// LocalMapping::CreateNewMapPoints (LocalMapping.cc:396-600), SURVEY.md §8f rank 4.
//
// Every match of every (current keyframe, neighbour) slot is independent -- the reference
// creates a MapPoint per accepted match without reading earlier ones -- so one thread owns one
// match: parallax test, the 4x4 linear triangulation through OpenCV's float one-sided Jacobi
// SVD (cv::SVD::compute with MODIFY_A | FULL_UV, lapack.cpp JacobiSVDImpl_: double norms and
// dots, hypot, float Givens rotations, descending selection sort) held in registers, or
// KeyFrame::UnprojectStereo, then the depth, reprojection-chi2 and scale-consistency gates.
// Float / double semantics follow oracle/newpts_oracle.c operation by operation (-ffp-contract=off);
// atan2f / hypot / cosf are the glibc algorithms restated in libm_restate.h / orb_device.h and
// pinned against the live libm by oracle/tools.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <vector>

#include "libm_restate.h"
#include "orb_device.h"
#include "orb_engine.h"
#include "orbslam2_amd.h"

using namespace orbamd;

#define NP_CHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd newpts: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace orbnp {

constexpr int kMaxKp = 65535;

struct KFHdr {
    float Tcw[12], Ow[3];
    float fx, fy, cx, cy, invfx, invfy, mb, mbf;
    float sf[16], s2[16];
};

struct SlotHdr {
    int npairs;
    float ratio_factor;
    KFHdr k[2];
};

struct Slots {
    const SlotHdr *hdr;
    const float4 *kp[2];        // [S][cap] (keys.x, keys.y, keys_un.x, keys_un.y)
    const int *oct[2];          // [S][cap] keys_un octave
    const float2 *ud[2];        // [S][cap] (mvuRight, mvDepth)
    const int2 *pairs;          // [S][cap_pairs]
    float *x3d;                 // [S][cap_pairs][3]
    uint8_t *ok;                // [S][cap_pairs]
    int *nnew;                  // [S]
    int cap, cap_pairs;
};

__device__ __forceinline__ double dot3d(const float *a, const float *b) {   // Mat::dot
    double r = 0;
    r += (double)a[0] * b[0];
    r += (double)a[1] * b[1];
    r += (double)a[2] * b[2];
    return r;
}

__device__ __forceinline__ double norm3d(const float *a) {   // cv::norm(NORM_L2)
    double r = 0;
    r += (double)a[0] * a[0];
    r += (double)a[1] * a[1];
    r += (double)a[2] * a[2];
    return sqrt(r);
}

__device__ __forceinline__ void rwc_mul(const float *T, const float x[3], float o[3]) {   // Rcw^T * x, float gemm
#pragma unroll
    for (int r = 0; r < 3; r++) {
        float s = T[r] * x[0];
        s = s + T[4 + r] * x[1];
        s = s + T[8 + r] * x[2];
        o[r] = s;
    }
}

// JacobiSVDImpl_<float> on At (rows = columns of A), m = n = 4; returns Vt's row of the smallest
// singular value after OpenCV's descending selection sort (vt.row(3)).
__device__ __forceinline__ void jacobi_svd4_vt3(float At[4][4], float v3[4]) {
    float Vt[4][4];
    double W[4];
    const float eps = FLT_EPSILON * 2;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) sd += (double)At[i][k] * At[i][k];
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < 4; k++) Vt[i][k] = i == k ? 1.0f : 0.0f;
    }
    for (int iter = 0; iter < 30; iter++) {   // std::max(m, 30)
        bool changed = false;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = i + 1; j < 4; j++) {
                double a = W[i], p = 0, b = W[j];
#pragma unroll
                for (int k = 0; k < 4; k++) p += (double)At[i][k] * At[j][k];
                if (fabs(p) <= (double)eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = lm_hypot(p, beta);
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
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float t0 = c * At[i][k] + s * At[j][k];
                    const float t1 = -s * At[i][k] + c * At[j][k];
                    At[i][k] = t0;
                    At[j][k] = t1;
                    a += (double)t0 * t0;
                    b += (double)t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float t0 = c * Vt[i][k] + s * Vt[j][k];
                    const float t1 = -s * Vt[i][k] + c * Vt[j][k];
                    Vt[i][k] = t0;
                    Vt[j][k] = t1;
                }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) sd += (double)At[i][k] * At[i][k];
        W[i] = sqrt(sd);
    }
    // selection sort, descending (strict <), swapping W and the Vt rows (At rows are not read)
#pragma unroll
    for (int i = 0; i < 3; i++) {
        int j = i;
#pragma unroll
        for (int k = i + 1; k < 4; k++)
            if (W[j] < W[k]) j = k;
#pragma unroll
        for (int jj = i + 1; jj < 4; jj++) {
            if (j == jj) {
                const double tw = W[i];
                W[i] = W[jj];
                W[jj] = tw;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const float t = Vt[i][k];
                    Vt[i][k] = Vt[jj][k];
                    Vt[jj][k] = t;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) v3[k] = Vt[3][k];
}

__global__ __launch_bounds__(256) void triangulate_kernel(Slots S) {
    const int s = blockIdx.y, ikp = blockIdx.x * 256 + threadIdx.x;
    const SlotHdr &H = S.hdr[s];
    if (ikp >= H.npairs) return;
    const KFHdr &k1 = H.k[0], &k2 = H.k[1];
    const long long o = (long long)s * S.cap;
    const long long po = (long long)s * S.cap_pairs + ikp;
    const int2 pr = S.pairs[po];
    const int idx1 = pr.x, idx2 = pr.y;
    const float4 P1 = S.kp[0][o + idx1], P2 = S.kp[1][o + idx2];   // (x, y, xUn, yUn)
    const int oct1 = S.oct[0][o + idx1], oct2 = S.oct[1][o + idx2];
    const float2 U1 = S.ud[0][o + idx1], U2 = S.ud[1][o + idx2];   // (uR, depth)
    const float kp1_ur = U1.x, kp2_ur = U2.x;
    const bool bStereo1 = kp1_ur >= 0, bStereo2 = kp2_ur >= 0;                       // :418-423
    const float xn1[3] = {(P1.z - k1.cx) * k1.invfx, (P1.w - k1.cy) * k1.invfy, 1.0f};   // :424
    const float xn2[3] = {(P2.z - k2.cx) * k2.invfx, (P2.w - k2.cy) * k2.invfy, 1.0f};
    float ray1[3], ray2[3];
    rwc_mul(k1.Tcw, xn1, ray1);                                                      // :428-429
    rwc_mul(k2.Tcw, xn2, ray2);
    const float cosParallaxRays = (float)(dot3d(ray1, ray2) / (norm3d(ray1) * norm3d(ray2)));   // :432
    float cosParallaxStereo = cosParallaxRays + 1;
    float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
    float sn;
    if (bStereo1)                                                                    // :442-447
        glibc_sincosf(2 * lm_atan2f(k1.mb / 2, U1.y), &sn, &cosParallaxStereo1);
    else if (bStereo2)
        glibc_sincosf(2 * lm_atan2f(k2.mb / 2, U2.y), &sn, &cosParallaxStereo2);
    cosParallaxStereo = cosParallaxStereo2 < cosParallaxStereo1 ? cosParallaxStereo2 : cosParallaxStereo1;
    float x3D[3];
    bool valid = true;
    if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
        (bStereo1 || bStereo2 || (double)cosParallaxRays < 0.9998)) {                 // :455
        float At[4][4];   // transpose(A): At[c][r] = A[r][c]                            :462-466
#pragma unroll
        for (int c = 0; c < 4; c++) {
            At[c][0] = (float)((double)k1.Tcw[8 + c] * (double)xn1[0] + (double)k1.Tcw[c] * -1.0 + 0.0);
            At[c][1] = (float)((double)k1.Tcw[8 + c] * (double)xn1[1] + (double)k1.Tcw[4 + c] * -1.0 + 0.0);
            At[c][2] = (float)((double)k2.Tcw[8 + c] * (double)xn2[0] + (double)k2.Tcw[c] * -1.0 + 0.0);
            At[c][3] = (float)((double)k2.Tcw[8 + c] * (double)xn2[1] + (double)k2.Tcw[4 + c] * -1.0 + 0.0);
        }
        float v3[4];
        jacobi_svd4_vt3(At, v3);                                                     // :469
        if (v3[3] == 0) {
            valid = false;                                                           // :473-474
        } else {
            const float sc = (float)(1.0 / (double)v3[3]);                           // :476
#pragma unroll
            for (int k = 0; k < 3; k++) x3D[k] = v3[k] * sc + 0.0f;
        }
    } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {               // :479-483 UnprojectStereo
        const float z = U1.y;
        valid = z > 0;   // an empty Mat in the reference (unreachable: uR >= 0 implies depth > 0)
        const float xc[3] = {(P1.x - k1.cx) * z * k1.invfx, (P1.y - k1.cy) * z * k1.invfy, z};
        rwc_mul(k1.Tcw, xc, x3D);
#pragma unroll
        for (int k = 0; k < 3; k++) x3D[k] = x3D[k] + k1.Ow[k];
    } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {               // :484-488
        const float z = U2.y;
        valid = z > 0;
        const float xc[3] = {(P2.x - k2.cx) * z * k2.invfx, (P2.y - k2.cy) * z * k2.invfy, z};
        rwc_mul(k2.Tcw, xc, x3D);
#pragma unroll
        for (int k = 0; k < 3; k++) x3D[k] = x3D[k] + k2.Ow[k];
    } else {
        valid = false;                                                               // :489-490
    }
    if (valid) {
        const float z1 = (float)(dot3d(k1.Tcw + 8, x3D) + (double)k1.Tcw[11]);     // :496-506
        const float z2 = (float)(dot3d(k2.Tcw + 8, x3D) + (double)k2.Tcw[11]);
        valid = z1 > 0 && z2 > 0;
        if (valid) {                                                                 // :509-531
            const float sigmaSquare1 = k1.s2[oct1];
            const float x1 = (float)(dot3d(k1.Tcw, x3D) + (double)k1.Tcw[3]);
            const float y1 = (float)(dot3d(k1.Tcw + 4, x3D) + (double)k1.Tcw[7]);
            const float invz1 = (float)(1.0 / (double)z1);
            const float u1 = k1.fx * x1 * invz1 + k1.cx, v1 = k1.fy * y1 * invz1 + k1.cy;
            const float errX1 = u1 - P1.z, errY1 = v1 - P1.w;
            if (!bStereo1) {
                valid = !((double)(errX1 * errX1 + errY1 * errY1) > 5.991 * (double)sigmaSquare1);
            } else {
                const float u1_r = u1 - k1.mbf * invz1;
                const float errX1_r = u1_r - kp1_ur;
                valid = !((double)(errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * (double)sigmaSquare1);
            }
        }
        if (valid) {                                                                 // :534-561
            const float sigmaSquare2 = k2.s2[oct2];
            const float x2 = (float)(dot3d(k2.Tcw, x3D) + (double)k2.Tcw[3]);
            const float y2 = (float)(dot3d(k2.Tcw + 4, x3D) + (double)k2.Tcw[7]);
            const float invz2 = (float)(1.0 / (double)z2);
            const float u2 = k2.fx * x2 * invz2 + k2.cx, v2 = k2.fy * y2 * invz2 + k2.cy;
            const float errX2 = u2 - P2.z, errY2 = v2 - P2.w;
            if (!bStereo2) {
                valid = !((double)(errX2 * errX2 + errY2 * errY2) > 5.991 * (double)sigmaSquare2);
            } else {
                const float u2_r = u2 - k1.mbf * invz2;   // mpCurrentKeyFrame->mbf (:553), as written
                const float errX2_r = u2_r - kp2_ur;
                valid = !((double)(errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * (double)sigmaSquare2);
            }
        }
        if (valid) {                                                                 // :566-587
            float n1[3], n2[3];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                n1[k] = x3D[k] - k1.Ow[k];
                n2[k] = x3D[k] - k2.Ow[k];
            }
            const float dist1 = (float)norm3d(n1), dist2 = (float)norm3d(n2);
            if (dist1 == 0 || dist2 == 0) {
                valid = false;
            } else {
                const float ratioDist = dist2 / dist1;
                const float ratioOctave = k1.sf[oct1] / k2.sf[oct2];
                valid = !(ratioDist * H.ratio_factor < ratioOctave || ratioDist > ratioOctave * H.ratio_factor);
            }
        }
    }
    float *xo = S.x3d + po * 3;
    xo[0] = valid ? x3D[0] : 0.0f;
    xo[1] = valid ? x3D[1] : 0.0f;
    xo[2] = valid ? x3D[2] : 0.0f;
    S.ok[po] = valid ? 1 : 0;
    const unsigned long long bal = __ballot(valid);
    if (bal && __lane_id() == (unsigned)__builtin_ctzll(bal)) atomicAdd(&S.nnew[s], __popcll(bal));
}

}  // namespace orbnp

using namespace orbnp;

struct orbn_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;          // end of the last run (fetch waits on it only)
    hipStream_t done_stream = nullptr;
    int nslots = 0, cap = 0, cap_pairs = 0;
    std::vector<SlotHdr> h;
    DevBuf hdr, kp[2], oct[2], ud[2], pairs, x3d, ok, nnew;
    std::vector<float4> tkp;
    std::vector<int> toct;
    std::vector<float2> tud;
};

static Slots make_slots(orbn_engine *e) {
    Slots S;
    S.hdr = e->hdr.as<SlotHdr>();
    for (int i = 0; i < 2; i++) {
        S.kp[i] = e->kp[i].as<float4>();
        S.oct[i] = e->oct[i].as<int>();
        S.ud[i] = e->ud[i].as<float2>();
    }
    S.pairs = e->pairs.as<int2>();
    S.x3d = e->x3d.as<float>();
    S.ok = e->ok.as<uint8_t>();
    S.nnew = e->nnew.as<int>();
    S.cap = e->cap;
    S.cap_pairs = e->cap_pairs;
    return S;
}

static int validate(const orbn_keyframe *k, int cap) {
    if (!k || k->n < 0 || k->n > cap) return ORBX_EINVAL;
    if (k->n > 0 && (!k->keys || !k->keys_un || !k->u_right || !k->depth)) return ORBX_EINVAL;
    if (k->nlevels < 1 || k->nlevels > 16) return ORBX_EINVAL;
    return ORBX_OK;
}

extern "C" {

int orbn_create(orbn_engine **out) {
    if (!out) return ORBX_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORBX_EDEVICE;
    orbn_engine *e = new orbn_engine();
    if (hipGetDevice(&e->device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        !(e->done = make_done_event())) {
        delete e;
        return ORBX_EDEVICE;
    }
    *out = e;
    return ORBX_OK;
}

void orbn_destroy(orbn_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) { (void)hipStreamSynchronize(e->stream); (void)hipStreamDestroy(e->stream); }
    if (e->done) { (void)hipEventSynchronize(e->done); (void)hipEventDestroy(e->done); }
    DevBuf *bufs[] = {&e->hdr, &e->kp[0], &e->kp[1], &e->oct[0], &e->oct[1], &e->ud[0], &e->ud[1],
                      &e->pairs, &e->x3d, &e->ok, &e->nnew};
    for (DevBuf *b : bufs) b->release();
    delete e;
}

int orbn_reserve(orbn_engine *e, int n_slots, int cap_kp, int cap_pairs) {
    if (!e || n_slots <= 0 || cap_kp <= 0 || cap_kp > kMaxKp || cap_pairs <= 0) return ORBX_EINVAL;
    NP_CHK(hipSetDevice(e->device));
    const size_t S = (size_t)n_slots, C = (size_t)cap_kp, P = (size_t)cap_pairs;
    for (int i = 0; i < 2; i++)
        if (e->kp[i].ensure(16 * S * C) || e->oct[i].ensure(4 * S * C) || e->ud[i].ensure(8 * S * C)) return ORBX_EDEVICE;
    if (e->hdr.ensure(sizeof(SlotHdr) * S) || e->pairs.ensure(8 * S * P) || e->x3d.ensure(12 * S * P) ||
        e->ok.ensure(S * P) || e->nnew.ensure(4 * S))
        return ORBX_EDEVICE;
    e->nslots = n_slots;
    e->cap = cap_kp;
    e->cap_pairs = cap_pairs;
    e->h.assign(n_slots, SlotHdr{});
    return ORBX_OK;
}

int orbn_stage(orbn_engine *e, int slot, const orbn_keyframe *kf1, const orbn_keyframe *kf2, const int32_t *pairs,
               int32_t npairs, float ratio_factor) {
    if (!e || slot < 0 || slot >= e->nslots || npairs < 0 || npairs > e->cap_pairs || (npairs && !pairs))
        return ORBX_EINVAL;
    int rc = validate(kf1, e->cap);
    if (!rc) rc = validate(kf2, e->cap);
    if (rc) return rc;
    for (int k = 0; k < npairs; k++)   // host-side bounds check: the kernel indexes with these
        if (pairs[2 * k] < 0 || pairs[2 * k] >= kf1->n || pairs[2 * k + 1] < 0 || pairs[2 * k + 1] >= kf2->n)
            return ORBX_EINVAL;
    const orbn_keyframe *K[2] = {kf1, kf2};
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < K[i]->n; j++)
            if (K[i]->keys_un[j].octave < 0 || K[i]->keys_un[j].octave >= K[i]->nlevels) return ORBX_EINVAL;
    NP_CHK(hipSetDevice(e->device));
    SlotHdr &h = e->h[slot];
    h = SlotHdr{};
    h.npairs = npairs;
    h.ratio_factor = ratio_factor;
    const size_t C = (size_t)e->cap, s = (size_t)slot;
    hipStream_t st = e->stream;
    NP_CHK(order_after_done(e, st));
    for (int i = 0; i < 2; i++) {
        KFHdr &d = h.k[i];
        const orbn_keyframe *k = K[i];
        std::memcpy(d.Tcw, k->Tcw, sizeof d.Tcw);
        std::memcpy(d.Ow, k->Ow, sizeof d.Ow);
        d.fx = k->fx; d.fy = k->fy; d.cx = k->cx; d.cy = k->cy;
        d.invfx = k->invfx; d.invfy = k->invfy; d.mb = k->mb; d.mbf = k->mbf;
        std::memcpy(d.sf, k->scale_factors, sizeof d.sf);
        std::memcpy(d.s2, k->level_sigma2, sizeof d.s2);
        e->tkp.resize(k->n);
        e->toct.resize(k->n);
        e->tud.resize(k->n);
        for (int j = 0; j < k->n; j++) {
            e->tkp[j] = make_float4(k->keys[j].x, k->keys[j].y, k->keys_un[j].x, k->keys_un[j].y);
            e->toct[j] = k->keys_un[j].octave;
            e->tud[j] = make_float2(k->u_right[j], k->depth[j]);
        }
        if (k->n) {
            NP_CHK(hipMemcpyAsync((char *)e->kp[i].p + 16 * s * C, e->tkp.data(), 16 * (size_t)k->n, hipMemcpyHostToDevice, st));
            NP_CHK(hipMemcpyAsync((char *)e->oct[i].p + 4 * s * C, e->toct.data(), 4 * (size_t)k->n, hipMemcpyHostToDevice, st));
            NP_CHK(hipMemcpyAsync((char *)e->ud[i].p + 8 * s * C, e->tud.data(), 8 * (size_t)k->n, hipMemcpyHostToDevice, st));
            NP_CHK(hipStreamSynchronize(st));   // the staging vectors are reused for kf2
        }
    }
    NP_CHK(hipMemcpyAsync((char *)e->hdr.p + sizeof(SlotHdr) * s, &h, sizeof h, hipMemcpyHostToDevice, st));
    if (npairs)
        NP_CHK(hipMemcpyAsync((char *)e->pairs.p + 8 * s * (size_t)e->cap_pairs, pairs, 8 * (size_t)npairs,
                              hipMemcpyHostToDevice, st));
    NP_CHK(hipStreamSynchronize(st));
    return ORBX_OK;
}

int orbn_run_batch(orbn_engine *e, int n_slots, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    NP_CHK(hipSetDevice(e->device));
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    int maxp = 1;
    for (int s = 0; s < n_slots; s++) maxp = std::max(maxp, e->h[s].npairs);
    NP_CHK(order_after_done(e, st));
    NP_CHK(hipMemsetAsync(e->nnew.p, 0, 4 * (size_t)n_slots, st));
    triangulate_kernel<<<dim3((maxp + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e));
    NP_CHK(hipGetLastError());
    NP_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbn_fetch(orbn_engine *e, int slot, float *x3d, uint8_t *ok, int32_t *nnew) {
    if (!e || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    NP_CHK(hipSetDevice(e->device));
    NP_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    const size_t s = (size_t)slot, P = (size_t)e->cap_pairs, n = (size_t)e->h[slot].npairs;
    if (nnew) NP_CHK(d2h_sync(nnew, (char *)e->nnew.p + 4 * s, 4, e->stream));
    if (n) {
        if (x3d) NP_CHK(d2h_sync(x3d, (char *)e->x3d.p + 12 * s * P, 12 * n, e->stream));
        if (ok) NP_CHK(d2h_sync(ok, (char *)e->ok.p + s * P, n, e->stream));
    }
    return ORBX_OK;
}

int orbn_triangulate(orbn_engine *e, const orbn_keyframe *kf1, const orbn_keyframe *kf2, const int32_t *pairs,
                     int32_t npairs, float ratio_factor, float *x3d, uint8_t *ok, int32_t *nnew) {
    if (!e || !kf1 || !kf2 || npairs < 0 || (npairs && (!pairs || !x3d || !ok)) || !nnew) return ORBX_EINVAL;
    const int need = std::max(1, std::max(kf1->n, kf2->n));
    if (e->nslots < 1 || e->cap < need || e->cap_pairs < std::max(1, npairs)) {
        const int rc = orbn_reserve(e, std::max(1, e->nslots), std::max(e->cap, need), std::max(e->cap_pairs, std::max(1, npairs)));
        if (rc) return rc;
    }
    int rc = orbn_stage(e, 0, kf1, kf2, pairs, npairs, ratio_factor);
    if (!rc) rc = orbn_run_batch(e, 1, nullptr);
    if (!rc) rc = orbn_fetch(e, 0, x3d, ok, nnew);
    return rc;
}

}  // extern "C"
