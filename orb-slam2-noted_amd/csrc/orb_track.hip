// MI355X-native per-frame tracking matchers:
//   Frame::isInFrustum                        Frame.cc:490-578 (+ MapPoint::PredictScale
//                                             MapPoint.cc:612-626, glibc logf restated)
//   ORBmatcher::SearchByProjection(F, vpMapPoints, th)      ORBmatcher.cc:78-176
//   ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono)  ORBmatcher.cc:1741-1904
//   ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
//                                             ORBmatcher.cc:1922-2066 (relocalisation; the
//                                             keyframe takes the last frame's slot)
//   ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint), search half  ORBmatcher.cc:1321-1437
//   ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)  ORBmatcher.cc:1472-1723
//   ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
//                                             ORBmatcher.cc:431-560 (loop closing: the
//                                             keyframe takes the frame's slot, Sim3 pose
//                                             unscaled on the host, queries = map points)
//
// Both matchers are greedy: map points (resp. last-frame keypoints) are visited in order and
// a keypoint claimed by a map point with Observations() > 0 is skipped by every later one.
// Everything that does not depend on the claims runs fully parallel, one thread per map
// point (resp. last keypoint), in the *_cand kernels: frustum test, grid window, level /
// stereo filters, Hamming distances, and the K smallest candidates by (distance, candidate
// position) -- the (best, second) pair of the reference's sequential update is exactly the
// two smallest (distance, position) keys among the unclaimed candidates. The *_resolve
// kernels replay the claim order per frame (one workgroup per frame, map-point records staged
// through LDS, the claim set in LDS); when claims remove too many of a point's K kept
// candidates the point's window is rescanned with the claim set (exact fallback).
//
// Frames are batched in slots (one (frame, map) problem per slot) for throughput; the
// single-frame C-ABI entry points use slot 0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "orb_device.h"
#include "orb_engine.h"

using namespace orbamd;

#define TR_CHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd track: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace orbtrack {

constexpr int GRID_COLS = 64, GRID_ROWS = 48;   // Frame.h:55-60
constexpr int NCELL = GRID_COLS * GRID_ROWS;
constexpr int TOPK = 4;                          // kept candidates per map point
constexpr int TH_HIGH = 100, HISTO_LENGTH = 30;  // ORBmatcher.cc:56-58
constexpr int kMaxKp = 8192;                     // grid keys sorted in LDS; idx fits 16 bits

struct FrameDev {
    int n, n_mp, n_last;
    float Tcw[12];
    float Ow[3];
    float fx, fy, cx, cy, mbf, mb;
    float min_x, max_x, min_y, max_y, inv_w, inv_h;
    int nlevels;
    float log_scale;
    float scale[16];
    float inv_s2[16];  // mvInvLevelSigma2 (Fuse)
    float lTcw[12];   // last frame pose (frame-to-frame matcher); source keyframe pose (SearchBySim3)
    float sT[12];     // SearchBySim3: [sR | t] from the source camera into this (target) keyframe's camera
    float pfx, pfy, pcx, pcy;   // SearchBySim3: pKF1's intrinsics project in both directions
};

// per-slot device arrays (slot stride = cap)
struct Slots {
    const FrameDev *fr;
    const orbx_kp *kun;      // [S][cap_kp]
    const float *uR;         // [S][cap_kp]
    const uint8_t *desc;     // [S][cap_kp][32]
    const uint8_t *blocked;  // [S][cap_kp]
    const float4 *grec;      // [S][sort_cap] grid-sorted {x, y, uR, idx | octave << 16 | blocked << 24}
    const int *cell_start;   // [S][NCELL + 1]
    const orbx_kp *lkun;     // [S][cap_kp] last frame
    const int *last_mp;      // [S][cap_kp]
    const uint8_t *last_out; // [S][cap_kp]
    const float *Xw, *nrm, *mind, *maxd;   // [S][cap_mp][3] / [S][cap_mp]
    const uint8_t *mdesc, *mflags;         // [S][cap_mp][32] / [S][cap_mp]
    int cap_kp, cap_mp, sort_cap;
};

struct Cand {   // K smallest candidate keys of one query (sorted ascending)
    uint32_t key[TOPK];   // dist << 16 | candidate position; 0xFFFFFFFF = empty
    uint16_t idx[TOPK];
    int8_t oct[TOPK];
    int8_t bin[TOPK];     // rotation-histogram bin (frame-to-frame only)
};

// ---- glibc 2.35 logf, restated (bit-identical to libm over every positive float: oracle pin
// oracle/tools/check_logf.c); std::log(float) of MapPoint::PredictScale
__constant__ double kLogfInvc[16] = {
    0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
    0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
    0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
    0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
__constant__ double kLogfLogc[16] = {
    -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
    -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3,   -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4,
    -0x1.252f438e10c1ep-5, 0x0p+0,                0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
    0x1.526e57720db08p-3,  0x1.bc2860d22477p-3,   0x1.1058bc8a07ee1p-2,  0x1.4043057b6ee09p-2};

__device__ inline float glibc_logf(float x) {
    uint32_t ix = __float_as_uint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;
        ix = __float_as_uint(x * 0x1p23f) - (23u << 23);
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double z = (double)__uint_as_float(iz);
    const double r = z * kLogfInvc[i] - 1;
    const double y0 = kLogfLogc[i] + (double)k * 0x1.62e42fefa39efp-1;
    const double r2 = r * r;
    double y = 0x1.5575b0be00b6ap-2 * r + -0x1.ffffef20a4123p-2;
    y = -0x1.00ea348b88334p-2 * r2 + y;
    y = y * r2 + (y0 + r);
    return (float)y;
}

// R * X + t with cv::Mat CV_32F semantics (float products summed left to right, then + t)
__device__ inline void mat_rx_t(const float *T, const float *X, float o[3]) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float s = T[4 * i] * X[0];
        s = s + T[4 * i + 1] * X[1];
        s = s + T[4 * i + 2] * X[2];
        o[i] = s + T[4 * i + 3];
    }
}


// insert into the sorted K-list; every index is a compile-time constant (unrolled compare-and-
// swap), so the list stays in registers instead of scratch memory
__device__ inline void cand_insert(Cand &c, uint32_t key, int idx, int oct, int bin) {
    if (key >= c.key[TOPK - 1]) return;
    c.key[TOPK - 1] = key; c.idx[TOPK - 1] = (uint16_t)idx; c.oct[TOPK - 1] = (int8_t)oct; c.bin[TOPK - 1] = (int8_t)bin;
#pragma unroll
    for (int p = TOPK - 1; p > 0; p--) {
        if (c.key[p] < c.key[p - 1]) {
            const uint32_t k = c.key[p]; c.key[p] = c.key[p - 1]; c.key[p - 1] = k;
            const uint16_t i = c.idx[p]; c.idx[p] = c.idx[p - 1]; c.idx[p - 1] = i;
            const int8_t o = c.oct[p]; c.oct[p] = c.oct[p - 1]; c.oct[p - 1] = o;
            const int8_t b = c.bin[p]; c.bin[p] = c.bin[p - 1]; c.bin[p - 1] = b;
        }
    }
}

// the first `want` (1 or 2) unclaimed entries of a K-list, constant-index scan
struct Pick {
    int found, last_ex;          // entries found; index of the last entry examined
    uint32_t key0, key1;
    int idx0, idx1, oct0, oct1, bin0;
};

__device__ inline Pick pick_unclaimed(const Cand &c, const uint8_t *claimed, int want) {
    Pick r;
    r.found = 0; r.last_ex = -1;
    r.key0 = r.key1 = 0xFFFFFFFFu;
    r.idx0 = r.idx1 = 0; r.oct0 = r.oct1 = -1; r.bin0 = -1;
    bool done = false;
#pragma unroll
    for (int k = 0; k < TOPK; k++) {
        if (!done && c.key[k] != 0xFFFFFFFFu) {
            r.last_ex = k;
            if (!claimed[c.idx[k]]) {
                if (r.found == 0) { r.key0 = c.key[k]; r.idx0 = c.idx[k]; r.oct0 = c.oct[k]; r.bin0 = c.bin[k]; }
                else { r.key1 = c.key[k]; r.idx1 = c.idx[k]; r.oct1 = c.oct[k]; }
                r.found++;
                if (r.found == want) done = true;
            }
        } else {
            done = true;
        }
    }
    return r;
}

// any kept entry in [0, last_ex] claimed (tag < lane) by an earlier lane of the window
__device__ inline bool examined_conflict(const Cand &c, int last_ex, const int *tag, int lane) {
    bool conflict = false;
#pragma unroll
    for (int k = 0; k < TOPK; k++)
        if (k <= last_ex) conflict |= tag[c.idx[k]] < lane;
    return conflict;
}

// Frame::GetFeaturesInArea (Frame.cc:590-671) window: returns false if empty.
__device__ inline bool grid_window(const FrameDev &f, float x, float y, float r, int &x0, int &x1, int &y0,
                                   int &y1) {
    x0 = max(0, (int)floorf((x - f.min_x - r) * f.inv_w));
    if (x0 >= GRID_COLS) return false;
    x1 = min(GRID_COLS - 1, (int)ceilf((x - f.min_x + r) * f.inv_w));
    if (x1 < 0) return false;
    y0 = max(0, (int)floorf((y - f.min_y - r) * f.inv_h));
    if (y0 >= GRID_ROWS) return false;
    y1 = min(GRID_ROWS - 1, (int)ceilf((y - f.min_y + r) * f.inv_h));
    if (y1 < 0) return false;
    return true;
}

// Scan the window in the reference's candidate order (ix, iy, insertion order) applying the
// static filters; `claimed` (may be null) adds the dynamic claim filter (rescan fallback).
// Returns the number of candidates that passed; keeps the K smallest (dist, position) keys.
template <bool kLocal>
__device__ int scan_window(const Slots &S, int s, const FrameDev &f, float x, float y, float r, int minL,
                           int maxL, const uint8_t *qdesc, float xr, float er_r, const uint8_t *claimed,
                           float last_angle, Cand &c) {
#pragma unroll
    for (int k = 0; k < TOPK; k++) { c.key[k] = 0xFFFFFFFFu; c.idx[k] = 0; c.oct[k] = -1; c.bin[k] = -1; }
    int cx0, cx1, cy0, cy1;
    if (!grid_window(f, x, y, r, cx0, cx1, cy0, cy1)) return 0;
    const bool bCheckLevels = (minL > 0) || (maxL >= 0);
    const float4 *rec = S.grec + (long long)s * S.sort_cap;
    const int *cs = S.cell_start + (long long)s * (NCELL + 1);
    const long long kb = (long long)s * S.cap_kp;
    int pos = 0, n = 0;
    for (int ix = cx0; ix <= cx1; ix++) {
        const int a = cs[ix * GRID_ROWS + cy0], b = cs[ix * GRID_ROWS + cy1 + 1];
        for (int t = a; t < b; t++) {
            const float4 g = rec[t];
            const uint32_t pk = __float_as_uint(g.w);
            const int idx = (int)(pk & 0xFFFFu), oct = (int)((pk >> 16) & 0xFF);
            if (bCheckLevels) {
                if (oct < minL) continue;
                if (maxL >= 0 && oct > maxL) continue;
            }
            const float distx = g.x - x, disty = g.y - y;
            if (!(fabsf(distx) < r && fabsf(disty) < r)) continue;
            const int p = pos++;                       // position in vIndices order
            if (pk >> 24) continue;                    // owned on entry by a point with observations
            if (claimed && claimed[idx]) continue;
            const float ur = g.z;
            if (ur > 0) {
                const float er = fabsf(xr - ur);
                if (er > er_r) continue;
            }
            const int dist = hamming32(qdesc, S.desc + (kb + idx) * 32);
            int bin = -1;
            if (!kLocal) {
                float rot = last_angle - S.kun[kb + idx].angle;   // ORBmatcher.cc:1872-1878
                if (rot < 0.0f) rot += 360.0f;
                bin = (int)roundf(rot * (HISTO_LENGTH / 360.0f));
                if (bin == HISTO_LENGTH) bin = 0;
            }
            n++;
            cand_insert(c, ((uint32_t)dist << 16) | (uint32_t)p, idx, oct, bin);
        }
    }
    return n;
}

// ---- grid: sorted (cell << 16 | idx) keys + CSR cell starts, one workgroup per slot
__global__ __launch_bounds__(1024) void track_grid_kernel(Slots S, float4 *rec_out, int *cell_start) {
    extern __shared__ uint32_t sk[];
    const int s = blockIdx.x, tid = threadIdx.x;
    const FrameDev &f = S.fr[s];
    const int n = f.n, sc = S.sort_cap;
    const long long kb = (long long)s * S.cap_kp;
    for (int i = tid; i < sc; i += 1024) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n) {
            const orbx_kp k = S.kun[kb + i];
            const int px = (int)roundf((k.x - f.min_x) * f.inv_w);   // PosInGrid (Frame.cc:682-698)
            const int py = (int)roundf((k.y - f.min_y) * f.inv_h);
            if (!(px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS))
                key = ((uint32_t)(px * GRID_ROWS + py) << 16) | (uint32_t)i;
        }
        sk[i] = key;
    }
    __syncthreads();
    for (int k = 2; k <= sc; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < sc; i += 1024) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t x = sk[i], y = sk[ixj];
                    const bool asc = (i & k) == 0;
                    if (asc ? (x > y) : (x < y)) { sk[i] = y; sk[ixj] = x; }
                }
            }
            __syncthreads();
        }
    float4 *ro = rec_out + (long long)s * sc;
    for (int i = tid; i < sc; i += 1024) {
        const uint32_t key = sk[i];
        float4 g = make_float4(0.f, 0.f, -1.f, __uint_as_float(0xFFFFFFFFu));
        if (key != 0xFFFFFFFFu) {
            const int idx = (int)(key & 0xFFFFu);
            const orbx_kp k = S.kun[kb + idx];
            const uint32_t pk = (uint32_t)idx | ((uint32_t)(k.octave & 0xFF) << 16) |
                                ((uint32_t)(S.blocked[kb + idx] ? 1 : 0) << 24);
            g = make_float4(k.x, k.y, S.uR[kb + idx], __uint_as_float(pk));
        }
        ro[i] = g;
    }
    int *cso = cell_start + (long long)s * (NCELL + 1);
    for (int c = tid; c <= NCELL; c += 1024) {   // lower_bound(c << 16)
        const uint32_t v = (uint32_t)c << 16;
        int lo = 0, hi = sc;
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (sk[m] < v) lo = m + 1; else hi = m;
        }
        cso[c] = lo;
    }
}

struct ViewOut {
    uint8_t *in_view;
    float *px, *py, *pxr, *vcos;
    int *level;
};

// ---- SearchLocalPoints candidates: one thread per (slot, map point)
__global__ __launch_bounds__(256) void track_local_cand_kernel(Slots S, float cos_limit, float th, ViewOut V,
                                                               Cand *cand, int *ncand) {
    const int m = blockIdx.x * 256 + threadIdx.x, s = blockIdx.y;
    const FrameDev &f = S.fr[s];
    if (m >= f.n_mp) return;
    const long long mb = (long long)s * S.cap_mp + m;
    const uint8_t flags = S.mflags[mb];
    uint8_t inv = 0;
    float u = 0, v = 0, uxr = 0, viewCos = 0;
    int nScale = 0;
    if (!(flags & (ORBT_MP_BAD | ORBT_MP_IN_FRAME))) {
        // Frame::isInFrustum (Frame.cc:490-578)
        const float *P = S.Xw + mb * 3;
        float Pc[3];
        mat_rx_t(f.Tcw, P, Pc);
        bool ok = !(Pc[2] < 0.0f);
        if (ok) {
            const float invz = 1.0f / Pc[2];
            u = f.fx * Pc[0] * invz + f.cx;
            v = f.fy * Pc[1] * invz + f.cy;
            ok = !(u < f.min_x || u > f.max_x) && !(v < f.min_y || v > f.max_y);
            if (ok) {
                const float maxDistance = 1.2f * S.maxd[mb], minDistance = 0.8f * S.mind[mb];
                const float PO[3] = {P[0] - f.Ow[0], P[1] - f.Ow[1], P[2] - f.Ow[2]};
                double ss = 0;
                for (int k = 0; k < 3; k++) { const double t = PO[k]; ss = ss + t * t; }
                const float dist = (float)sqrt(ss);                       // cv::norm
                ok = !(dist < minDistance || dist > maxDistance);
                if (ok) {
                    const float *Pn = S.nrm + mb * 3;
                    double dot = 0;
                    for (int k = 0; k < 3; k++) dot = dot + (double)PO[k] * (double)Pn[k];   // Mat::dot
                    viewCos = (float)(dot / (double)dist);
                    ok = !(viewCos < cos_limit);
                    if (ok) {
                        const float ratio = S.maxd[mb] / dist;            // PredictScale
                        nScale = (int)ceilf(glibc_logf(ratio) / f.log_scale);
                        if (nScale < 0) nScale = 0;
                        else if (nScale >= f.nlevels) nScale = f.nlevels - 1;
                        uxr = u - f.mbf * invz;
                        inv = 1;
                    }
                }
            }
        }
    }
    if (V.in_view) V.in_view[mb] = inv;
    if (V.px) V.px[mb] = inv ? u : 0.f;
    if (V.py) V.py[mb] = inv ? v : 0.f;
    if (V.pxr) V.pxr[mb] = inv ? uxr : 0.f;
    if (V.vcos) V.vcos[mb] = inv ? viewCos : 0.f;
    if (V.level) V.level[mb] = inv ? nScale : 0;
    Cand c;
    int nc = 0;
    if (inv) {
        // ORBmatcher::SearchByProjection(F, vpMapPoints, th), ORBmatcher.cc:78-176
        float r = (viewCos > 0.998) ? 2.5f : 4.0f;                        // RadiusByViewingCos
        if (th != 1.0f) r *= th;
        const float rs = r * f.scale[nScale];
        nc = scan_window<true>(S, s, f, u, v, rs, nScale - 1, nScale, S.mdesc + mb * 32, uxr, rs, nullptr, 0.f, c);
    } else {
#pragma unroll
        for (int k = 0; k < TOPK; k++) { c.key[k] = 0xFFFFFFFFu; c.idx[k] = 0; c.oct[k] = -1; c.bin[k] = -1; }
    }
    cand[mb] = c;
    ncand[mb] = inv ? nc : -1;
}

// ---- claim replay, one wave per slot, speculative 64-query windows.
// Each lane decides one query of the window against the claim set as of the window start
// and records the candidates it examined (its kept entries up to the decision). An earlier
// lane that claims -- with a map point that has observations -- a keypoint a later lane
// examined invalidates that later lane and everything after it; the valid prefix is
// committed and the window restarts at the first invalid lane. A lane whose kept entries
// are exhausted by claims (fallback) is a window barrier, rescanned exactly with the claims.
// Result = the reference's strictly sequential order.
constexpr int kNoTag = 1 << 30;

__device__ inline float local_radius(float vc, int lvl, float th, const FrameDev &f) {
    float r = (vc > 0.998) ? 2.5f : 4.0f;                            // RadiusByViewingCos
    if (th != 1.0f) r *= th;
    return r * f.scale[lvl];
}

__global__ __launch_bounds__(64) void track_local_resolve_kernel(Slots S, float th, float nnratio, ViewOut V,
                                                                 const Cand *cand, const int *ncand, int *owner,
                                                                 int *nmatch) {
    extern __shared__ uint8_t lds[];
    uint8_t *claimed = lds;                                 // [cap_kp]
    int *tag = (int *)(lds + ((S.cap_kp + 15) & ~15));       // [cap_kp] lowest claiming lane
    const int s = blockIdx.x, lane = threadIdx.x;
    const FrameDev &f = S.fr[s];
    const long long kb = (long long)s * S.cap_kp, mb0 = (long long)s * S.cap_mp;
    for (int i = lane; i < f.n; i += 64) { claimed[i] = S.blocked[kb + i]; tag[i] = kNoTag; owner[kb + i] = -1; }
    __syncthreads();
    int nm = 0, base = 0;
    while (base < f.n_mp) {
        const int q = base + lane;
        const bool live = q < f.n_mp;
        Cand c;
        int nc = -1;
        uint8_t fl = 0;
        if (live) { c = cand[mb0 + q]; nc = ncand[mb0 + q]; fl = S.mflags[mb0 + q]; }
        Pick pk;
        pk.found = 0; pk.last_ex = -1; pk.key0 = pk.key1 = 0xFFFFFFFFu; pk.idx0 = 0; pk.oct0 = pk.oct1 = -1;
        if (nc > 0) pk = pick_unclaimed(c, claimed, 2);
        const bool fallback = nc > TOPK && pk.found < 2;
        bool accept = false;
        if (nc > 0 && !fallback && pk.found >= 1) {
            const int bestDist = (int)(pk.key0 >> 16), bestLevel = pk.oct0;
            const int bestDist2 = pk.found >= 2 ? (int)(pk.key1 >> 16) : 256, bestLevel2 = pk.found >= 2 ? pk.oct1 : -1;
            accept = bestDist <= TH_HIGH && !(bestLevel == bestLevel2 && (float)bestDist > nnratio * (float)bestDist2);
        }
        const bool obs = (fl & ORBT_MP_HAS_OBS) != 0;
        const int idx = pk.idx0;
        if (accept && obs) atomicMin(&tag[idx], lane);
        __syncthreads();
        const bool conflict = nc > 0 && examined_conflict(c, pk.last_ex, tag, lane);
        const unsigned long long stop = __ballot(live && (conflict || fallback));
        const int cut = stop ? __ffsll((long long)stop) - 1 : 64;
        __syncthreads();
        if (accept && obs) tag[idx] = kNoTag;
        const bool commit = accept && lane < cut;
        if (commit) {
            atomicMax(&owner[kb + idx], q);   // later map points overwrite observation-less owners
            if (obs) claimed[idx] = 1;
        }
        nm += __popcll(__ballot(commit));
        __syncthreads();
        if (cut < 64 && base + cut < f.n_mp && ((stop >> cut) & 1)) {
            // the barrier lane: conflict -> re-decide in the next window; fallback -> rescan now
            bool is_fb = __shfl(fallback ? 1 : 0, cut) != 0;
            if (is_fb) {
                if (lane == 0) {
                    const int qq = base + cut;
                    const long long mb = mb0 + qq;
                    const int lvl = V.level[mb];
                    const float rs = local_radius(V.vcos[mb], lvl, th, f);
                    Cand full;
                    scan_window<true>(S, s, f, V.px[mb], V.py[mb], rs, lvl - 1, lvl, S.mdesc + mb * 32, V.pxr[mb], rs,
                                      claimed, 0.f, full);
                    if (full.key[0] != 0xFFFFFFFFu) {
                        const int bd = (int)(full.key[0] >> 16), bl = full.oct[0];
                        const int bd2 = full.key[1] != 0xFFFFFFFFu ? (int)(full.key[1] >> 16) : 256;
                        const int bl2 = full.key[1] != 0xFFFFFFFFu ? full.oct[1] : -1;
                        if (bd <= TH_HIGH && !(bl == bl2 && (float)bd > nnratio * (float)bd2)) {
                            const int id = full.idx[0];
                            owner[kb + id] = qq;
                            if (S.mflags[mb] & ORBT_MP_HAS_OBS) claimed[id] = 1;
                            nm++;
                        }
                    }
                }
                nm = __shfl(nm, 0);
                __syncthreads();
                base += cut + 1;
            } else {
                base += cut;
            }
        } else {
            base += 64;
        }
    }
    if (lane == 0) nmatch[s] = nm;
}

constexpr int kModeMotion = 0, kModeReloc = 1, kModeSim3 = 2;

// ---- relocalisation query of keyframe keypoint i (ORBmatcher.cc:1944-2019): map point not bad
// and not in sAlreadyFound, projection without a depth-sign test, scale-invariance gate,
// PredictScale(dist3D, &CurrentFrame), window at levels [lvl - 1, lvl + 1], no stereo gate
__device__ int reloc_query(const Slots &S, int s, const FrameDev &f, int i, float th, const uint8_t *claimed,
                           Cand &c) {
#pragma unroll
    for (int k = 0; k < TOPK; k++) { c.key[k] = 0xFFFFFFFFu; c.idx[k] = 0; c.oct[k] = -1; c.bin[k] = -1; }
    const long long lb = (long long)s * S.cap_kp + i;
    const int m = S.last_mp[lb];
    if (m < 0) return -1;
    const long long mb = (long long)s * S.cap_mp + m;
    if (S.mflags[mb] & (ORBT_MP_BAD | ORBT_MP_FOUND)) return -1;
    const float *P = S.Xw + mb * 3;
    float x3Dc[3];
    mat_rx_t(f.Tcw, P, x3Dc);
    const float invzc = (float)(1.0 / (double)x3Dc[2]);
    const float u = f.fx * x3Dc[0] * invzc + f.cx;
    const float v = f.fy * x3Dc[1] * invzc + f.cy;
    if (u < f.min_x || u > f.max_x || v < f.min_y || v > f.max_y) return 0;
    const float PO[3] = {P[0] - f.Ow[0], P[1] - f.Ow[1], P[2] - f.Ow[2]};
    double ss = 0;
    for (int k = 0; k < 3; k++) { const double t = PO[k]; ss = ss + t * t; }
    const float dist3D = (float)sqrt(ss);                                   // cv::norm
    const float maxDistance = 1.2f * S.maxd[mb], minDistance = 0.8f * S.mind[mb];
    if (dist3D < minDistance || dist3D > maxDistance) return 0;
    int lvl = (int)ceilf(glibc_logf(S.maxd[mb] / dist3D) / f.log_scale);    // PredictScale
    if (lvl < 0) lvl = 0;
    else if (lvl >= f.nlevels) lvl = f.nlevels - 1;
    const float radius = th * f.scale[lvl];
    return scan_window<false>(S, s, f, u, v, radius, lvl - 1, lvl + 1, S.mdesc + mb * 32, 0.f, INFINITY, claimed,
                              S.lkun[lb].angle, c);
}

// ---- loop-closing query of map point m (ORBmatcher.cc:457-551): not bad and not already in
// vpMatched (ORBT_MP_FOUND), depth sign test, KeyFrame::IsInImage, scale-invariance and
// viewing-angle (PO.Pn >= 0.5 dist) gates, PredictScale(dist, pKF), KeyFrame::GetFeaturesInArea
// window then levels [lvl - 1, lvl]; `f` holds pKF with the unscaled Sim3 pose [Rcw | tcw], Ow
__device__ int sim3_query(const Slots &S, int s, const FrameDev &f, int m, float th, const uint8_t *claimed,
                          Cand &c) {
#pragma unroll
    for (int k = 0; k < TOPK; k++) { c.key[k] = 0xFFFFFFFFu; c.idx[k] = 0; c.oct[k] = -1; c.bin[k] = -1; }
    const long long mb = (long long)s * S.cap_mp + m;
    if (S.mflags[mb] & (ORBT_MP_BAD | ORBT_MP_FOUND)) return -1;
    const float *P = S.Xw + mb * 3;
    float p3Dc[3];
    mat_rx_t(f.Tcw, P, p3Dc);
    if (p3Dc[2] < 0.0f) return 0;
    const float invz = 1 / p3Dc[2];
    const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
    const float u = f.fx * x + f.cx, v = f.fy * y + f.cy;
    if (!(u >= f.min_x && u < f.max_x && v >= f.min_y && v < f.max_y)) return 0;   // KeyFrame::IsInImage
    const float maxDistance = 1.2f * S.maxd[mb], minDistance = 0.8f * S.mind[mb];
    const float PO[3] = {P[0] - f.Ow[0], P[1] - f.Ow[1], P[2] - f.Ow[2]};
    double ss = 0;
    for (int k = 0; k < 3; k++) { const double t = PO[k]; ss = ss + t * t; }
    const float dist = (float)sqrt(ss);                                      // cv::norm
    if (dist < minDistance || dist > maxDistance) return 0;
    const float *Pn = S.nrm + mb * 3;
    double dot = 0;
    for (int k = 0; k < 3; k++) dot = dot + (double)PO[k] * (double)Pn[k];   // Mat::dot
    if (dot < 0.5 * (double)dist) return 0;
    int lvl = (int)ceilf(glibc_logf(S.maxd[mb] / dist) / f.log_scale);       // PredictScale(dist, pKF)
    if (lvl < 0) lvl = 0;
    else if (lvl >= f.nlevels) lvl = f.nlevels - 1;
    const float radius = th * f.scale[lvl];
    return scan_window<false>(S, s, f, u, v, radius, lvl - 1, lvl, S.mdesc + mb * 32, 0.f, INFINITY, claimed, 0.f, c);
}

// ---- SearchByProjection(CurrentFrame, LastFrame) query of last keypoint i (ORBmatcher.cc:1786-1870);
// `claimed` != null adds the claim filter (resolve fallback). Returns -1 if not projected.
__device__ int frame_query(const Slots &S, int s, const FrameDev &f, int i, float th, int mono,
                           const uint8_t *claimed, Cand &c, int mode = kModeMotion) {
    if (mode == kModeReloc) return reloc_query(S, s, f, i, th, claimed, c);
    if (mode == kModeSim3) return sim3_query(S, s, f, i, th, claimed, c);
#pragma unroll
    for (int k = 0; k < TOPK; k++) { c.key[k] = 0xFFFFFFFFu; c.idx[k] = 0; c.oct[k] = -1; c.bin[k] = -1; }
    const long long lb = (long long)s * S.cap_kp + i;
    const int m = S.last_mp[lb];
    if (m < 0 || S.last_out[lb]) return -1;
    // twc = -Rcw^T tcw; tlc = Rlw twc + tlw (ORBmatcher.cc:1757-1771)
    float twc[3];
    for (int k = 0; k < 3; k++) {
        float t = f.Tcw[k] * f.Tcw[3];
        t = t + f.Tcw[4 + k] * f.Tcw[7];
        t = t + f.Tcw[8 + k] * f.Tcw[11];
        twc[k] = -t;
    }
    float tlc[3];
    mat_rx_t(f.lTcw, twc, tlc);
    const bool bForward = tlc[2] > f.mb && !mono;
    const bool bBackward = -tlc[2] > f.mb && !mono;
    const long long mb = (long long)s * S.cap_mp + m;
    float x3Dc[3];
    mat_rx_t(f.Tcw, S.Xw + mb * 3, x3Dc);
    const float invzc = (float)(1.0 / (double)x3Dc[2]);
    if (invzc < 0) return 0;
    const float u = f.fx * x3Dc[0] * invzc + f.cx;
    const float v = f.fy * x3Dc[1] * invzc + f.cy;
    if (u < f.min_x || u > f.max_x || v < f.min_y || v > f.max_y) return 0;
    const orbx_kp lk = S.lkun[lb];
    const int nLastOctave = lk.octave;
    const float radius = th * f.scale[nLastOctave];
    int minL, maxL;
    if (bForward) { minL = nLastOctave; maxL = -1; }
    else if (bBackward) { minL = 0; maxL = nLastOctave; }
    else { minL = nLastOctave - 1; maxL = nLastOctave + 1; }
    const float ur = u - f.mbf * invzc;
    return scan_window<false>(S, s, f, u, v, radius, minL, maxL, S.mdesc + mb * 32, ur, radius, claimed, lk.angle, c);
}

// one thread per (slot, last keypoint)
__global__ __launch_bounds__(256) void track_frame_cand_kernel(Slots S, float th, int mono, int mode, Cand *cand,
                                                               int *ncand) {
    const int i = blockIdx.x * 256 + threadIdx.x, s = blockIdx.y;
    const FrameDev &f = S.fr[s];
    if (i >= (mode == kModeSim3 ? f.n_mp : f.n_last)) return;   // queries: last keypoints / map points
    Cand c;
    const int nc = frame_query(S, s, f, i, th, mono, nullptr, c, mode);
    const long long lb = (long long)s * (mode == kModeSim3 ? S.cap_mp : S.cap_kp) + i;
    cand[lb] = c;
    ncand[lb] = nc;
}

// mode kModeMotion: accept <= TH_HIGH, a claim blocks later points only if the claiming point
// has observations; kModeReloc: accept <= ORBdist (max_dist), every claim blocks (:2007-2008);
// kModeSim3: queries are the map points themselves, accept <= TH_LOW, every claim blocks (:552-555)
__global__ __launch_bounds__(64) void track_frame_resolve_kernel(Slots S, float th, int mono, int check_ori,
                                                                 int mode, int max_dist,
                                                                 const Cand *cand, const int *ncand, int *owner,
                                                                 int *nmatch, int *hist_idx, int8_t *hist_bin) {
    extern __shared__ uint8_t lds[];
    uint8_t *claimed = lds;                                 // [cap_kp]
    int *tag = (int *)(lds + ((S.cap_kp + 15) & ~15));       // [cap_kp]
    int *wl = tag + S.cap_kp;                                // [cap_kp] last committed writer lane
    __shared__ int counts[HISTO_LENGTH];
    const int s = blockIdx.x, lane = threadIdx.x;
    const FrameDev &f = S.fr[s];
    const long long kb = (long long)s * S.cap_kp, mb0 = (long long)s * S.cap_mp;
    for (int i = lane; i < f.n; i += 64) {
        claimed[i] = S.blocked[kb + i]; tag[i] = kNoTag; wl[i] = -1; owner[kb + i] = -1;
    }
    if (lane < HISTO_LENGTH) counts[lane] = 0;
    __syncthreads();
    int nm = 0, nh = 0, base = 0;
    int *HI = hist_idx + kb;
    int8_t *HB = hist_bin + kb;
    const bool sim3 = mode == kModeSim3;
    const int nq = sim3 ? f.n_mp : f.n_last;
    const long long qb = sim3 ? mb0 : kb;   // query record base
    while (base < nq) {
        const int q = base + lane;
        const bool live = q < nq;
        Cand c;
        int nc = -1, m = -1;
        if (live) { c = cand[qb + q]; nc = ncand[qb + q]; m = sim3 ? q : S.last_mp[kb + q]; }
        Pick pk;
        pk.found = 0; pk.last_ex = -1; pk.key0 = 0xFFFFFFFFu; pk.idx0 = 0; pk.bin0 = -1;
        if (nc > 0) pk = pick_unclaimed(c, claimed, 1);
        const bool fallback = nc > TOPK && pk.found < 1;
        const bool accept = nc > 0 && !fallback && pk.found >= 1 && (int)(pk.key0 >> 16) <= max_dist;
        const bool obs = m >= 0 && (mode != kModeMotion || (S.mflags[mb0 + m] & ORBT_MP_HAS_OBS) != 0);
        const int idx = pk.idx0;
        if (accept && obs) atomicMin(&tag[idx], lane);
        __syncthreads();
        const bool conflict = nc > 0 && examined_conflict(c, pk.last_ex, tag, lane);
        const unsigned long long stop = __ballot(live && (conflict || fallback));
        const int cut = stop ? __ffsll((long long)stop) - 1 : 64;
        __syncthreads();
        if (accept && obs) tag[idx] = kNoTag;
        const bool commit = accept && lane < cut;
        if (commit) {
            // CurrentFrame.mvpMapPoints[bestIdx2] = pMP: the last committed lane wins
            atomicMax(&wl[idx], lane);
            if (obs) claimed[idx] = 1;
        }
        __syncthreads();
        if (commit && wl[idx] == lane) owner[kb + idx] = m;
        __syncthreads();
        if (commit) wl[idx] = -1;
        const unsigned long long cm = __ballot(commit);
        if (commit && check_ori) {   // rotHist push order = query order
            const int slot = nh + __popcll(cm & ((1ull << lane) - 1));
            HI[slot] = idx;
            HB[slot] = (int8_t)pk.bin0;
            atomicAdd(&counts[pk.bin0], 1);
        }
        nm += __popcll(cm);
        if (check_ori) nh += __popcll(cm);
        __syncthreads();
        if (cut < 64 && base + cut < nq && ((stop >> cut) & 1)) {
            const bool is_fb = __shfl(fallback ? 1 : 0, cut) != 0;
            if (is_fb) {
                if (lane == 0) {
                    const int qq = base + cut;
                    Cand full;
                    frame_query(S, s, f, qq, th, mono, claimed, full, mode);
                    if (full.key[0] != 0xFFFFFFFFu && (int)(full.key[0] >> 16) <= max_dist) {
                        const int id = full.idx[0], mm = sim3 ? qq : S.last_mp[kb + qq];
                        owner[kb + id] = mm;
                        if (mode != kModeMotion || (S.mflags[mb0 + mm] & ORBT_MP_HAS_OBS)) claimed[id] = 1;
                        nm++;
                        if (check_ori) {
                            HI[nh] = id;
                            HB[nh] = full.bin[0];
                            counts[full.bin[0]]++;
                            nh++;
                        }
                    }
                }
                nm = __shfl(nm, 0);
                nh = __shfl(nh, 0);
                __syncthreads();
                base += cut + 1;
            } else {
                base += cut;
            }
        } else {
            base += 64;
        }
    }
    if (check_ori) {
        __shared__ int top[3];
        if (lane == 0) {   // ComputeThreeMaxima (ORBmatcher.cc:2076-2118)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO_LENGTH; i++) {
                const int v = counts[i];
                if (v > max1) { max3 = max2; max2 = max1; max1 = v; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (v > max2) { max3 = max2; max2 = v; ind3 = ind2; ind2 = i; }
                else if (v > max3) { max3 = v; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            top[0] = ind1; top[1] = ind2; top[2] = ind3;
        }
        __syncthreads();
        int removed = 0;
        for (int k = lane; k < nh; k += 64) {   // mvpMapPoints[rotHist[bin][j]] = NULL outside the top three
            const int bb = HB[k];
            if (bb == top[0] || bb == top[1] || bb == top[2]) continue;
            owner[kb + HI[k]] = -2;
            removed++;
        }
        for (int off = 32; off > 0; off >>= 1) removed += __shfl_xor(removed, off);
        nm -= removed;
    }
    if (lane == 0) nmatch[s] = nm;
}

// ---- ORBmatcher::Fuse(pKF, vpMapPoints, th) search half (ORBmatcher.cc:1139-1240): one thread
// per (slot, map point); no claims -- every point's best keypoint is independent
// sim3 != 0: LoopClosing's Fuse(pKF, Scw, ...) (ORBmatcher.cc:1347-1433): Sim3-derived pose in the
// slot, invz = 1.0 / z in double, no chi2 gate, bestDist starting at INT_MAX
__global__ __launch_bounds__(256) void track_fuse_kernel(Slots S, float th, int sim3, int *best_idx, int *best_dist) {
    const int m = blockIdx.x * 256 + threadIdx.x, s = blockIdx.y;
    const FrameDev &f = S.fr[s];
    if (m >= f.n_mp) return;
    const long long mb = (long long)s * S.cap_mp + m;
    int bestIdx = -1, bestDist = sim3 ? INT_MAX : 256;
    if (!(S.mflags[mb] & (ORBT_MP_BAD | ORBT_MP_IN_FRAME))) {   // isBad() || IsInKeyFrame(pKF)
        const float *P = S.Xw + mb * 3;
        float p3Dc[3];
        mat_rx_t(f.Tcw, P, p3Dc);
        bool ok = !(p3Dc[2] < 0.0f);
        float u = 0, v = 0, ur = 0;
        int lvl = 0;
        if (ok) {
            const float invz = sim3 ? (float)(1.0 / (double)p3Dc[2]) : 1 / p3Dc[2];
            const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
            u = f.fx * x + f.cx;
            v = f.fy * y + f.cy;
            ok = u >= f.min_x && u < f.max_x && v >= f.min_y && v < f.max_y;   // KeyFrame::IsInImage
            ur = u - f.mbf * invz;
        }
        if (ok) {
            const float maxDistance = 1.2f * S.maxd[mb], minDistance = 0.8f * S.mind[mb];
            const float PO[3] = {P[0] - f.Ow[0], P[1] - f.Ow[1], P[2] - f.Ow[2]};
            double ss = 0;
            for (int k = 0; k < 3; k++) { const double t = PO[k]; ss = ss + t * t; }
            const float dist3D = (float)sqrt(ss);
            ok = !(dist3D < minDistance || dist3D > maxDistance);
            if (ok) {
                const float *Pn = S.nrm + mb * 3;
                double dot = 0;
                for (int k = 0; k < 3; k++) dot = dot + (double)PO[k] * (double)Pn[k];
                ok = !(dot < 0.5 * (double)dist3D);
                if (ok) {   // MapPoint::PredictScale(dist3D, pKF)
                    const float ratio = S.maxd[mb] / dist3D;
                    lvl = (int)ceilf(glibc_logf(ratio) / f.log_scale);
                    if (lvl < 0) lvl = 0;
                    else if (lvl >= f.nlevels) lvl = f.nlevels - 1;
                }
            }
        }
        int cx0, cx1, cy0, cy1;
        const float radius = th * f.scale[lvl];
        if (ok && grid_window(f, u, v, radius, cx0, cx1, cy0, cy1)) {
            const float4 *rec = S.grec + (long long)s * S.sort_cap;
            const int *cs = S.cell_start + (long long)s * (NCELL + 1);
            const long long kb = (long long)s * S.cap_kp;
            const uint8_t *dMP = S.mdesc + mb * 32;
            for (int ix = cx0; ix <= cx1; ix++) {
                const int a = cs[ix * GRID_ROWS + cy0], b = cs[ix * GRID_ROWS + cy1 + 1];
                for (int t = a; t < b; t++) {
                    const float4 g = rec[t];
                    const float distx = g.x - u, disty = g.y - v;
                    if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
                    const uint32_t pk = __float_as_uint(g.w);
                    const int idx = (int)(pk & 0xFFFFu), kpLevel = (int)((pk >> 16) & 0xFF);
                    if (kpLevel < lvl - 1 || kpLevel > lvl) continue;
                    const float ex = u - g.x, ey = v - g.y;
                    if (sim3) {
                    } else if (g.z >= 0) {
                        const float er = ur - g.z;
                        const float e2 = ex * ex + ey * ey + er * er;
                        if ((double)(e2 * f.inv_s2[kpLevel]) > 7.8) continue;
                    } else {
                        const float e2 = ex * ex + ey * ey;
                        if ((double)(e2 * f.inv_s2[kpLevel]) > 5.99) continue;
                    }
                    const int dist = hamming32(dMP, S.desc + (kb + idx) * 32);
                    if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
                }
            }
        }
    }
    best_idx[mb] = bestIdx;
    best_dist[mb] = bestDist;
}

// ---- ORBmatcher::SearchBySim3, one direction (ORBmatcher.cc:1530-1618 / 1623-1700): thread per
// (slot, source keypoint i); the slot's frame is the target keyframe, `last` the source keyframe
// with its map points and vbAlreadyMatched (last_out). out[i] = vnMatch[i] (-1 = none).
__global__ __launch_bounds__(256) void track_sim3_match_kernel(Slots S, float th, int *out) {
    const int i = blockIdx.x * 256 + threadIdx.x, s = blockIdx.y;
    const FrameDev &f = S.fr[s];
    if (i >= f.n_last) return;
    const long long lb = (long long)s * S.cap_kp + i;
    const int m = S.last_mp[lb];
    int vn = -1;
    if (m >= 0 && !S.last_out[lb]) {
        const long long mb = (long long)s * S.cap_mp + m;
        if (!(S.mflags[mb] & ORBT_MP_BAD)) {
            const float *P = S.Xw + mb * 3;
            float pc1[3], pc2[3];
            mat_rx_t(f.lTcw, P, pc1);
            mat_rx_t(f.sT, pc1, pc2);
            bool ok = !(pc2[2] < 0.0f);
            float u = 0, v = 0, dist3D = 0;
            if (ok) {
                const float invz = (float)(1.0 / (double)pc2[2]);
                const float x = pc2[0] * invz, y = pc2[1] * invz;
                u = f.pfx * x + f.pcx;
                v = f.pfy * y + f.pcy;
                ok = u >= f.min_x && u < f.max_x && v >= f.min_y && v < f.max_y;   // KeyFrame::IsInImage
            }
            if (ok) {
                double ss = 0;
                for (int k = 0; k < 3; k++) { const double t = pc2[k]; ss = ss + t * t; }
                dist3D = (float)sqrt(ss);                                          // cv::norm(p3Dc2)
                ok = !(dist3D < 0.8f * S.mind[mb] || dist3D > 1.2f * S.maxd[mb]);
            }
            int cx0, cx1, cy0, cy1;
            int lvl = 0;
            if (ok) {
                lvl = (int)ceilf(glibc_logf(S.maxd[mb] / dist3D) / f.log_scale);   // PredictScale(dist3D, target)
                if (lvl < 0) lvl = 0;
                else if (lvl >= f.nlevels) lvl = f.nlevels - 1;
            }
            const float radius = th * f.scale[lvl];
            if (ok && grid_window(f, u, v, radius, cx0, cx1, cy0, cy1)) {
                const float4 *rec = S.grec + (long long)s * S.sort_cap;
                const int *cs = S.cell_start + (long long)s * (NCELL + 1);
                const long long kb = (long long)s * S.cap_kp;
                const uint8_t *dMP = S.mdesc + mb * 32;
                int bestDist = INT_MAX, bestIdx = -1;
                for (int ix = cx0; ix <= cx1; ix++) {
                    const int a = cs[ix * GRID_ROWS + cy0], b = cs[ix * GRID_ROWS + cy1 + 1];
                    for (int t = a; t < b; t++) {
                        const float4 g = rec[t];
                        if (!(fabsf(g.x - u) < radius && fabsf(g.y - v) < radius)) continue;
                        const uint32_t pk = __float_as_uint(g.w);
                        const int idx = (int)(pk & 0xFFFFu), o = (int)((pk >> 16) & 0xFF);
                        if (o < lvl - 1 || o > lvl) continue;
                        const int d = hamming32(dMP, S.desc + (kb + idx) * 32);
                        if (d < bestDist) { bestDist = d; bestIdx = idx; }
                    }
                }
                if (bestDist <= TH_HIGH) vn = bestIdx;
            }
        }
    }
    out[lb] = vn;
}

}  // namespace orbtrack

using namespace orbtrack;

struct orbt_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;          // end of the last run (fetch waits on it only)
    hipStream_t done_stream = nullptr;
    int nslots = 0, cap_kp = 0, cap_mp = 0, sort_cap = 0;
    DevBuf fr, kun, uR, desc, blocked, keys, cell_start, lkun, last_mp, last_out;
    DevBuf Xw, nrm, mind, maxd, mdesc, mflags;
    DevBuf in_view, px, py, pxr, vcos, level, cand, ncand, owner, nmatch, hist_idx, hist_bin, fuse_idx, fuse_dist;
    std::vector<FrameDev> hfr;
};

namespace {

Slots make_slots(orbt_engine *e) {
    Slots S;
    S.fr = e->fr.as<FrameDev>();
    S.kun = e->kun.as<orbx_kp>(); S.uR = e->uR.as<float>(); S.desc = e->desc.as<uint8_t>();
    S.blocked = e->blocked.as<uint8_t>(); S.grec = e->keys.as<float4>(); S.cell_start = e->cell_start.as<int>();
    S.lkun = e->lkun.as<orbx_kp>(); S.last_mp = e->last_mp.as<int>(); S.last_out = e->last_out.as<uint8_t>();
    S.Xw = e->Xw.as<float>(); S.nrm = e->nrm.as<float>(); S.mind = e->mind.as<float>(); S.maxd = e->maxd.as<float>();
    S.mdesc = e->mdesc.as<uint8_t>(); S.mflags = e->mflags.as<uint8_t>();
    S.cap_kp = e->cap_kp; S.cap_mp = e->cap_mp; S.sort_cap = e->sort_cap;
    return S;
}

ViewOut make_view(orbt_engine *e) {
    ViewOut V;
    V.in_view = e->in_view.as<uint8_t>(); V.px = e->px.as<float>(); V.py = e->py.as<float>();
    V.pxr = e->pxr.as<float>(); V.vcos = e->vcos.as<float>(); V.level = e->level.as<int>();
    return V;
}

int max_n(orbt_engine *e, int which, int n) {
    int m = 0;
    for (int s = 0; s < n; s++) m = std::max(m, which == 0 ? e->hfr[s].n_mp : e->hfr[s].n_last);
    return m;
}

size_t resolve_lds(const orbt_engine *e) { return ((e->cap_kp + 15) & ~15) + 2 * sizeof(int) * e->cap_kp; }

hipStream_t pick(orbt_engine *e, void *stream) { return stream ? (hipStream_t)stream : e->stream; }

int grid(orbt_engine *e, int n, hipStream_t st) {
    track_grid_kernel<<<n, 1024, sizeof(uint32_t) * e->sort_cap, st>>>(make_slots(e), e->keys.as<float4>(),
                                                                        e->cell_start.as<int>());
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

// LoopClosing's Sim3 pose, unscaled as cv::Mat evaluates it (ORBmatcher.cc:442-446): scw =
// (float)sqrt(row0 . row0) with Mat::dot in double; sRcw / scw, st / scw = convertTo(alpha =
// 1.0 / scw) in float; Ow = -Rcw^T tcw (float gemm)
void sim3_unscale(const float Scw[16], float Tcw[12], float Ow[3]) {
    double d = 0;
    for (int k = 0; k < 3; k++) d += (double)Scw[k] * Scw[k];
    const float scw = (float)std::sqrt(d);
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

void fill_frame(FrameDev &d, const orbt_frame *F) {
    d.n = F->n;
    std::memcpy(d.Tcw, F->Tcw, sizeof d.Tcw);
    std::memcpy(d.Ow, F->Ow, sizeof d.Ow);
    d.fx = F->fx; d.fy = F->fy; d.cx = F->cx; d.cy = F->cy; d.mbf = F->mbf; d.mb = F->mb;
    d.min_x = F->min_x; d.max_x = F->max_x; d.min_y = F->min_y; d.max_y = F->max_y;
    // Frame.cc:183-184 (static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX))
    d.inv_w = (float)GRID_COLS / (F->max_x - F->min_x);
    d.inv_h = (float)GRID_ROWS / (F->max_y - F->min_y);
    d.nlevels = F->nlevels;
    d.log_scale = F->log_scale_factor;
    std::memcpy(d.scale, F->scale_factors, sizeof d.scale);
    std::memcpy(d.inv_s2, F->inv_level_sigma2, sizeof d.inv_s2);
}

}  // namespace

extern "C" {

int orbt_create(orbt_engine **out) {
    if (!out) return ORBX_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORBX_EDEVICE;
    orbt_engine *e = new orbt_engine();
    if (hipGetDevice(&e->device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        !(e->done = make_done_event())) {
        delete e;
        return ORBX_EDEVICE;
    }
    *out = e;
    return ORBX_OK;
}

void orbt_destroy(orbt_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) { (void)hipStreamSynchronize(e->stream); (void)hipStreamDestroy(e->stream); }
    if (e->done) { (void)hipEventSynchronize(e->done); (void)hipEventDestroy(e->done); }
    DevBuf *bufs[] = {&e->fr, &e->kun, &e->uR, &e->desc, &e->blocked, &e->keys, &e->cell_start, &e->lkun, &e->last_mp,
                      &e->last_out, &e->Xw, &e->nrm, &e->mind, &e->maxd, &e->mdesc, &e->mflags, &e->in_view, &e->px,
                      &e->py, &e->pxr, &e->vcos, &e->level, &e->cand, &e->ncand, &e->owner, &e->nmatch, &e->hist_idx,
                      &e->hist_bin, &e->fuse_idx, &e->fuse_dist};
    for (DevBuf *b : bufs) b->release();
    delete e;
}

int orbt_reserve(orbt_engine *e, int n_slots, int cap_kp, int cap_mp) {
    if (!e || n_slots <= 0 || cap_kp < 0 || cap_mp < 0 || cap_kp > kMaxKp) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    cap_kp = std::max(cap_kp, 1);
    cap_mp = std::max(cap_mp, 1);
    int sc = 64;
    while (sc < cap_kp) sc <<= 1;
    const size_t S = (size_t)n_slots, K = (size_t)cap_kp, M = (size_t)cap_mp;
    if (e->fr.ensure(sizeof(FrameDev) * S) || e->kun.ensure(sizeof(orbx_kp) * S * K) || e->uR.ensure(4 * S * K) ||
        e->desc.ensure(32 * S * K) || e->blocked.ensure(S * K) || e->keys.ensure(16 * S * (size_t)sc) ||
        e->cell_start.ensure(4 * S * (NCELL + 1)) || e->lkun.ensure(sizeof(orbx_kp) * S * K) ||
        e->last_mp.ensure(4 * S * K) || e->last_out.ensure(S * K) || e->Xw.ensure(12 * S * M) ||
        e->nrm.ensure(12 * S * M) || e->mind.ensure(4 * S * M) || e->maxd.ensure(4 * S * M) ||
        e->mdesc.ensure(32 * S * M) || e->mflags.ensure(S * M) || e->in_view.ensure(S * M) || e->px.ensure(4 * S * M) ||
        e->py.ensure(4 * S * M) || e->pxr.ensure(4 * S * M) || e->vcos.ensure(4 * S * M) || e->level.ensure(4 * S * M) ||
        e->cand.ensure(sizeof(Cand) * S * std::max(K, M)) || e->ncand.ensure(4 * S * std::max(K, M)) ||
        e->owner.ensure(4 * S * K) || e->nmatch.ensure(4 * S) || e->hist_idx.ensure(4 * S * K) ||
        e->hist_bin.ensure(S * K) || e->fuse_idx.ensure(4 * S * M) || e->fuse_dist.ensure(4 * S * M))
        return ORBX_EDEVICE;
    e->nslots = n_slots;
    e->cap_kp = cap_kp;
    e->cap_mp = cap_mp;
    e->sort_cap = sc;
    e->hfr.assign(n_slots, FrameDev{});
    return ORBX_OK;
}

int orbt_stage(orbt_engine *e, int slot, const orbt_frame *F, const orbt_mappoints *M, const orbt_frame *last,
               const int32_t *last_mp, const uint8_t *last_outlier, const uint8_t *kp_blocked) {
    if (!e || !F || !M || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    if (F->n < 0 || F->n > e->cap_kp || M->n < 0 || M->n > e->cap_mp) return ORBX_ECAP;
    if (last && (last->n < 0 || last->n > e->cap_kp || !last_mp)) return ORBX_EINVAL;
    if (F->nlevels < 1 || F->nlevels > 16) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = e->stream;
    TR_CHK(order_after_done(e, st));   // a run on another stream may still read the slot
    FrameDev &d = e->hfr[slot];
    d = FrameDev{};
    fill_frame(d, F);
    d.n_mp = M->n;
    d.n_last = last ? last->n : 0;
    if (last) std::memcpy(d.lTcw, last->Tcw, sizeof d.lTcw);
    // validate indices the kernels dereference
    for (int i = 0; i < F->n; i++) {
        const int o = F->keys_un[i].octave;
        if (o < 0 || o >= F->nlevels) return ORBX_EINVAL;
    }
    if (last)
        for (int i = 0; i < last->n; i++) {
            if (last_mp[i] >= M->n) return ORBX_EINVAL;
            const int o = last->keys_un[i].octave;
            if (last_mp[i] >= 0 && (o < 0 || o >= F->nlevels)) return ORBX_EINVAL;
        }
    const size_t K = (size_t)e->cap_kp, Mc = (size_t)e->cap_mp, s = (size_t)slot;
    auto up = [&](DevBuf &b, size_t off, const void *src, size_t bytes) -> bool {
        return bytes == 0 || hipMemcpyAsync((char *)b.p + off, src, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
    };
    const int n = F->n, m = M->n;
    bool ok = up(e->fr, sizeof(FrameDev) * s, &d, sizeof(FrameDev)) &&
              up(e->kun, sizeof(orbx_kp) * s * K, F->keys_un, sizeof(orbx_kp) * n) &&
              up(e->uR, 4 * s * K, F->u_right, 4 * (size_t)n) && up(e->desc, 32 * s * K, F->desc, 32 * (size_t)n) &&
              up(e->Xw, 12 * s * Mc, M->Xw, 12 * (size_t)m) && up(e->nrm, 12 * s * Mc, M->normal, 12 * (size_t)m) &&
              up(e->mind, 4 * s * Mc, M->min_dist, 4 * (size_t)m) && up(e->maxd, 4 * s * Mc, M->max_dist, 4 * (size_t)m) &&
              up(e->mdesc, 32 * s * Mc, M->desc, 32 * (size_t)m) && up(e->mflags, s * Mc, M->flags, (size_t)m);
    if (!ok) return ORBX_EDEVICE;
    if (kp_blocked) ok = up(e->blocked, s * K, kp_blocked, (size_t)n);
    else ok = hipMemsetAsync((char *)e->blocked.p + s * K, 0, (size_t)n, st) == hipSuccess;
    if (ok && last) {
        ok = up(e->lkun, sizeof(orbx_kp) * s * K, last->keys_un, sizeof(orbx_kp) * (size_t)last->n) &&
             up(e->last_mp, 4 * s * K, last_mp, 4 * (size_t)last->n);
        if (ok) {
            if (last_outlier) ok = up(e->last_out, s * K, last_outlier, (size_t)last->n);
            else ok = hipMemsetAsync((char *)e->last_out.p + s * K, 0, (size_t)last->n, st) == hipSuccess;
        }
    }
    if (!ok) return ORBX_EDEVICE;
    TR_CHK(hipStreamSynchronize(st));   // host arrays may be freed by the caller on return
    return ORBX_OK;
}

int orbt_run_local_batch(orbt_engine *e, int n_slots, float view_cos_limit, float th, float nnratio, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    if (grid(e, n_slots, st)) return ORBX_EDEVICE;
    const int mm = std::max(1, max_n(e, 0, n_slots));
    track_local_cand_kernel<<<dim3((mm + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e), view_cos_limit, th,
                                                                             make_view(e), e->cand.as<Cand>(),
                                                                             e->ncand.as<int>());
    track_local_resolve_kernel<<<n_slots, 64, resolve_lds(e), st>>>(make_slots(e), th, nnratio, make_view(e),
                                                                e->cand.as<Cand>(), e->ncand.as<int>(),
                                                                e->owner.as<int>(), e->nmatch.as<int>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_run_frame_batch(orbt_engine *e, int n_slots, float th, int mono, int check_ori, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    if (grid(e, n_slots, st)) return ORBX_EDEVICE;
    const int nl = std::max(1, max_n(e, 1, n_slots));
    track_frame_cand_kernel<<<dim3((nl + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e), th, mono, kModeMotion,
                                                                             e->cand.as<Cand>(), e->ncand.as<int>());
    track_frame_resolve_kernel<<<n_slots, 64, resolve_lds(e), st>>>(make_slots(e), th, mono, check_ori, kModeMotion,
                                                                TH_HIGH, e->cand.as<Cand>(),
                                                                e->ncand.as<int>(), e->owner.as<int>(),
                                                                e->nmatch.as<int>(), e->hist_idx.as<int>(),
                                                                e->hist_bin.as<int8_t>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_run_reloc_batch(orbt_engine *e, int n_slots, float th, int orb_dist, int check_ori, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    if (grid(e, n_slots, st)) return ORBX_EDEVICE;
    const int nl = std::max(1, max_n(e, 1, n_slots));
    track_frame_cand_kernel<<<dim3((nl + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e), th, 0, kModeReloc,
                                                                             e->cand.as<Cand>(), e->ncand.as<int>());
    track_frame_resolve_kernel<<<n_slots, 64, resolve_lds(e), st>>>(make_slots(e), th, 0, check_ori, kModeReloc,
                                                                orb_dist, e->cand.as<Cand>(), e->ncand.as<int>(),
                                                                e->owner.as<int>(), e->nmatch.as<int>(),
                                                                e->hist_idx.as<int>(), e->hist_bin.as<int8_t>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_fetch(orbt_engine *e, int slot, orbt_view *view, int32_t *owner, int32_t *nmatches) {
    if (!e || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = e->stream;
    TR_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    const FrameDev &d = e->hfr[slot];
    const size_t K = (size_t)e->cap_kp, M = (size_t)e->cap_mp, s = (size_t)slot, m = (size_t)d.n_mp;
    auto dn = [&](void *dst, const DevBuf &b, size_t off, size_t bytes) -> bool {
        return !dst || bytes == 0 || hipMemcpyAsync(dst, (const char *)b.p + off, bytes, hipMemcpyDeviceToHost, st) == hipSuccess;
    };
    bool ok = dn(owner, e->owner, 4 * s * K, 4 * (size_t)d.n) && dn(nmatches, e->nmatch, 4 * s, 4);
    if (ok && view)
        ok = dn(view->in_view, e->in_view, s * M, m) && dn(view->proj_x, e->px, 4 * s * M, 4 * m) &&
             dn(view->proj_y, e->py, 4 * s * M, 4 * m) && dn(view->proj_xr, e->pxr, 4 * s * M, 4 * m) &&
             dn(view->view_cos, e->vcos, 4 * s * M, 4 * m) && dn(view->level, e->level, 4 * s * M, 4 * m);
    if (!ok) return ORBX_EDEVICE;
    TR_CHK(hipStreamSynchronize(st));
    return ORBX_OK;
}

int orbt_search_local_points(orbt_engine *e, const orbt_frame *F, const orbt_mappoints *M, float view_cos_limit,
                             float th, float nnratio, const uint8_t *kp_blocked, orbt_view *view, int32_t *owner,
                             int32_t *nmatches) {
    if (!e || !F || !M || !owner) return ORBX_EINVAL;
    if (e->nslots < 1 || e->cap_kp < F->n || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(1, e->nslots), std::max(e->cap_kp, F->n), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage(e, 0, F, M, nullptr, nullptr, nullptr, kp_blocked);
    if (rc) return rc;
    rc = orbt_run_local_batch(e, 1, view_cos_limit, th, nnratio, nullptr);
    if (rc) return rc;
    return orbt_fetch(e, 0, view, owner, nmatches);
}

int orbt_search_by_projection_frame(orbt_engine *e, const orbt_frame *cur, const orbt_frame *last,
                                    const int32_t *last_mp, const uint8_t *last_outlier, const orbt_mappoints *M,
                                    float th, int mono, int check_ori, const uint8_t *kp_blocked, int32_t *owner,
                                    int32_t *nmatches) {
    if (!e || !cur || !last || !last_mp || !M || !owner) return ORBX_EINVAL;
    const int need_kp = std::max(cur->n, last->n);
    if (e->nslots < 1 || e->cap_kp < need_kp || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(1, e->nslots), std::max(e->cap_kp, need_kp), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage(e, 0, cur, M, last, last_mp, last_outlier, kp_blocked);
    if (rc) return rc;
    rc = orbt_run_frame_batch(e, 1, th, mono, check_ori, nullptr);
    if (rc) return rc;
    return orbt_fetch(e, 0, nullptr, owner, nmatches);
}

int orbt_search_by_projection_keyframe(orbt_engine *e, const orbt_frame *cur, const orbt_frame *kf,
                                       const int32_t *kf_mp, const orbt_mappoints *M, float th, int orb_dist,
                                       int check_ori, const uint8_t *kp_blocked, int32_t *owner, int32_t *nmatches) {
    if (!e || !cur || !kf || !kf_mp || !M || !owner) return ORBX_EINVAL;
    const int need_kp = std::max(cur->n, kf->n);
    if (e->nslots < 1 || e->cap_kp < need_kp || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(1, e->nslots), std::max(e->cap_kp, need_kp), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage(e, 0, cur, M, kf, kf_mp, nullptr, kp_blocked);
    if (rc) return rc;
    rc = orbt_run_reloc_batch(e, 1, th, orb_dist, check_ori, nullptr);
    if (rc) return rc;
    return orbt_fetch(e, 0, nullptr, owner, nmatches);
}

int orbt_stage_sim3(orbt_engine *e, int slot, const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M,
                    const int32_t *matched) {
    if (!e || !kf || !Scw || !M || !matched || kf->n < 0 || M->n < 0) return ORBX_EINVAL;
    orbt_frame K = *kf;
    sim3_unscale(Scw, K.Tcw, K.Ow);
    std::vector<uint8_t> flags(M->flags, M->flags + M->n), blocked((size_t)kf->n + 1);
    for (auto &f : flags) f &= (uint8_t)~ORBT_MP_FOUND;
    for (int i = 0; i < kf->n; i++) {
        if (matched[i] >= M->n) return ORBX_EINVAL;
        blocked[i] = matched[i] != -1;                          // vpMatched[idx] != NULL
        if (matched[i] >= 0) flags[matched[i]] |= ORBT_MP_FOUND;   // spAlreadyFound
    }
    orbt_mappoints M2 = *M;
    M2.flags = flags.data();
    return orbt_stage(e, slot, &K, &M2, nullptr, nullptr, nullptr, blocked.data());
}

int orbt_run_sim3_batch(orbt_engine *e, int n_slots, int th, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    if (grid(e, n_slots, st)) return ORBX_EDEVICE;
    const int mm = std::max(1, max_n(e, 0, n_slots));
    const float thf = (float)th;
    track_frame_cand_kernel<<<dim3((mm + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e), thf, 0, kModeSim3,
                                                                             e->cand.as<Cand>(), e->ncand.as<int>());
    track_frame_resolve_kernel<<<n_slots, 64, resolve_lds(e), st>>>(make_slots(e), thf, 0, 0, kModeSim3, 50,
                                                                e->cand.as<Cand>(), e->ncand.as<int>(),
                                                                e->owner.as<int>(), e->nmatch.as<int>(),
                                                                e->hist_idx.as<int>(), e->hist_bin.as<int8_t>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_search_by_projection_sim3(orbt_engine *e, const orbt_frame *kf, const float Scw[16],
                                   const orbt_mappoints *M, int th, int32_t *matched, int32_t *nmatches) {
    if (!e || !kf || !Scw || !M || !matched || !nmatches) return ORBX_EINVAL;
    if (e->nslots < 1 || e->cap_kp < kf->n || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(1, e->nslots), std::max(e->cap_kp, kf->n), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage_sim3(e, 0, kf, Scw, M, matched);
    if (rc) return rc;
    rc = orbt_run_sim3_batch(e, 1, th, nullptr);
    if (rc) return rc;
    std::vector<int32_t> owner((size_t)kf->n + 1);
    rc = orbt_fetch(e, 0, nullptr, owner.data(), nmatches);
    if (rc) return rc;
    for (int i = 0; i < kf->n; i++)
        if (owner[i] >= 0) matched[i] = owner[i];   // vpMatched[bestIdx] = pMP
    return ORBX_OK;
}

int orbt_stage_fuse_sim3(orbt_engine *e, int slot, const orbt_frame *kf, const float Scw[16],
                         const orbt_mappoints *M) {
    if (!e || !kf || !Scw || !M) return ORBX_EINVAL;
    orbt_frame K = *kf;
    sim3_unscale(Scw, K.Tcw, K.Ow);
    return orbt_stage(e, slot, &K, M, nullptr, nullptr, nullptr, nullptr);
}

int orbt_run_fuse_sim3_batch(orbt_engine *e, int n_slots, float th, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    if (grid(e, n_slots, st)) return ORBX_EDEVICE;
    const int mm = std::max(1, max_n(e, 0, n_slots));
    track_fuse_kernel<<<dim3((mm + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e), th, 1, e->fuse_idx.as<int>(),
                                                                       e->fuse_dist.as<int>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_fuse_sim3_candidates(orbt_engine *e, const orbt_frame *kf, const float Scw[16], const orbt_mappoints *M,
                              float th, int32_t *best_idx, int32_t *best_dist) {
    if (!e || !kf || !Scw || !M || !best_idx || !best_dist) return ORBX_EINVAL;
    if (e->nslots < 1 || e->cap_kp < kf->n || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(1, e->nslots), std::max(e->cap_kp, kf->n), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage_fuse_sim3(e, 0, kf, Scw, M);
    if (rc) return rc;
    rc = orbt_run_fuse_sim3_batch(e, 1, th, nullptr);
    if (rc) return rc;
    return orbt_fetch_fuse(e, 0, best_idx, best_dist);
}

// SearchBySim3 pair k -> slots 2k (target pKF2, source pKF1) and 2k+1 (target pKF1, source pKF2)
int orbt_stage_search_by_sim3(orbt_engine *e, int pair, const orbt_frame *kf1, const int32_t *kf1_mp,
                              const orbt_frame *kf2, const int32_t *kf2_mp, const orbt_mappoints *M, float s12,
                              const float R12[9], const float t12[3], const int32_t *matches12) {
    if (!e || !kf1 || !kf1_mp || !kf2 || !kf2_mp || !M || !R12 || !t12 || !matches12) return ORBX_EINVAL;
    if (pair < 0 || 2 * pair + 1 >= e->nslots) return ORBX_EINVAL;
    float sR12[9], sR21[9], t21[3];
    for (int k = 0; k < 9; k++) sR12[k] = R12[k] * s12 + 0.0f;             // s12 * R12 (convertTo)
    const float a = (float)(1.0 / (double)s12);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) sR21[3 * i + j] = R12[3 * j + i] * a + 0.0f;   // (1.0 / s12) * R12.t()
    for (int i = 0; i < 3; i++) {                                           // t21 = -sR21 * t12
        float t = sR21[3 * i] * t12[0];
        t = t + sR21[3 * i + 1] * t12[1];
        t = t + sR21[3 * i + 2] * t12[2];
        t21[i] = -t;
    }
    // vbAlreadyMatched1 / 2 (ORBmatcher.cc:1509-1522; GetIndexInKeyFrame = the kf2 keypoint holding it)
    std::vector<uint8_t> am1((size_t)kf1->n + 1, 0), am2((size_t)kf2->n + 1, 0);
    for (int i = 0; i < kf1->n; i++) {
        const int m = matches12[i];
        if (m < 0) continue;
        if (m >= M->n) return ORBX_EINVAL;
        am1[i] = 1;
        for (int j = 0; j < kf2->n; j++)
            if (kf2_mp[j] == m) { am2[j] = 1; break; }
    }
    const orbt_frame *tgt[2] = {kf2, kf1}, *src[2] = {kf1, kf2};
    const int32_t *mps[2] = {kf1_mp, kf2_mp};
    const uint8_t *ams[2] = {am1.data(), am2.data()};
    const float *sRs[2] = {sR21, sR12}, *sts[2] = {t21, t12};
    for (int d = 0; d < 2; d++) {
        const int slot = 2 * pair + d;
        int rc = orbt_stage(e, slot, tgt[d], M, src[d], mps[d], ams[d], nullptr);
        if (rc) return rc;
        FrameDev &fd = e->hfr[slot];
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) fd.sT[4 * r + c] = sRs[d][3 * r + c];
            fd.sT[4 * r + 3] = sts[d][r];
        }
        fd.pfx = kf1->fx; fd.pfy = kf1->fy; fd.pcx = kf1->cx; fd.pcy = kf1->cy;
        TR_CHK(hipMemcpyAsync((char *)e->fr.p + sizeof(FrameDev) * (size_t)slot, &fd, sizeof(FrameDev), hipMemcpyHostToDevice,
                              e->stream));
        TR_CHK(hipStreamSynchronize(e->stream));
    }
    return ORBX_OK;
}

int orbt_run_sim3_match_batch(orbt_engine *e, int n_pairs, float th, void *stream) {
    if (!e || n_pairs <= 0 || 2 * n_pairs > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    const int ns = 2 * n_pairs;
    if (grid(e, ns, st)) return ORBX_EDEVICE;
    const int nl = std::max(1, max_n(e, 1, ns));
    track_sim3_match_kernel<<<dim3((nl + 255) / 256, ns), 256, 0, st>>>(make_slots(e), th, e->owner.as<int>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_fetch_search_by_sim3(orbt_engine *e, int pair, const int32_t *kf2_mp, int32_t *matches12, int32_t *nfound) {
    if (!e || pair < 0 || 2 * pair + 1 >= e->nslots || !kf2_mp || !matches12 || !nfound) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    TR_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    const size_t K = (size_t)e->cap_kp;
    const int N1 = e->hfr[2 * pair].n_last, N2 = e->hfr[2 * pair + 1].n_last;
    std::vector<int32_t> v1((size_t)N1 + 1), v2((size_t)N2 + 1);
    if (N1) TR_CHK(d2h_sync(v1.data(), (char *)e->owner.p + 4 * K * (size_t)(2 * pair), 4 * (size_t)N1, e->stream));
    if (N2) TR_CHK(d2h_sync(v2.data(), (char *)e->owner.p + 4 * K * (size_t)(2 * pair + 1), 4 * (size_t)N2, e->stream));
    int nf = 0;
    for (int i1 = 0; i1 < N1; i1++) {   // agreement check (ORBmatcher.cc:1706-1720)
        const int idx2 = v1[i1];
        if (idx2 >= 0 && idx2 < N2 && v2[idx2] == i1) {
            matches12[i1] = kf2_mp[idx2];
            nf++;
        }
    }
    *nfound = nf;
    return ORBX_OK;
}

int orbt_search_by_sim3(orbt_engine *e, const orbt_frame *kf1, const int32_t *kf1_mp, const orbt_frame *kf2,
                        const int32_t *kf2_mp, const orbt_mappoints *M, float s12, const float R12[9],
                        const float t12[3], float th, int32_t *matches12, int32_t *nfound) {
    if (!e || !kf1 || !kf2 || !M) return ORBX_EINVAL;
    const int need = std::max(kf1->n, kf2->n);
    if (e->nslots < 2 || e->cap_kp < need || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(2, e->nslots), std::max(e->cap_kp, need), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage_search_by_sim3(e, 0, kf1, kf1_mp, kf2, kf2_mp, M, s12, R12, t12, matches12);
    if (!rc) rc = orbt_run_sim3_match_batch(e, 1, th, nullptr);
    if (!rc) rc = orbt_fetch_search_by_sim3(e, 0, kf2_mp, matches12, nfound);
    return rc;
}

int orbt_run_fuse_batch(orbt_engine *e, int n_slots, float th, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    hipStream_t st = pick(e, stream);
    TR_CHK(order_after_done(e, st));
    if (grid(e, n_slots, st)) return ORBX_EDEVICE;
    const int mm = std::max(1, max_n(e, 0, n_slots));
    track_fuse_kernel<<<dim3((mm + 255) / 256, n_slots), 256, 0, st>>>(make_slots(e), th, 0, e->fuse_idx.as<int>(),
                                                                       e->fuse_dist.as<int>());
    TR_CHK(hipGetLastError());
    TR_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbt_fetch_fuse(orbt_engine *e, int slot, int32_t *best_idx, int32_t *best_dist) {
    if (!e || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    TR_CHK(hipSetDevice(e->device));
    TR_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    const size_t M = (size_t)e->cap_mp, s = (size_t)slot, m = (size_t)e->hfr[slot].n_mp;
    if (m && best_idx) TR_CHK(d2h_sync(best_idx, (char *)e->fuse_idx.p + 4 * s * M, 4 * m, e->stream));
    if (m && best_dist) TR_CHK(d2h_sync(best_dist, (char *)e->fuse_dist.p + 4 * s * M, 4 * m, e->stream));
    return ORBX_OK;
}

int orbt_fuse_candidates(orbt_engine *e, const orbt_frame *kf, const orbt_mappoints *M, float th, int32_t *best_idx,
                         int32_t *best_dist) {
    if (!e || !kf || !M || !best_idx || !best_dist) return ORBX_EINVAL;
    if (e->nslots < 1 || e->cap_kp < kf->n || e->cap_mp < M->n) {
        const int rc = orbt_reserve(e, std::max(1, e->nslots), std::max(e->cap_kp, kf->n), std::max(e->cap_mp, M->n));
        if (rc) return rc;
    }
    int rc = orbt_stage(e, 0, kf, M, nullptr, nullptr, nullptr, nullptr);
    if (rc) return rc;
    rc = orbt_run_fuse_batch(e, 1, th, nullptr);
    if (rc) return rc;
    return orbt_fetch_fuse(e, 0, best_idx, best_dist);
}

}  // extern "C"
