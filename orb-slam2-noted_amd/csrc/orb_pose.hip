// MI355X-native Optimizer::PoseOptimization (Optimizer.cc:375-622), SURVEY.md §8f rank 2.
//
// One 256-thread workgroup per frame runs the whole thing on the device: four rounds of
// SparseOptimizer::optimize(10) (g2o OptimizationAlgorithmLevenberg, levenberg.cpp:61-164) on
// the single VertexSE3Expmap, each round restarting from the frame's pose, with the unary
// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose edges
// (types_six_dof_expmap.cpp:266-364) spread over the threads:
//   per LM iteration   residuals + Huber weights + J^T W J / J^T W e partials per thread,
//                      one block reduction of 1 + 21 + 6 doubles
//   per LM trial       thread 0: Eigen::LDLT (diagonal pivoting) of H + lambda I,
//                      SE3Quat::exp update; all threads: trial residuals (kept as g2o's
//                      stale _error) + robust chi2 reduction; thread 0: accept / reject
//   between rounds     chi2 (float) > 5.991 / 7.815 -> level 1 (outlier), Huber off after
//                      round 2 (Optimizer.cc:537-595)
// No host round trip inside the solve; frames are batched one workgroup each.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "orb_engine.h"
#include "orbslam2_amd.h"
#include "se3_device.h"

using namespace orbamd;
using namespace g2oamd;

#define PO_CHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd pose: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace orbpose {

constexpr int kThreads = 256;
constexpr int kRed = 28;   // chi2 + 21 (upper H) + 6 (b)

struct FrameHdr {
    int n;
    float Tcw[16];
    double fx, fy, cx, cy, bf;
};

struct PoseSlots {
    const FrameHdr *hdr;
    const float4 *xw;      // [S][cap] Xw, w unused
    const float4 *ob;      // [S][cap] u, v, uR, invSigma2
    double *err;           // [S][cap][3] g2o _error
    uint8_t *outlier;      // [S][cap] mvbOutlier / level
    float *Tout;           // [S][16]
    int *nin;              // [S]
    int *iters;            // [S][4]
    int cap;
};

// computeError (types_six_dof_expmap.h:153-157, 184-188 + cam_project .cpp:302-332)
__device__ inline void edge_error(const Pose &T, const FrameHdr &h, float4 xw, float4 ob, double e[3]) {
    const double X[3] = {xw.x, xw.y, xw.z};
    double p[3];
    quat_rotate(T.q, X, p);
    p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
    if (!(ob.z >= 0)) {
        const double u = p[0] / p[2], v = p[1] / p[2];
        e[0] = (double)ob.x - (u * h.fx + h.cx);
        e[1] = (double)ob.y - (v * h.fy + h.cy);
        e[2] = 0;
    } else {
        const float invz = (float)(1.0 / p[2]);
        const double r0 = p[0] * invz * h.fx + h.cx;
        const double r1 = p[1] * invz * h.fy + h.cy;
        const double r2 = r0 - h.bf * invz;
        e[0] = (double)ob.x - r0;
        e[1] = (double)ob.y - r1;
        e[2] = (double)ob.z - r2;
    }
}

__device__ inline double edge_chi2(const double e[3], double info, bool stereo) {
    double s = e[0] * info * e[0] + e[1] * info * e[1];
    if (stereo) s += e[2] * info * e[2];
    return s;
}

// RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-90): rho0, weight rho1
__device__ inline double huber(double chi, bool stereo, bool robust, double &w) {
    w = 1.0;
    if (!robust) return chi;
    const double delta = stereo ? (double)(float)sqrt(7.815) : (double)(float)sqrt(5.991);   // Optimizer.cc:459-460
    const double dsqr = delta * delta;
    if (chi <= dsqr) return chi;
    const double s = sqrt(chi);
    w = delta / s;
    return 2 * s * delta - dsqr;
}

// sum-reduce v[0..N) over the workgroup into red[] (every thread reads the result)
template <int N>
__device__ inline void block_reduce(double *v, double *red, double (*wsum)[kRed]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < N; k++) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        v[k] = x;
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < N; k++) wsum[wv][k] = v[k];
    __syncthreads();
    if (threadIdx.x < N) red[threadIdx.x] = ((wsum[0][threadIdx.x] + wsum[1][threadIdx.x]) + wsum[2][threadIdx.x]) +
                                            wsum[3][threadIdx.x];
    __syncthreads();
}

// Eigen::LDLT<MatrixXd> (lower, diagonal pivoting) + solve; false when !isPositive().
// Register-resident: the matrix is kept fully symmetric (every lower-triangle write is
// mirrored), so Eigen's partial lower-triangle swap of pivot k <-> big equals a full symmetric
// row + column swap, done with compile-time indices and selects on the runtime `big`. Same
// operation sequence as the oracle's restatement (oracle/lba_oracle.c orc_ldlt_solve6).
__device__ bool ldlt_solve6(const double *Hin, const double *b, double *x) {
    double a[6][6];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) a[i][j] = i >= j ? Hin[6 * i + j] : Hin[6 * j + i];
    int tr[6];
    int sign = 0;
    bool fail = false;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        int big = k;
        double bv = fabs(a[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (fabs(a[i][i]) > bv) { bv = fabs(a[i][i]); big = i; }
        tr[k] = big;
#pragma unroll
        for (int r = k + 1; r < 6; r++) {
            if (r == big) {
#pragma unroll
                for (int j = 0; j < 6; j++) { const double t = a[k][j]; a[k][j] = a[r][j]; a[r][j] = t; }
#pragma unroll
                for (int i = 0; i < 6; i++) { const double t = a[i][k]; a[i][k] = a[i][r]; a[i][r] = t; }
            }
        }
        if (k > 0) {
            double temp[6];
#pragma unroll
            for (int j = 0; j < k; j++) temp[j] = a[j][j] * a[k][j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += a[k][j] * temp[j];
            a[k][k] -= s;
#pragma unroll
            for (int i = k + 1; i < 6; i++) {
                double t = 0;
#pragma unroll
                for (int j = 0; j < k; j++) t += a[i][j] * temp[j];
                a[i][k] -= t;
                a[k][i] = a[i][k];
            }
        }
        const double akk = a[k][k];
        const bool valid = fabs(akk) > 0;
        if (k == 0 && !valid) fail = true;
        if (valid)
#pragma unroll
            for (int i = k + 1; i < 6; i++) { a[i][k] /= akk; a[k][i] = a[i][k]; }
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    if (fail || !(sign == 1 || sign == 0)) return false;
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = b[i];
#pragma unroll
    for (int k = 0; k < 6; k++)
#pragma unroll
        for (int r = k + 1; r < 6; r++)
            if (r == tr[k]) { const double t = y[k]; y[k] = y[r]; y[r] = t; }
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < i; j++) y[i] -= a[i][j] * y[j];
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = fabs(a[i][i]) > DBL_MIN ? y[i] / a[i][i] : 0.0;
#pragma unroll
    for (int i = 5; i >= 0; i--)
#pragma unroll
        for (int j = i + 1; j < 6; j++) y[i] -= a[j][i] * y[j];
#pragma unroll
    for (int k = 5; k >= 0; k--)
#pragma unroll
        for (int r = k + 1; r < 6; r++)
            if (r == tr[k]) { const double t = y[k]; y[k] = y[r]; y[r] = t; }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

struct Shared {
    Pose T, T2;
    double red[kRed];
    double wsum[4][kRed];
    double H[36], b[6];
    double Hl[36], x[6];
    double lambda, ni, currentChi, iniChi, rho;
    int qmax, nBad, stop, cnt;
};

// errors of the active edges at `T` (+ the robust chi2 partial; + H/b partials if `lin`)
template <bool lin>
__device__ void accumulate(const PoseSlots &P, int s, const FrameHdr &h, const Pose &T, bool robust,
                           Shared &sh) {
    double v[kRed];
#pragma unroll
    for (int k = 0; k < kRed; k++) v[k] = 0;
    const long long base = (long long)s * P.cap;
    for (int k = threadIdx.x; k < h.n; k += kThreads) {
        if (P.outlier[base + k]) continue;
        const float4 xw = P.xw[base + k], ob = P.ob[base + k];
        const bool stereo = ob.z >= 0;
        double e[3];
        edge_error(T, h, xw, ob, e);
        double *E = P.err + (base + k) * 3;
        E[0] = e[0]; E[1] = e[1]; E[2] = e[2];
        const double info = ob.w;
        double w;
        v[0] += huber(edge_chi2(e, info, stereo), stereo, robust, w);
        if constexpr (lin) {
            // linearizeOplus (types_six_dof_expmap.cpp:283-301, 337-362)
            const double X[3] = {xw.x, xw.y, xw.z};
            double p[3];
            quat_rotate(T.q, X, p);
            p[0] += T.t[0]; p[1] += T.t[1]; p[2] += T.t[2];
            const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
            double J[18];
            J[0] = x * y * invz_2 * h.fx; J[1] = -(1 + (x * x * invz_2)) * h.fx; J[2] = y * invz * h.fx;
            J[3] = -invz * h.fx; J[4] = 0; J[5] = x * invz_2 * h.fx;
            J[6] = (1 + y * y * invz_2) * h.fy; J[7] = -x * y * invz_2 * h.fy; J[8] = -x * invz * h.fy;
            J[9] = 0; J[10] = -invz * h.fy; J[11] = y * invz_2 * h.fy;
            J[12] = J[0] - h.bf * y * invz_2; J[13] = J[1] + h.bf * x * invz_2; J[14] = J[2];
            J[15] = J[3]; J[16] = 0; J[17] = J[5] - h.bf * invz_2;
            // lower triangle (the part Eigen::LDLT reads), row-major; constant register indices
            const double W = w * info;
            int u = 1;
#pragma unroll
            for (int a = 0; a < 6; a++)
#pragma unroll
                for (int c = 0; c <= a; c++) {
                    double hh = J[a] * W * J[c];
                    hh += J[6 + a] * W * J[6 + c];
                    if (stereo) hh += J[12 + a] * W * J[12 + c];
                    v[u++] += hh;
                }
#pragma unroll
            for (int a = 0; a < 6; a++) {
                double t = J[a] * (info * e[0]);
                t += J[6 + a] * (info * e[1]);
                if (stereo) t += J[12 + a] * (info * e[2]);
                v[22 + a] -= w * t;
            }
        }
    }
    if constexpr (lin) block_reduce<kRed>(v, sh.red, sh.wsum);
    else block_reduce<1>(v, sh.red, sh.wsum);
}

// SparseOptimizer::optimize(iterations) + OptimizationAlgorithmLevenberg::solve on the pose
__device__ int optimize(const PoseSlots &P, int s, const FrameHdr &h, bool robust, int iterations, Shared &sh) {
    const int tid = threadIdx.x;
    const long long base = (long long)s * P.cap;
    int act = 0;
    for (int k = tid; k < h.n; k += kThreads) act += !P.outlier[base + k];
    if (tid == 0) sh.cnt = 0;
    __syncthreads();
    atomicAdd(&sh.cnt, act);
    __syncthreads();
    if (sh.cnt == 0) return -1;
    int it = 0;
#ifdef ORBP_PROFILE
    long long t_lin = 0, t_solve = 0, t_trial = 0, t_acc = 0, t0;
#define PT0() t0 = clock64()
#define PT1(v) v += clock64() - t0
#else
#define PT0()
#define PT1(v)
#endif
    for (int i = 0; i < iterations; i++) {
        PT0();
        accumulate<true>(P, s, h, sh.T, robust, sh);
        PT1(t_lin);
        if (tid == 0) {
            sh.currentChi = sh.iniChi = sh.red[0];
            int u = 1;
            for (int a = 0; a < 6; a++)
                for (int c = 0; c <= a; c++) { sh.H[6 * a + c] = sh.red[u]; sh.H[6 * c + a] = sh.red[u]; u++; }
            for (int a = 0; a < 6; a++) sh.b[a] = sh.red[22 + a];
            if (i == 0) {
                double mx = 0;
                for (int a = 0; a < 6; a++) mx = fmax(fabs(sh.H[7 * a]), mx);
                sh.lambda = 1e-5 * mx;
                sh.ni = 2;
                sh.nBad = 0;
            }
            sh.qmax = 0;
        }
        __syncthreads();
        bool ok2 = true;
        do {
            PT0();
            if (tid == 0) {
                for (int k = 0; k < 36; k++) sh.Hl[k] = sh.H[k];
                for (int a = 0; a < 6; a++) sh.Hl[7 * a] += sh.lambda;
                ok2 = ldlt_solve6(sh.Hl, sh.b, sh.x);
                sh.T2 = pose_oplus(sh.T, sh.x);           // VertexSE3Expmap::oplusImpl
            }
            __syncthreads();
            PT1(t_solve);
            PT0();
            accumulate<false>(P, s, h, sh.T2, robust, sh);
            PT1(t_trial);
            PT0();
            if (tid == 0) {
                double tempChi = sh.red[0];
                if (!ok2) tempChi = DBL_MAX;
                double rho = sh.currentChi - tempChi;
                double scale = 0;
                for (int a = 0; a < 6; a++) scale += sh.x[a] * (sh.lambda * sh.x[a] + sh.b[a]);
                scale += 1e-3;
                rho /= scale;
                if (rho > 0 && isfinite(tempChi)) {
                    double alpha = 1. - pow((2 * rho - 1), 3);
                    alpha = fmin(alpha, 2. / 3.);
                    sh.lambda *= fmax(1. / 3., alpha);
                    sh.ni = 2;
                    sh.currentChi = tempChi;
                    sh.T = sh.T2;                       // discardTop
                } else {
                    sh.lambda *= sh.ni;                 // pop: the edges keep the trial _error
                    sh.ni *= 2;
                }
                sh.rho = rho;
                sh.qmax++;
            }
            __syncthreads();
            PT1(t_acc);
        } while (sh.rho < 0 && sh.qmax < 10);
        it++;
        if (tid == 0) {
            bool ok = true;
            if (sh.qmax == 10 || sh.rho == 0) ok = false;
            else {
                if ((sh.iniChi - sh.currentChi) * 1e3 < sh.iniChi) sh.nBad++; else sh.nBad = 0;
                if (sh.nBad >= 3) ok = false;
            }
            sh.stop = ok ? 0 : 1;
        }
        __syncthreads();
        if (sh.stop) break;
    }
#ifdef ORBP_PROFILE
    if (tid == 0 && blockIdx.x == 0) printf("orbp prof: it=%d lin=%lld solve=%lld trial=%lld accept=%lld cycles\n", it, t_lin, t_solve, t_trial, t_acc);
#endif
    return it;
}

__global__ __launch_bounds__(kThreads) void pose_opt_kernel(PoseSlots P) {
    __shared__ Shared sh;
    const int s = blockIdx.x, tid = threadIdx.x;
    const FrameHdr &h = P.hdr[s];
    const long long base = (long long)s * P.cap;
    for (int k = tid; k < h.n; k += kThreads) P.outlier[base + k] = 0;
    if (tid < 16) P.Tout[16 * s + tid] = h.Tcw[tid];
    if (tid < 4) P.iters[4 * s + tid] = -1;
    if (h.n < 3) {                                     // nInitialCorrespondences < 3
        if (tid == 0) P.nin[s] = 0;
        return;
    }
    Pose T0;
    {   // Converter::toSE3Quat(pFrame->mTcw)
        const float *m = h.Tcw;
        const double R[9] = {m[0], m[1], m[2], m[4], m[5], m[6], m[8], m[9], m[10]};
        quat_from_R_norm(R, T0.q);
        T0.t[0] = m[3]; T0.t[1] = m[7]; T0.t[2] = m[11];
        T0.pad = 0;
    }
    __syncthreads();
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        if (tid == 0) sh.T = T0;                        // vSE3->setEstimate(toSE3Quat(mTcw))
        __syncthreads();
        const int iters = optimize(P, s, h, it < 3, 10, sh);
        if (tid == 0) P.iters[4 * s + it] = iters;
        int bad = 0;
        for (int k = tid; k < h.n; k += kThreads) {
            const float4 xw = P.xw[base + k], ob = P.ob[base + k];
            const bool stereo = ob.z >= 0;
            double *E = P.err + (base + k) * 3;
            if (P.outlier[base + k]) edge_error(sh.T, h, xw, ob, E);   // e->computeError()
            const double e[3] = {E[0], E[1], E[2]};
            const float chi2 = (float)edge_chi2(e, ob.w, stereo);
            const bool out = chi2 > (stereo ? 7.815f : 5.991f);
            P.outlier[base + k] = out ? 1 : 0;
            bad += out;
        }
        __syncthreads();
        if (tid == 0) sh.cnt = 0;
        __syncthreads();
        atomicAdd(&sh.cnt, bad);
        __syncthreads();
        nBad = sh.cnt;
        if (h.n < 10) break;                            // optimizer.edges().size() < 10
    }
    if (tid == 0) {   // pFrame->SetPose(Converter::toCvMat(SE3quat_recov))
        double R[9];
        quat_to_R(sh.T.q, R);
        float *o = P.Tout + 16 * s;
        for (int a = 0; a < 3; a++) {
            for (int c = 0; c < 3; c++) o[4 * a + c] = (float)R[3 * a + c];
            o[4 * a + 3] = (float)sh.T.t[a];
        }
        o[12] = 0; o[13] = 0; o[14] = 0; o[15] = 1;
        P.nin[s] = h.n - nBad;
    }
}

}  // namespace orbpose

using namespace orbpose;

struct orbp_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;          // end of the last run (fetch waits on it only)
    hipStream_t done_stream = nullptr;
    int nslots = 0, cap = 0;
    DevBuf hdr, xw, ob, err, outlier, Tout, nin, iters;
    std::vector<int> n;
};

extern "C" {

int orbp_create(orbp_engine **out) {
    if (!out) return ORBX_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORBX_EDEVICE;
    orbp_engine *e = new orbp_engine();
    if (hipGetDevice(&e->device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        !(e->done = make_done_event())) {
        delete e;
        return ORBX_EDEVICE;
    }
    *out = e;
    return ORBX_OK;
}

void orbp_destroy(orbp_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) { (void)hipStreamSynchronize(e->stream); (void)hipStreamDestroy(e->stream); }
    if (e->done) { (void)hipEventSynchronize(e->done); (void)hipEventDestroy(e->done); }
    DevBuf *bufs[] = {&e->hdr, &e->xw, &e->ob, &e->err, &e->outlier, &e->Tout, &e->nin, &e->iters};
    for (DevBuf *b : bufs) b->release();
    delete e;
}

int orbp_reserve(orbp_engine *e, int n_slots, int cap_edges) {
    if (!e || n_slots <= 0 || cap_edges < 0) return ORBX_EINVAL;
    PO_CHK(hipSetDevice(e->device));
    cap_edges = std::max(cap_edges, 1);
    const size_t S = (size_t)n_slots, C = (size_t)cap_edges;
    if (e->hdr.ensure(sizeof(FrameHdr) * S) || e->xw.ensure(16 * S * C) || e->ob.ensure(16 * S * C) ||
        e->err.ensure(24 * S * C) || e->outlier.ensure(S * C) || e->Tout.ensure(64 * S) || e->nin.ensure(4 * S) ||
        e->iters.ensure(16 * S))
        return ORBX_EDEVICE;
    e->nslots = n_slots;
    e->cap = cap_edges;
    e->n.assign(n_slots, 0);
    return ORBX_OK;
}

int orbp_stage(orbp_engine *e, int slot, const orbp_frame *f) {
    if (!e || !f || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    if (f->n < 0 || f->n > e->cap) return ORBX_ECAP;
    if (f->n > 0 && (!f->Xw || !f->obs || !f->inv_sigma2)) return ORBX_EINVAL;
    PO_CHK(hipSetDevice(e->device));
    FrameHdr h;
    h.n = f->n;
    std::memcpy(h.Tcw, f->Tcw, sizeof h.Tcw);
    h.fx = f->fx; h.fy = f->fy; h.cx = f->cx; h.cy = f->cy; h.bf = f->bf;
    std::vector<float4> xw(std::max(f->n, 1)), ob(std::max(f->n, 1));
    for (int k = 0; k < f->n; k++) {
        xw[k] = make_float4(f->Xw[3 * k], f->Xw[3 * k + 1], f->Xw[3 * k + 2], 0.f);
        ob[k] = make_float4(f->obs[3 * k], f->obs[3 * k + 1], f->obs[3 * k + 2], f->inv_sigma2[k]);
    }
    const size_t s = (size_t)slot, C = (size_t)e->cap;
    hipStream_t st = e->stream;
    PO_CHK(order_after_done(e, st));
    PO_CHK(hipMemcpyAsync((char *)e->hdr.p + sizeof(FrameHdr) * s, &h, sizeof h, hipMemcpyHostToDevice, st));
    if (f->n) {
        PO_CHK(hipMemcpyAsync((char *)e->xw.p + 16 * s * C, xw.data(), 16 * (size_t)f->n, hipMemcpyHostToDevice, st));
        PO_CHK(hipMemcpyAsync((char *)e->ob.p + 16 * s * C, ob.data(), 16 * (size_t)f->n, hipMemcpyHostToDevice, st));
    }
    PO_CHK(hipStreamSynchronize(st));
    e->n[slot] = f->n;
    return ORBX_OK;
}

int orbp_run_batch(orbp_engine *e, int n_slots, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    PO_CHK(hipSetDevice(e->device));
    PoseSlots P;
    P.hdr = e->hdr.as<FrameHdr>(); P.xw = e->xw.as<float4>(); P.ob = e->ob.as<float4>();
    P.err = e->err.as<double>(); P.outlier = e->outlier.as<uint8_t>(); P.Tout = e->Tout.as<float>();
    P.nin = e->nin.as<int>(); P.iters = e->iters.as<int>(); P.cap = e->cap;
    const hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    PO_CHK(order_after_done(e, st));
    pose_opt_kernel<<<n_slots, kThreads, 0, st>>>(P);
    PO_CHK(hipGetLastError());
    PO_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbp_fetch(orbp_engine *e, int slot, orbp_result *r) {
    if (!e || !r || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    PO_CHK(hipSetDevice(e->device));
    PO_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    hipStream_t st = e->stream;
    const size_t s = (size_t)slot, C = (size_t)e->cap;
    PO_CHK(hipMemcpyAsync(r->Tcw, (char *)e->Tout.p + 64 * s, 64, hipMemcpyDeviceToHost, st));
    PO_CHK(hipMemcpyAsync(&r->n_inliers, (char *)e->nin.p + 4 * s, 4, hipMemcpyDeviceToHost, st));
    PO_CHK(hipMemcpyAsync(r->iterations, (char *)e->iters.p + 16 * s, 16, hipMemcpyDeviceToHost, st));
    if (r->outlier && e->n[slot])
        PO_CHK(hipMemcpyAsync(r->outlier, (char *)e->outlier.p + s * C, (size_t)e->n[slot], hipMemcpyDeviceToHost, st));
    PO_CHK(hipStreamSynchronize(st));
    return ORBX_OK;
}

int orbp_pose_optimization(orbp_engine *e, const orbp_frame *f, orbp_result *r) {
    if (!e || !f || !r) return ORBX_EINVAL;
    if (e->nslots < 1 || e->cap < f->n) {
        const int rc = orbp_reserve(e, std::max(1, e->nslots), std::max(e->cap, f->n));
        if (rc) return rc;
    }
    int rc = orbp_stage(e, 0, f);
    if (rc) return rc;
    rc = orbp_run_batch(e, 1, nullptr);
    if (rc) return rc;
    return orbp_fetch(e, 0, r);
}

}  // extern "C"
