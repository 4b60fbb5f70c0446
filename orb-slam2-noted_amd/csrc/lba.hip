// MI355X-native Optimizer::LocalBundleAdjustment core (Optimizer.cc:900-1008) over the
// g2o LM + Schur path it uses (BlockSolver_6_3 + OptimizationAlgorithmLevenberg), FP64.
//
// Device work per LM trial (N10-N13 of SURVEY.md §2.1); the per-slot linearisation is kept
// per estimate buffer, so a new iteration starts from the one lba_errors formed for the
// accepted trial:
//   lba_linearize     (first slot of an optimize() only) one thread per active edge: residual,
//                     Huber weight, analytic 2x9 / 3x9 Jacobians, the quadratic-form pieces as
//                     landmark-major (Hll, bl, Hpl) and pose-major (Hpp, bp) records
//   lba_reduce_points 16 lanes per landmark: Hll (3x3), b_l over the landmark's contiguous
//                     records in CSR order; in a new iteration after the first (lambda known)
//                     also the landmark half of the Schur step: Dinv = (Hll + lambda I)^-1,
//                     L = chol(Dinv), w = L^T b_l and every edge's 6x3 block of Y = Hpl L
//   lba_reduce_poses  one 1024-thread workgroup per free pose: Hpp (6x6), b_p, fixed-order sums
//   lba_prep_slots    the landmark half of the Schur step when lba_reduce_points did not do it
//                     (the first iteration: lambda = tau * maxDiagonal; retried trials)
//   lba_schur_tiles   Hschur = Hpp + lambda I - Y Y^T block-sparse on FP64 matrix cores
//                     (v_mfma_f64_16x16x4f64) over the landmark rows each upper 16 x 16 tile
//                     pair shares, Y stored transposed, chunks of 64 MFMA steps per 4-wave
//                     workgroup, lba_schur_finish sums a pair's chunk tiles; b_schur = b_p - Y w
//   lba_chol_tiled    (6P <= 128) dense Cholesky in LDS over 16-column panels (diagonal tiles by
//                     DPP64 broadcasts folded into v_fmac_f64, FP64 MFMA panel / trailing
//                     updates) + the two solves
//   lba_chol_panel/_update/_solve_blocked  blocked Cholesky for 6P > 128
//   lba_update        x_l = Dinv (b_l - Hpl^T x_p) (8 lanes per landmark), T <- exp(x_p) T
//                     (SE3Quat::exp, left-multiplied), X <- X + x_l, computeScale block sums
//   lba_errors        trial residuals (kept as g2o's stale _error), robust chi2 block sums and
//                     the trial's linearisation into the trial estimate's record set
//   lba_decide        the LM accept/reject/lambda logic (optimization_algorithm_levenberg.cpp
//                     :61-164) and SparseOptimizer::optimize's stop rules: rho, lambda / nu,
//                     nBad; an accepted trial swaps the estimate (and linearisation) buffers
// The LM state lives on the device (LMState): every kernel of a trial slot reads it and
// returns at once when the optimisation has finished (the reductions also when the slot is a
// retry of the same iteration). The host enqueues slots in chunks and reads the state back
// once per chunk instead of once per trial.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <climits>
#include <cstring>
#include <numeric>
#include <sched.h>
#include <string>
#include <thread>
#include <vector>

#include "orb_engine.h"
#include "orbslam2_amd.h"
#include "se3_device.h"
#include "lba_host.h"

#define LBA_CHK(x)                                                                  \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd lba: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace lbaamd {

using namespace g2oamd;

constexpr int kSmallNP = 128;        // Schur dimension factored in one workgroup's LDS
constexpr int kMaxPoses = 2048;      // 6 * 2048 = 12288: Hs 1.2 GB, far beyond any LocalBA window
constexpr int kCB = 32;              // blocked Cholesky panel width (Schur dimension > kSmallNP)
constexpr int kRedBlocks = 16384;    // partial-sum region stride (blocks) for scalar reductions

// device-resident LM control (optimization_algorithm_levenberg.cpp:61-164 state)
struct LMState {
    double lambda, ni, currentChi, iniChi, rho, final_chi;
    int qmax, nBad, it, iterations, done, newiter, accepted, trials;   // trials: LM trials decided
    int cur;        // estimate buffers: cur = 0 -> (T, X) current, (T2, X2) trial; 1 -> swapped
    int stop_at;    // test hook: pbStopFlag counts as raised once `trials` reaches it (INT_MAX: never)
    int seen;       // a terminate() check of this optimize() found pbStopFlag raised
    int gate;       // the second optimize()'s start (lba_phase2_begin): 0 run, 1 deferred (enqueued before the
                    // first optimize() had ended), 2 skipped (bDoMore false, Optimizer.cc:913-917)
    int fault;      // a trial's in-launch hand-off timed out (Graph::arrive[1]): the optimisation ended
                    // there and lba_solve returns ORBX_EDEVICE
};

struct EdgeDev {
    int point, pose;
    double obs[3];
    double info, delta, dsqr;
    double fx, fy, cx, cy, bf;
    int stereo, robust;
};

struct Graph {
    // vertices
    Pose *T, *T2;
    double *X, *X2;
    // edges
    const EdgeDev *E;
    double *err;           // [ne][3] g2o _error
    const int *act;        // active edge indices (edge order)
    const uint8_t *on;     // per active slot: 1 = level 0; 0 = set to level 1 by the phase-1 outlier test
    EdgeDev *E_lm;         // the edge records in landmark-major (pt_items) order: lba_lin_points reads
    uint8_t *on_lm;        // them and the level flags by record position, one dependent load fewer
    int nact;
    const int *pose_hidx;  // per pose vertex, -1 = fixed / inactive
    const int *point_hidx;
    const int *hpose, *hpoint;  // hessian index -> vertex
    int P, Lm;
    const int *pt_start, *pt_items;  // per active point: active slots (all edges of the point)
    const int *ps_start, *ps_items;  // per free pose: active slots
    const int *slot_ppos;            // per active slot: its position in ps_items (-1 fixed pose)
    double *ywp;                     // [ps_items][6]: the slot's Y block times w_l (b_schur pieces)
    const int *slot_pt, *slot_ph;    // per active slot: hessian point / pose index (-1 fixed)
    const int *slot_lpos;            // per active slot: its position in pt_items
    const int *lpos_ph;              // per pt_items position: the slot's hessian pose index (-1 fixed)
    const int *lpos_ppos;            // per pt_items position: the slot's ps_items position (-1 fixed)
    // system; the per-slot linearisation is kept per estimate buffer (index = LMState::cur of the
    // estimate it was formed at): lba_errors linearises the trial, and accepting it swaps both
    double *conl[2];       // [pt_items][9]: Hll upper (6) bl (3), landmark-major (point CSR order)
    double *conp[2];       // [ps_items][27]: Hpp upper (21) bp (6), pose-major
    double *hpl[2];        // [pt_items][18]: Hpl, landmark-major
    double *Hll, *bl;      // [Lm][9], [Lm][3]
    double *Hpp, *bp;      // [P][36], [P][6]
    double *Dinv;          // [Lm][9]
    double *Lc;            // [Lm][6] chol(Dinv): L00 L10 L20 L11 L21 L22
    double *Y;             // [Kpad][NPW] (point columns major: Y^T); column wrow = w
    double *w;             // = Y + wrow, stride NPW
    double *Hs, *bs;       // [NP][NP], [NP]
    double *x;             // [6P + 3Lm]
    double *partial;       // [4][kRedBlocks]: robust chi2 block sums of linearisation set 0 | point
                           // maxDiagonal | pose maxDiagonal | robust chi2 block sums of set 1
    double *scalars;       // [8]: chi2, maxdiag, tempChi, scale, ok, lambda
    LMState *lm;           // the LM state this launch reads (and, for a deciding launch, writes)
    const LMState *lm_src; // a deciding lba_reduce_points: the state before the decision (ping-pong)
    LMState *lm_buf[2];    // the two state buffers (host bookkeeping: lm is one of them)
    const unsigned *stopf; // pbStopFlag mirrored by lba_solve's host loop into page-locked, device-mapped memory
    unsigned *arrive;      // [0]: lba_finish_chol's finish-block arrivals; [1]: its hand-off timeout (fault) word
    unsigned spin_limit;   // the hand-off wait's poll bound (kSpinLimit; lba_set_test_option)
    double *W;             // 6P > kSmallNP: the Cholesky's work matrix [N2][LDW] (chol_global_body)
    int LDW;
    int Kpad;              // Y^T rows 3 Lm rounded up to 4; row Kpad (and up to Kpad + 3) is zero
    int NP;                // Schur dimension 6P padded to a multiple of kCB
    const int2 *tp_ij;     // upper tile pairs (I, J) of the Schur matrix
    const int *tp_start, *tp_rows;   // per pair: Y^T rows of the landmarks seen from both tiles (CSR)
    const int4 *tp_chunk;  // per chunk workgroup: pair, first step, steps, chunk index in the pair
    const int2 *tp_nch;    // per pair: first chunk, chunk count
    double *tp_part;       // [nchunks][256] chunk tiles (MFMA C layout)
    int npairs, nchunks;
    int NPW, wrow;         // Y^T leading dimension (NP + 16); Y^T column holding w (16 * ceil(6P / 16))
};

__device__ inline void decide_sums(const Graph &g, int nbt, double *sums_s);
__device__ LMState lm_next(const Graph &g, LMState s, double sc_sum, double chi_sum);

__device__ inline void edge_error_at(const EdgeDev &e, const Pose &T, const double *Xp, double err[3]) {
    double p[3];
    pose_map(T, Xp, p);
    if (!e.stereo) {
        const double u = p[0] / p[2], v = p[1] / p[2];
        err[0] = e.obs[0] - (u * e.fx + e.cx);
        err[1] = e.obs[1] - (v * e.fy + e.cy);
        err[2] = 0;
    } else {
        const float invz = (float)(1.0f / p[2]);          // types_six_dof_expmap.cpp:151
        const float bff = (float)e.bf;
        const double r0 = p[0] * invz * e.fx + e.cx;
        const double r1 = p[1] * invz * e.fy + e.cy;
        const double r2 = r0 - (double)(bff * invz);
        err[0] = e.obs[0] - r0;
        err[1] = e.obs[1] - r1;
        err[2] = e.obs[2] - r2;
    }
}
__device__ inline void edge_error(const Graph &g, const EdgeDev &e, const Pose *T, const double *X, double err[3]) {
    edge_error_at(e, T[e.pose], X + 3 * e.point, err);
}

__device__ inline double edge_chi2(const EdgeDev &e, const double err[3]) {
    double s = err[0] * e.info * err[0] + err[1] * e.info * err[1];
    if (e.stereo) s += err[2] * e.info * err[2];
    return s;
}

__device__ inline void huber(const EdgeDev &e, double chi, double &rho0, double &rho1) {
    if (chi <= e.dsqr) { rho0 = chi; rho1 = 1.0; }
    else { const double s = sqrt(chi); rho0 = 2 * s * e.delta - e.dsqr; rho1 = e.delta / s; }
}

// block sum of one double per thread (threads < 256) into *dst; the sum is returned to thread 0.
// The tree is the 8-step LDS fold's (t += t + s for s = 128 .. 1, the same additions in the same
// order, so the same bits) in one barrier: wave 0 adds (v_t + v_t+128) + (v_t+64 + v_t+192) and
// folds the rest across its lanes
__device__ inline double block_sum_to(double v, double *dst) {
    __shared__ double sh[256];
    if (threadIdx.x < 256) sh[threadIdx.x] = v;   // (lba_lin_points' trial-pose wave holds 0)
    __syncthreads();
    double a = 0;
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        a = (sh[t] + sh[t + 128]) + (sh[t + 64] + sh[t + 192]);
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) a += __shfl_down(a, s);   // lane 0: the tree's additions
        if (t == 0) *dst = a;
    }
    return a;
}

// ---- linearize: errors + robust chi2 + per-edge quadratic-form pieces
// Active slot s is edge s: every optimize() runs on all edges in edge order (build_active; the
// second one marks its level-1 edges in `on`), so the kernels index the edges by slot directly and
// issue the edge record with the LM-state load instead of after it.
__device__ __forceinline__ int chi_off(int set) { return set ? 3 * kRedBlocks : 0; }

// One slot's share of the system at estimate (Tc, Xc) into linearisation set `set`: the
// residual (g2o _error), Huber weight, analytic 2x9 / 3x9 Jacobians (types_six_dof_expmap.cpp
// :103-139, 188-234) and the quadratic-form pieces, landmark part at the slot's pt_items position
// `lpos`, pose part at its ps_items position `ppos` (-1: fixed pose, no pose part). A level-1 slot
// (on = 0) keeps its stale _error and contributes zeros. Two wave-uniform roles share a slot
// (twice the waves, each with about half the FP64 chain): role 0 writes the residual, Hll / bl
// and Hpl and returns the robust chi2; role 1 writes Hpp / bp (and returns 0).
__device__ __forceinline__ double linearize_slot_at(const Graph &g, const EdgeDev &e, bool on, int s, int lpos, int ppos,
                                                    const Pose &T, const double *Xp, int set, int role) {
    double *cl = g.conl[set] + 9LL * lpos, *hp = g.hpl[set] + 18LL * lpos;
    double *cp = g.conp[set] + 27LL * (ppos < 0 ? 0 : ppos);
    if (role == 1 && ppos < 0) return 0.0;   // no pose part
    if (!on) {
        if (role != 1) {
            for (int u = 0; u < 9; u++) cl[u] = 0.0;
            for (int u = 0; u < 18; u++) hp[u] = 0.0;
        }
        if (role != 0 && ppos >= 0)
            for (int u = 0; u < 27; u++) cp[u] = 0.0;
        return 0.0;
    }
    double err[3];
    edge_error_at(e, T, Xp, err);
    if (role != 1) { g.err[3 * s] = err[0]; g.err[3 * s + 1] = err[1]; g.err[3 * s + 2] = err[2]; }
    const double chi = edge_chi2(e, err);
    double r0 = chi, r1 = 1.0;
    if (e.robust) huber(e, chi, r0, r1);
    double p[3], R[9];
    pose_map(T, Xp, p);
    quat_to_R(T.q, R);
    const double x = p[0], y = p[1], z = p[2], fx = e.fx, fy = e.fy, bf = e.bf;
    double Jt[18];
    // g2o's Jacobians (types_six_dof_expmap.cpp:103-139, 188-234) with one division, 1 / z, and
    // products by it: within an ulp or two of the quotients, and ~20 FP64 division sequences fewer
    // per record on the linearisation's dependent chain
    const double iz = 1.0 / z, iz2 = iz * iz;
    Jt[0] = x * y * iz2 * fx; Jt[1] = -(1 + (x * x * iz2)) * fx; Jt[2] = y * iz * fx;
    Jt[3] = -iz * fx; Jt[4] = 0; Jt[5] = x * iz2 * fx;
    Jt[6] = (1 + y * y * iz2) * fy; Jt[7] = -x * y * iz2 * fy; Jt[8] = -x * iz * fy;
    Jt[9] = 0; Jt[10] = -iz * fy; Jt[11] = y * iz2 * fy;
    if (e.stereo) {
        Jt[12] = Jt[0] - bf * y * iz2; Jt[13] = Jt[1] + bf * x * iz2; Jt[14] = Jt[2];
        Jt[15] = Jt[3]; Jt[16] = 0; Jt[17] = Jt[5] - bf * iz2;
    }
    const int D = e.stereo ? 3 : 2;
    const double wW = r1 * e.info;
    double omr[3];
    _Pragma("unroll") for (int i = 0; i < 3; i++) if (i < D) omr[i] = -(e.info * err[i]) * r1;
    if (role != 0 && ppos >= 0) {
        int u = 0;
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int b = a; b < 6; b++) {
                double h = 0;
                _Pragma("unroll") for (int i = 0; i < 3; i++) if (i < D) h += Jt[6 * i + a] * wW * Jt[6 * i + b];
                cp[u++] = h;
            }
#pragma unroll
        for (int a = 0; a < 6; a++) {
            double v = 0;
            _Pragma("unroll") for (int i = 0; i < 3; i++) if (i < D) v += Jt[6 * i + a] * omr[i];
            cp[21 + a] = v;
        }
    }
    if (role == 1) return 0.0;
    double Jp[9];
    if (!e.stereo) {
        const double tmp[6] = {fx, 0, -x * iz * fx, 0, fy, -y * iz * fy};
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++)
                Jp[3 * i + j] = (-iz * tmp[3 * i]) * R[j] + (-iz * tmp[3 * i + 1]) * R[3 + j] + (-iz * tmp[3 * i + 2]) * R[6 + j];
    } else {
        for (int j = 0; j < 3; j++) {
            Jp[j] = -fx * R[j] * iz + fx * x * R[6 + j] * iz2;
            Jp[3 + j] = -fy * R[3 + j] * iz + fy * y * R[6 + j] * iz2;
            Jp[6 + j] = Jp[j] - bf * R[6 + j] * iz2;
        }
    }
    int u = 0;
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = a; b < 3; b++) {
            double h = 0;
            _Pragma("unroll") for (int i = 0; i < 3; i++) if (i < D) h += Jp[3 * i + a] * wW * Jp[3 * i + b];
            cl[u++] = h;
        }
#pragma unroll
    for (int a = 0; a < 3; a++) {
        double v = 0;
        _Pragma("unroll") for (int i = 0; i < 3; i++) if (i < D) v += Jp[3 * i + a] * omr[i];
        cl[6 + a] = v;
    }
    if (ppos >= 0) {
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) {
                double h = 0;
                _Pragma("unroll") for (int i = 0; i < 3; i++) if (i < D) h += Jt[6 * i + a] * wW * Jp[3 * i + b];
                hp[3 * a + b] = h;
            }
    }
    return r0;
}
__device__ __forceinline__ double linearize_slot(const Graph &g, const EdgeDev &e, bool on, int s, int lpos, int ppos,
                                                 const Pose *Tc, const double *Xc, int set, int role) {
    return linearize_slot_at(g, e, on, s, lpos, ppos, Tc[e.pose], Xc + 3 * e.point, set, role);
}

// Landmark-major linearisation, kLPL lanes per landmark (kLPB landmarks per workgroup): lane r
// takes records r, r + kLPL, ... of the landmark's contiguous run (CSR, pt_items) and linearises
// those slots (linearize_slot_at: residual, Huber weight, Jacobians, the quadratic-form pieces at
// the record's landmark-major and pose-major positions). Workgroups [0, nbl): landmarks;
// [nbl, nbt): free poses (UPDATE only). Chi2 block sums -> chi_part[b] and the set's partials.
//  !UPDATE (the first slot of an optimize(), was lba_linearize): at the current estimate, into
//          the current linearisation set.
//   UPDATE (every trial, was lba_update + lba_errors): the landmark back substitution x_l =
//          Dinv (b_l - Hpl^T x_p) (a fixed-order butterfly over the group), X_t = X + x_l, and each
//          slot's trial pose T_t = exp(x_p) T (the fifth wave's, below), then the trial's
//          residuals and linearisation into the trial set;
//          computeScale pieces x (lambda x + b) -> scale_part[b]. One launch instead of two, and
//          no grid-wide wait between the update and the residuals.
// The two linearize_slot_at roles run on two waves per 8 landmarks (role 0: residual, Hll / bl,
// Hpl; role 1: Hpp / bp), each redoing the landmark update. Same box: update_errors 0.256 -> 0.232 ms
// per call against one wave doing both (profiles/r04_ab_lba_roles.log)
constexpr int kLPL = 8, kLPB = 256 / kLPL / 2;
// lba_lin_points<true> workgroups carry a fifth wave that forms the trial poses T_t = exp(x_p) T
// of a small window (6P <= kSmallNP: lba_chol_tiled's) into LDS while the other four run the
// landmark update: the exp chain overlaps the update's loads instead of ending the solve
// (trial_pose, which the blocked path keeps)
constexpr int kLinThreads = 320;
template <bool UPDATE>
__global__ __launch_bounds__(UPDATE ? kLinThreads : 256) void lba_lin_points(Graph g, double *scale_part, double *chi_part,
                                                                           int nbl) {
    __shared__ Pose tps[kSmallNP / 6];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int role = wv & 1;   // wave-uniform
    const int grp = (wv >> 1) * (64 / kLPL) + lane / kLPL;
    const int r = threadIdx.x % kLPL;
    const int l = blockIdx.x * kLPB + grp;
    const bool isl = (int)blockIdx.x < nbl && wv < 4 && l < g.Lm;
    const bool small = UPDATE && 6 * g.P <= kSmallNP;   // trial poses: tps (else the solve's trial_pose)
    // the landmark's record range goes out with the LM-state load
    const int i0 = isl ? g.pt_start[l] : 0, i1 = isl ? g.pt_start[l + 1] : 0;
    const LMState lm = *g.lm;
    if (lm.done || (!UPDATE && !lm.newiter)) return;
    const bool cur = lm.cur;
    const int set = UPDATE ? !cur : cur;
    const Pose *Tc = cur ? g.T2 : g.T;
    const double *Xc = cur ? g.X2 : g.X;
    const double lambda = UPDATE ? lm.lambda : 0.0;
    // pbStopFlag snapshot for the decision of this trial (every workgroup of the deciding launch
    // must see the same value): one read of the mapped word, into device memory
    if (UPDATE && blockIdx.x == 0 && threadIdx.x == 0)
        g.scalars[6] = __hip_atomic_load(g.stopf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ? 1.0 : 0.0;
    double sc = 0, chi = 0;
    if ((int)blockIdx.x >= nbl) {   // free poses (UPDATE): T_t (small windows), computeScale pieces
        const int t = ((int)blockIdx.x - nbl) * 256 + threadIdx.x;
        if (UPDATE && t < g.P && threadIdx.x < 256) {
            const double *xp = g.x + 6 * t;
            if (small) {
                const int v = g.hpose[t];
                (cur ? g.T : g.T2)[v] = pose_oplus(Tc[v], xp);
            }
            for (int k = 0; k < 6; k++) sc += xp[k] * (lambda * xp[k] + g.bp[6 * t + k]);
        }
    } else {
      if (small && wv == 4 && lane < g.P) tps[lane] = pose_oplus(Tc[g.hpose[lane]], g.x + 6 * lane);
      double Xn[3] = {0, 0, 0};
      if (isl) {
        const int v = g.hpoint[l];
        Xn[0] = Xc[3 * v]; Xn[1] = Xc[3 * v + 1]; Xn[2] = Xc[3 * v + 2];
        if (UPDATE) {
            double c[3] = {0, 0, 0};
            const double *hpL = g.hpl[cur];
            for (int i = i0 + r; i < i1; i += kLPL) {
                const int ph = g.lpos_ph[i];
                if (ph < 0) continue;
                const double *B = hpL + 18LL * i;
                const double *xp = g.x + 6 * ph;
                for (int cc = 0; cc < 3; cc++) {
                    double a = 0;
                    for (int k = 0; k < 6; k++) a += B[3 * k + cc] * (-xp[k]);
                    c[cc] += a;
                }
            }
#pragma unroll
            for (int m = kLPL / 2; m > 0; m >>= 1)
#pragma unroll
                for (int cc = 0; cc < 3; cc++) c[cc] += __shfl_xor(c[cc], m);
            const double *bl = g.bl + 3 * l, *Di = g.Dinv + 9 * l;
            c[0] += bl[0]; c[1] += bl[1]; c[2] += bl[2];
            double *Xt = cur ? g.X : g.X2;
            double *xl = g.x + 6 * g.P + 3 * l;
#pragma unroll
            for (int a = 0; a < 3; a++) {
                const double xa = Di[3 * a] * c[0] + Di[3 * a + 1] * c[1] + Di[3 * a + 2] * c[2];
                Xn[a] += xa;
                if (r == 0 && role != 1) {
                    xl[a] = xa;
                    Xt[3 * v + a] = Xn[a];
                    sc += xa * (lambda * xa + bl[a]);
                }
            }
        }
      }
      if (small) __syncthreads();   // workgroup-uniform: tps complete
      if (isl)
        for (int i = i0 + r; i < i1; i += kLPL) {
            const int s = g.pt_items[i], ph = g.lpos_ph[i];
            const EdgeDev e = g.E_lm[i];
            // a free pose's trial T_t
            const Pose T = (UPDATE && ph >= 0) ? (small ? tps[ph] : (cur ? g.T : g.T2)[e.pose]) : Tc[e.pose];
            chi += linearize_slot_at(g, e, g.on_lm[i] != 0, s, i, ph >= 0 ? g.lpos_ppos[i] : -1, T, Xn, set, role);
        }
    }
    if (UPDATE) {
        block_sum_to(sc, scale_part + blockIdx.x);
        __syncthreads();   // block_sum_to's LDS is reused: every thread has read the first sum
    }
    const double bsum = block_sum_to(chi, chi_part + blockIdx.x);
    if (threadIdx.x == 0) g.partial[chi_off(set) + blockIdx.x] = bsum;
}

// ---- Schur: per landmark Dinv, L = chol(Dinv), Y block and w
__device__ inline void inv3(const double m[9], double o[9]) {
    const double c00 = m[4] * m[8] - m[5] * m[7];
    const double c10 = m[5] * m[6] - m[3] * m[8];
    const double c20 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c00 + m[1] * c10 + m[2] * c20;
    const double id = 1.0 / det;
    o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    o[3] = c10 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    o[6] = c20 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// (Hll + lambda I)^-1 (Eigen cofactor inverse) and L = chol(Dinv) of one landmark
__device__ inline void point_factor_of(const double H[9], double lambda, double Di[9], double L[6]) {
    double D[9];
    for (int k = 0; k < 9; k++) D[k] = H[k];
    D[0] += lambda; D[4] += lambda; D[8] += lambda;
    inv3(D, Di);
    // Dinv = L L^T (symmetrised)
    const double a00 = Di[0], a10 = 0.5 * (Di[3] + Di[1]), a11 = Di[4];
    const double a20 = 0.5 * (Di[6] + Di[2]), a21 = 0.5 * (Di[7] + Di[5]), a22 = Di[8];
    L[0] = sqrt(a00); L[1] = a10 / L[0]; L[2] = a20 / L[0];
    L[3] = sqrt(a11 - L[1] * L[1]); L[4] = (a21 - L[2] * L[1]) / L[3];
    L[5] = sqrt(a22 - L[2] * L[2] - L[4] * L[4]);
}
__device__ inline void point_factor(const Graph &g, int l, double lambda, double Di[9], double L[6]) {
    double H[9];
    for (int k = 0; k < 9; k++) H[k] = g.Hll[9 * l + k];
    point_factor_of(H, lambda, Di, L);
}

// The 6x3 Y block (Y = Hpl L: the pose's rows, the point's columns of Y^T) of one slot and its
// b_schur piece Y w (w = L^T b_l), from the slot's Hpl record B
__device__ __forceinline__ void slot_y(const Graph &g, int l, int ph, int ppos, const double *B, const double L[6],
                                       const double *bl) {
    const long long W = g.NPW;
    double *y = g.Y + 3LL * l * W + 6 * ph;   // Y^T rows 3l..3l+2, columns 6ph..6ph+5
    const double w0 = L[0] * bl[0] + L[1] * bl[1] + L[2] * bl[2], w1 = L[3] * bl[1] + L[4] * bl[2], w2 = L[5] * bl[2];
    double *yw = g.ywp + 6LL * ppos;
#pragma unroll
    for (int r = 0; r < 6; r++) {
        const double b0 = B[3 * r], b1 = B[3 * r + 1], b2 = B[3 * r + 2];
        const double y0 = b0 * L[0] + b1 * L[1] + b2 * L[2], y1 = b1 * L[3] + b2 * L[4], y2 = b2 * L[5];
        y[r] = y0;
        y[W + r] = y1;
        y[2 * W + r] = y2;
        yw[r] = y0 * w0 + y1 * w1 + y2 * w2;
    }
}

// Hll (3x3), b_l: one 16-lane group per landmark, lane k < 9 sums component k (Hll upper 6,
// bl 3) of the landmark's contiguous run of landmark-major records (conl) in CSR order, 8 records
// in flight; the |diagonal| maximum of the block's 16 landmarks -> partial[kRedBlocks + blockIdx]
constexpr int kRPL = 16;   // landmarks per lba_reduce_points workgroup
// With lambda known (a new iteration after the first) the landmark half of the Schur step runs in
// lba_reduce_points, and lba_prep_slots returns at once: it runs only in an optimize()'s first slot.
// fused (lambda = the LM state's): after the sums, the group's lanes gather the landmark's 9
// values through LDS, each factors (Hll + lambda I)^-1 = L L^T (point_factor_of: the bits
// lba_prep_slots forms) and lane r writes the Y blocks of records r, r + 16, ...; lane 0 writes
// Dinv and w. Block 0 also does lba_prep_slots' mode-1 work (chi2 sum -> scalars[0], lambda ->
// scalars[5]).
// retry (a rejected trial's next slot: same linearisation, new lambda): no sums -- the landmark's
// stored Hll / b_l feed the same fused tail (what lba_prep_slots' mode 0 formed before)
__device__ __forceinline__ void reduce_points_body(Graph &g, int set, bool fused, bool retry, double lambda, int n0,
                                                   double *sh) {
    const int l = blockIdx.x * kRPL + (threadIdx.x >> 4), k = threadIdx.x & 15;
    __shared__ double hv_s[256];
    double dmax = 0, v = 0;
    int i0 = 0, i1 = 0;
    if (l < g.Lm) {
        i0 = g.pt_start[l];
        i1 = g.pt_start[l + 1];
    }
    if (retry) {   // uniform
        if (l < g.Lm && k < 9) {
            // packed upper 00 01 02 11 12 22 -> the stored symmetric 3 x 3 (0, 1, 2, 4, 5, 8)
            v = k < 6 ? g.Hll[9 * l + (k < 3 ? k : k == 5 ? 8 : k + 1)] : g.bl[3 * l + k - 6];
        }
        hv_s[threadIdx.x] = v;
        __syncthreads();
    } else {
    if (l < g.Lm && k < 9) {
        const double *cl = g.conl[set] + k;
        for (int i = i0; i < i1; i += 8) {
            double r[8];
#pragma unroll
            for (int u = 0; u < 8; u++) r[u] = i + u < i1 ? cl[9LL * (i + u)] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (i + u < i1) v += r[u];
        }
        double *H = g.Hll + 9 * l;
        switch (k) {   // packed upper 00 01 02 11 12 22 -> the symmetric 3 x 3
            case 0: H[0] = v; break;
            case 1: H[1] = v; H[3] = v; break;
            case 2: H[2] = v; H[6] = v; break;
            case 3: H[4] = v; break;
            case 4: H[5] = v; H[7] = v; break;
            case 5: H[8] = v; break;
            default: g.bl[3 * l + k - 6] = v;
        }
        if (k == 0 || k == 3 || k == 5) dmax = fabs(v);
    }
    hv_s[threadIdx.x] = v;
    sh[threadIdx.x] = dmax;
    __syncthreads();
    if (threadIdx.x < 64) {   // a maximum: any order gives the same bits
        const int t = threadIdx.x;
        double m = fmax(fmax(sh[t], sh[t + 64]), fmax(sh[t + 128], sh[t + 192]));
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) m = fmax(m, __shfl_xor(m, s));
        if (t == 0) g.partial[kRedBlocks + blockIdx.x] = m;
    }
    if (!fused) return;   // uniform
    }
    if (l >= g.Lm) return;
    const double *hv = hv_s + (threadIdx.x & ~15);
    const double Hm[9] = {hv[0], hv[1], hv[2], hv[1], hv[3], hv[4], hv[2], hv[4], hv[5]}, bl[3] = {hv[6], hv[7], hv[8]};
    double Di[9], L[6];
    point_factor_of(Hm, lambda, Di, L);
    if (k == 0) {
        const long long W = g.NPW, c0 = 3LL * l;
        for (int q = 0; q < 9; q++) g.Dinv[9 * l + q] = Di[q];
        g.w[c0 * W] = L[0] * bl[0] + L[1] * bl[1] + L[2] * bl[2];
        g.w[(c0 + 1) * W] = L[3] * bl[1] + L[4] * bl[2];
        g.w[(c0 + 2) * W] = L[5] * bl[2];
    }
    for (int i = i0 + k; i < i1; i += 16) {
        const int ph = g.lpos_ph[i];
        if (ph < 0) continue;
        slot_y(g, l, ph, g.lpos_ppos[i], g.hpl[set] + 18LL * i, L, bl);
    }
}

// One component `comp` of a free pose's quadratic form (Hpp upper 0..20, b_p 21..26): the pose's
// contiguous run of pose-major records (conp), lane-strided with 8 loads in flight, then an xor
// butterfly -- a fixed order, so lba_reduce_points' pose workgroups (first slot) and lba_schur_tiles (every slot) form
// the same bits. Returns the sum to every lane.
__device__ __forceinline__ double pose_comp_sum(const Graph &g, int set, int ph, int comp, int lane) {
    const int t0 = g.ps_start[ph], t1 = g.ps_start[ph + 1];
    const double *cp = g.conp[set] + comp;
    double acc = 0;
    for (int tb = t0 + lane; tb < t1; tb += 64 * 8) {
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; u++) a[u] = tb + 64 * u < t1 ? cp[27LL * (tb + 64 * u)] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; u++) acc += a[u];
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) acc += __shfl_xor(acc, m);
    return acc;
}
// packed upper index u of a 6 x 6 -> (a, b), a <= b
__device__ __forceinline__ void upper6(int u, int &a, int &b) {
    a = 0;
    int start = 0;
    while (u >= start + 6 - a) { start += 6 - a; a++; }
    b = a + (u - start);
}
// Hpp (6x6) and b_p of every free pose, one wave per (pose, component): Hpp entries (comp < 21,
// both triangles), b_p (comp >= 21) and, for the 6 diagonal entries, |H| into the maxDiagonal
// partials. Only the first trial slot of an optimize() launches it (lambda init); later slots get
// the same sums from lba_schur_tiles' pose waves.
__device__ __forceinline__ void pose_comp_store(Graph &g, int set, int w, int lane, bool maxdiag) {
    const int ph = w / 27, comp = w - 27 * ph;
    if (ph >= g.P) return;
    const double v = pose_comp_sum(g, set, ph, comp, lane);
    if (lane != 0) return;
    if (comp >= 21) { g.bp[6 * ph + comp - 21] = v; return; }
    int a, b;
    upper6(comp, a, b);
    g.Hpp[36 * ph + 6 * a + b] = v;
    g.Hpp[36 * ph + 6 * b + a] = v;
    if (maxdiag && a == b) g.partial[2 * kRedBlocks + 6 * ph + a] = fabs(v);
}

// the landmark reductions on 256-thread workgroups (one landmark per thread: a merged launch with
// the pose reductions on 1024-thread workgroups spread the landmarks over 4x fewer CUs and took
// 22 us against 8 + 10), the pose reductions one 1024-thread workgroup per free pose
// A deciding launch (lm_src set: every trial slot of a chunk but its first) first runs the previous
// trial's LM decision: every workgroup forms the same state from lm_src (same sums, same flag
// snapshot, a pure function), workgroup 0 stores it into lm -- the other buffer, so no workgroup
// can read a state another one already advanced. One launch per trial fewer than a separate
// lba_decide.
// npw > 0 (an optimize()'s first slot, never a deciding one): the last npw workgroups are
// the pose reductions (Hpp, b_p and the pose maxDiagonal partials the lambda initialisation needs),
// in the same launch as the landmark reductions instead of one of their own
__global__ __launch_bounds__(256) void lba_reduce_points(Graph g, int n0, int nbt, int npw) {
    __shared__ double shp[256];
    __shared__ LMState lm_s;
    LMState lm;
    if ((int)blockIdx.x >= (int)gridDim.x - npw) {   // uniform: pose workgroups
        lm = *g.lm;
        if (lm.done || !lm.newiter) return;
        pose_comp_store(g, lm.cur, 4 * ((int)blockIdx.x - ((int)gridDim.x - npw)) + (threadIdx.x >> 6), threadIdx.x & 63, true);
        return;
    }
    if (g.lm_src) {   // uniform
        const LMState s0 = *g.lm_src;
        if (!s0.done) {
            decide_sums(g, nbt, shp);
            __syncthreads();
            if (threadIdx.x == 0) lm_s = lm_next(g, s0, shp[0], shp[1]);
        } else if (threadIdx.x == 0) {
            lm_s = s0;
        }
        __syncthreads();
        lm = lm_s;
        if (blockIdx.x == 0 && threadIdx.x == 0) *g.lm = lm;
        __syncthreads();   // shp is reused below
    } else {
        lm = *g.lm;
    }
    if (lm.done) return;
    reduce_points_body(g, lm.cur, lm.it > 0, !lm.newiter, lm.lambda, n0, shp);
}

// First kernel of an LM trial (setLambda + the landmark half of the Schur complement).
// Threads [0, nact): the 6x3 block Y = Hpl L of one active edge (its pose's rows, its point's
// columns of Y^T); threads [nact, nact + Lm): Dinv and w = L^T b_l of one landmark. The edge
// threads refactor their landmark (same arithmetic, so the same bits) instead of waiting for
// a separate landmark pass.
// mode 1: block 0 also finishes the linearisation's chi2 reduction -> scalars[0];
// mode 2 (first trial of the first iteration): every block reduces chi2 and maxDiagonal and
// uses lambda = tau * maxDiagonal (tau = 1e-5, optimization_algorithm_levenberg.cpp:179-191);
// otherwise lambda = the LM state's. Block 0 publishes lambda in scalars[5].
__global__ __launch_bounds__(256) void lba_prep_slots(Graph g, int n0, int n1, int n2) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    // the slot's index entries go out with the LM-state load (no dependence on it)
    const bool ist = t < g.nact;
    const int ph = ist ? g.slot_ph[t] : -1, l_t = ist ? g.slot_pt[t] : 0, lpos = ist ? g.slot_lpos[t] : 0,
              ppos = ist ? g.slot_ppos[t] : 0;
    const LMState lm = *g.lm;
    if (lm.done || (lm.newiter && lm.it > 0)) return;   // lba_reduce_points did it
    const int mode = lm.newiter ? (lm.it == 0 ? 2 : 1) : 0;
    double lambda = lm.lambda;
    if (mode == 2 || (mode == 1 && blockIdx.x == 0)) {   // uniform per block
        __shared__ double sa[256], sb[256];
        double a = 0, b = 0;
        const double *chi = g.partial + chi_off(lm.cur);   // the current linearisation's chi2 sums
        for (int i = threadIdx.x; i < n0; i += 256) a += chi[i];
        for (int i = threadIdx.x; i < n1; i += 256) b = fmax(b, g.partial[kRedBlocks + i]);
        for (int i = threadIdx.x; i < n2; i += 256) b = fmax(b, g.partial[2 * kRedBlocks + i]);
        sa[threadIdx.x] = a;
        sb[threadIdx.x] = b;
        __syncthreads();
        for (int s = 128; s > 0; s >>= 1) {
            if ((int)threadIdx.x < s) {
                sa[threadIdx.x] += sa[threadIdx.x + s];
                sb[threadIdx.x] = fmax(sb[threadIdx.x], sb[threadIdx.x + s]);
            }
            __syncthreads();
        }
        if (mode == 2) lambda = 1e-5 * sb[0];
        if (blockIdx.x == 0 && threadIdx.x == 0) { g.scalars[0] = sa[0]; g.scalars[1] = sb[0]; }
    }
    if (t == 0) {
        g.scalars[5] = lambda;
        if (mode == 2) g.lm->lambda = lambda;   // the trial's lambda lives in the LM state; no block reads
    }                                           // this field (mode 2 forms lambda itself)
    const long long W = g.NPW;
    double Di[9], L[6];
    if (ist) {
        if (ph < 0) return;
        const int l = l_t;
        point_factor(g, l, lambda, Di, L);
        // w_l = L^T b_l exactly as the landmark threads form it, for this block's share of Y w
        slot_y(g, l, ph, ppos, g.hpl[lm.cur] + 18LL * lpos, L, g.bl + 3 * l);
    } else if (t < g.nact + g.Lm) {
        const int l = t - g.nact;
        point_factor(g, l, lambda, Di, L);
        for (int k = 0; k < 9; k++) g.Dinv[9 * l + k] = Di[k];
        const double *b = g.bl + 3 * l;
        const long long c0 = 3LL * l;
        g.w[c0 * W] = L[0] * b[0] + L[1] * b[1] + L[2] * b[2];
        g.w[(c0 + 1) * W] = L[3] * b[1] + L[4] * b[2];
        g.w[(c0 + 2) * W] = L[5] * b[2];
    }
}

typedef double double4_t __attribute__((ext_vector_type(4)));

// Schur complement Hs = Hpp + lambda I - Y Y^T and b_schur = b_p - Y w (BlockSolver::buildSystem +
// schur, block_solver.hpp:354-439) over the 16 x 16 tiles of the 6P x 6P matrix, block-sparse on
// FP64 MFMA (v_mfma_f64_16x16x4f64): for every upper tile pair (I <= J) only the Y^T rows of the
// landmarks that have a free pose in both tile I's and tile J's columns are multiplied (tp_rows: 3
// rows per landmark, lists padded to 4-row steps with the zero row Kpad, built on the host per
// LocalBA call: build_schur_tiles). On C4 that issues 1.4x the algorithmic pair products instead of
// the dense SYRK's 10x. A pair's steps are cut into chunks of kSCH steps, one 4-wave workgroup per
// chunk (each wave 8 steps: the row indices in flight, then the 16 Y^T loads in flight, then 8
// MFMAs), the waves' accumulators summed in LDS in wave order into the chunk's tile (tp_part);
// lba_schur_finish sums each pair's chunk tiles in chunk order and writes tile (I, J) and its
// transpose (a last-arrival reduction in this kernel measured 77 us against 32 us: 420 agent-scope
// release fences), with Hpp on the pose-
// diagonal 6 x 6 blocks and lambda on the diagonal (setLambda). Workgroups past the chunks form
// b_schur, one wave per row: b_p - the sum of the pose's slot pieces Y_block w_l (ywp, written
// pose-major by lba_prep_slots).
constexpr int kSCH = 64;   // MFMA steps (4 Y^T rows each) per chunk workgroup
__global__ __launch_bounds__(256) void lba_schur_tiles(Graph g) {
    if (g.lm->done) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n6 = 6 * g.P;
    const long long W = g.NPW;
    if ((int)blockIdx.x >= g.nchunks + (n6 + 3) / 4) {   // Hpp: one wave per (pose, upper component)
        const int w = 4 * ((int)blockIdx.x - g.nchunks - (n6 + 3) / 4) + wv, ph = w / 21;
        if (ph < g.P) pose_comp_store(g, g.lm->cur, 27 * ph + (w - 21 * ph), lane, false);
        return;
    }
    if ((int)blockIdx.x >= g.nchunks) {   // b_schur rows 4 (blockIdx - nchunks) + wv
        const int row = 4 * ((int)blockIdx.x - g.nchunks) + wv;
        if (row >= n6) return;
        const int ph = row / 6, a = row % 6, i0 = g.ps_start[ph], i1 = g.ps_start[ph + 1];
        const double bpv = pose_comp_sum(g, g.lm->cur, ph, 21 + a, lane);   // b_p, the first slot's order
        if (lane == 0) g.bp[row] = bpv;
        double v = 0;
        for (int i = i0 + lane; i < i1; i += 256) {
            double q[4];
#pragma unroll
            for (int u = 0; u < 4; u++) q[u] = i + 64 * u < i1 ? g.ywp[6LL * (i + 64 * u) + a] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; u++) v += q[u];
        }
        // fixed-order wave sum (DPP-free: through LDS, lane order)
        __shared__ double bsum[4][64];
        bsum[wv][lane] = v;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            double sum = 0;
            for (int k = 0; k < 64; k++) sum += bsum[wv][k];
            g.bs[row] = bpv - sum;
        }
        return;
    }
    const int4 ch = g.tp_chunk[blockIdx.x];   // pair, first step, steps, chunk index within the pair
    const int2 ij = g.tp_ij[ch.x];
    const int I = ij.x, J = ij.y;
    const double *ya = g.Y + 16 * I + (lane & 15), *yb = g.Y + 16 * J + (lane & 15);
    const int *rows = g.tp_rows + g.tp_start[ch.x] + 4 * ch.y + (lane >> 4);   // rows[4 * step]
    const int nst = ch.z;
    double4_t acc = {0, 0, 0, 0};
    constexpr int kSB = kSCH / 4;   // steps per wave: wv, wv + 4, ...
    constexpr int kSU = kSB < 8 ? kSB : 8;   // steps per batch of loads in flight
#pragma unroll
    for (int u0 = 0; u0 < kSB; u0 += kSU) {
        if (wv + 4 * u0 >= nst) break;   // wave-uniform
        int r[kSU];
#pragma unroll
        for (int u = 0; u < kSU; u++) r[u] = wv + 4 * (u0 + u) < nst ? rows[4 * (wv + 4 * (u0 + u))] : g.Kpad;
        double av[kSU], bv[kSU];
#pragma unroll
        for (int u = 0; u < kSU; u++) { av[u] = ya[r[u] * W]; bv[u] = yb[r[u] * W]; }
#pragma unroll
        for (int u = 0; u < kSU; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
    }
    __shared__ double red[4][4][64];
#pragma unroll
    for (int q = 0; q < 4; q++) red[wv][q][lane] = acc[q];
    __syncthreads();
    if (wv != 0) return;
    double *part = g.tp_part + 256LL * blockIdx.x;
#pragma unroll
    for (int q = 0; q < 4; q++) part[64 * q + lane] = ((red[0][q][lane] + red[1][q][lane]) + red[2][q][lane]) + red[3][q][lane];
}

// one 4-wave workgroup per tile pair, wave q = rows 4q..4q+3 of the MFMA C tile: the pair's
// chunk tiles summed in chunk order (up to 32 chunk loads in flight per lane), Hpp on the
// pose-diagonal 6 x 6 blocks, lambda on the diagonal; tile (I, J) and its transpose into Hs
__global__ __launch_bounds__(256) void lba_schur_finish(Graph g) {
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6, p = blockIdx.x;
    const int2 ij = g.tp_ij[p], nc = g.tp_nch[p];   // (I, J); first chunk, chunk count
    if (g.lm->done) return;
    const int I = ij.x, J = ij.y, n6 = 6 * g.P;
    const long long NP = g.NP;
    const double lambda = g.lm->lambda;
    double v = 0;
    const double *tp = g.tp_part + 256LL * nc.x + 64 * q + lane;
    for (int c0 = 0; c0 < nc.y; c0 += 32) {
        double t[32];
#pragma unroll
        for (int u = 0; u < 32; u++) t[u] = c0 + u < nc.y ? tp[256LL * (c0 + u)] : 0.0;
#pragma unroll
        for (int u = 0; u < 32; u++)
            if (c0 + u < nc.y) v += t[u];
    }
    // C/D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * q
    const int row = 16 * I + (lane >> 4) + 4 * q, col = 16 * J + (lane & 15);
    if (row >= n6 || col >= n6) return;
    double h = 0;
    if (row / 6 == col / 6) h = g.Hpp[36 * (row / 6) + 6 * (row % 6) + (col % 6)];
    if (row == col) h += lambda;
    h -= v;
    g.Hs[row * NP + col] = h;
    if (I != J) g.Hs[(long long)col * NP + row] = h;
}

// Dense Cholesky of the n6 x n6 Schur matrix + forward / back substitution (replaces
// LinearSolverEigen's SimplicialLDLT, linear_solver_eigen.h:94-124; a non-positive pivot ->
// ok = 0 and the LM trial is rejected, optimization_algorithm_levenberg.cpp:126-127).
//
// n6 <= kSmallNP: the Schur system [Hs bs; bs^T 0] (the right-hand side appended as row n,
// padded to N2 = 16 * ceil((n + 1) / 16) with identity rows) factored in LDS by one
// 512-thread workgroup, right-looking over 16-column panels:
//   1. wave 0 factors the 16 x 16 diagonal tile in registers (lane i = row i; L[c][j] and the
//      pivot are DPP row broadcasts, one reciprocal square root per column) and inverts it
//      (lane c = column c of L_kk^-1, kept in LDS for the back substitution);
//   2. the panel below, L_ik = A_ik L_kk^-T, on FP64 MFMA (v_mfma_f64_16x16x4f64), one wave
//      per 16-row tile;
//   3. the trailing lower tiles A_ij -= L_ik L_jk^T on FP64 MFMA, one wave per tile.
// The appended row comes out as y^T with L y = bs (forward substitution for free); the back
// substitution L^T x = y runs block by block: x_K = L_KK^-T y_K (wave 0), then every earlier
// row subtracts L_K^T x_K in parallel. Rows >= n are treated as unit pivots. 3 barriers per
// panel + 2 per back-substitution block.
// The 16 x 16 diagonal tile: lane i of each 16-lane row holds row i of the tile and column i of
// L_kk^-1; pivot J's column is broadcast by DPP64 row_newbcast, scaled by v_rsq_f64 + one Newton
// step (the near-singular windows of tests/test_lba_gpu.py::test_lba_near_singular, pivot ratios
// down to 2e-5, keep the oracle's LM path) and subtracted from the later columns with
// v_fmac_f64_dpp. chol16_pipe is straight-line code generated by tools/gen_chol16.py (pivot J's
// non-critical updates placed between the dependent steps of pivot J + 1's chain, wait states
// written out): 3108 -> 2416 cycles a tile against the compiler-scheduled form
// (profiles/r05_chol16_bench.txt).
#include "lba_chol16.inc"

// The trial poses T_t = exp(x_p) T of the free poses (VertexSE3Expmap::oplusImpl) of a window
// beyond lba_chol_tiled's, formed at the end of the blocked solve into the trial estimate buffer
// (lba_lin_points<true> forms a small window's itself). Tc: the current pose of free pose t.
__device__ __forceinline__ void trial_pose(const Graph &g, bool cur, int t, const Pose &Tc, const double *xp) {
    Pose *Tt = cur ? g.T : g.T2;
    Tt[g.hpose[t]] = pose_oplus(Tc, xp + 6 * t);
}

__host__ __device__ constexpr int chol_tiled_dim(int n) { return 16 * ((n + 16) / 16); }
__host__ __device__ constexpr size_t chol_tiled_lds(int n) {
    return sizeof(double) * ((size_t)chol_tiled_dim(n) * (chol_tiled_dim(n) + 1) + (size_t)(chol_tiled_dim(n) / 16) * 16 * 17 +
                             2 * (size_t)chol_tiled_dim(n));
}

// the sum of x over the 4 lanes of a quad, (l0 + l1) + (l2 + l3) in every lane, by DPP quad_perm
template <int CTL> __device__ __forceinline__ double dpp_perm64(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)b, CTL, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(b >> 32), CTL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double quad_sum(double x) {
    x += dpp_perm64<0xB1>(x);          // quad_perm [1, 0, 3, 2]: lane ^ 1
    return x + dpp_perm64<0x4E>(x);    // quad_perm [2, 3, 0, 1]: lane ^ 2
}
// the sum of x over the four 16-lane rows, in every lane: two swap steps on the VALU
// (v_permlane16_swap: odd rows of the first operand <-> even rows of the second; v_permlane32_swap:
// the upper half <-> the lower half), each lane adding its pair in the same order, so every row
// holds the same bits (r0 + r1) + (r2 + r3)
__device__ __forceinline__ double rows4_sum(double x) {
    auto step = [](double v, bool half) -> double {
        const unsigned lo = (unsigned)__double_as_longlong(v), hi = (unsigned)(__double_as_longlong(v) >> 32);
        const auto a = half ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false) : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto b = half ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false) : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        const double u = __longlong_as_double((long long)(((unsigned long long)b[0] << 32) | a[0]));
        const double w = __longlong_as_double((long long)(((unsigned long long)b[1] << 32) | a[1]));
        return u + w;
    };
    return step(step(x, false), true);
}
// 1024 threads: 84k cycles per 120 x 120 solve against 87k for 512 (faster load phase)
constexpr int kCT = 1024, kCW = kCT / 64;   // threads, waves of lba_chol_tiled
constexpr unsigned kSpinLimit = 1u << 24;   // bounded hand-off wait (~1 s of polls): Graph::spin_limit's default
// HANDOFF: the Schur matrix Hs comes from the finish blocks of the same launch (lba_finish_chol):
// they store it write-through (sc1) and add to g.arrive[0] after their stores have drained; thread
// 0 polls that counter, the workgroup barrier orders every wave's loads after the match, and every
// load of Hs is an sc1 load -- MI355X_MICROARCH.md's valid hand-off form that replaces the release /
// acquire pair (an agent-scope release here writes back L2: 20.5 us per trial measured);
// the memory clobber of the producer's `s_waitcnt vmcnt(0)` keeps the compiler from moving its
// stores past the counter add. tests/test_lba_gpu.py::test_lba_fused_finish_bit_identical runs the
// fused and the two-launch path (lba_set_test_option) and requires identical outputs.
// A wait that exceeds g.spin_limit polls records a fault in g.arrive[1] and abandons the trial; the
// next LM decision turns it into LMState::fault (done), and lba_solve returns ORBX_EDEVICE.
template <bool HANDOFF> __device__ __forceinline__ void chol_tiled_body(Graph &g, int nfb) {
    extern __shared__ double A[];   // N2 x LDA, then Linv[NT][16][17], y[N2], x[N2]
    __shared__ int fail, tmo;
    if (g.lm->done) return;
    if constexpr (HANDOFF) {
        if (threadIdx.x == 0) {
            unsigned spins = 0;
            int to = g.spin_limit == 0;   // 0: fault injection (lba_set_test_option), every wait times out
            while (!to && __hip_atomic_load(g.arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nfb) {
                if (++spins >= g.spin_limit) { to = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (to) {   // late finish blocks still add to arrive[0]: it is left alone (every later launch of
                        // the call is a no-op once the fault is decided; lba_solve's setup zeroes it)
                __hip_atomic_store(g.arrive + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                g.scalars[4] = 0;
            } else {
                __hip_atomic_store(g.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // for the next launch
            }
            tmo = to;
        }
        __syncthreads();
        if (tmo) return;   // uniform
    }
    const int n = 6 * g.P, N2 = chol_tiled_dim(n), NT = N2 / 16, LDA = N2 + 1;
    double *Linv = A + N2 * LDA, *yv = Linv + NT * 16 * 17, *xv = yv + N2;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#ifdef LBA_PROFILE
    long long t_diag = 0, t_trsm = 0, t_trail = 0, t0 = clock64(), ta;
#define LBA_T(acc) do { __syncthreads(); const long long tb = clock64(); acc += tb - ta; ta = tb; } while (0)
#else
#define LBA_T(acc) do {} while (0)
#endif
    const long long NP = g.NP;
    // element (r, c <= r) of the system [Hs bs; bs^T 0] padded with identity rows, branch-free: Hs and
    // bs through buffer descriptors over exactly their n rows / n entries, every other offset past
    // the descriptor's end (the hardware returns 0), so all of a lane's loads stay in flight together
    // (with a branch per case the compiler waited vmcnt(0) before each load: a round trip per element).
    // HANDOFF: the Hs loads carry sc1 (aux 16), the hand-off's load form (MI355X_MICROARCH.md, row 1)
    const auto hs_rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)g.Hs, 0, (int)(n * NP * 8), 0x00020000);
    const auto bs_rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)g.bs, 0, n * 8, 0x00020000);
    constexpr int kOOR = 0x40000000;   // an offset past both descriptors
    // sys_ld issues the two loads of element (r, c) -- zero unless `ok` -- and sys_val sums them once
    // they are needed (at most one term is nonzero), so a caller issues all of its loads first
    auto sys_ld = [&](int r, int c, bool ok, double &h, double &b) {
        h = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(hs_rsrc, ok && r < n ? (r * (int)NP + c) * 8 : kOOR, 0,
                                                                            HANDOFF ? 16 : 0));
        b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(bs_rsrc, ok && r == n ? c * 8 : kOOR, 0, 0));
    };
    auto sys_val = [&](int r, int c, bool ok, double h, double b) -> double { return h + b + (ok && r > n && r == c ? 1.0 : 0.0); };
    if (tid == 0) fail = 0;
#ifdef LBA_PROFILE
    __shared__ long long prof_d[2];
#endif
    // wave 0: factor + invert diagonal tile K (lane i of each 16-lane row = row i); wave 0 loads tile
    // 0 itself while waves 1.. load the rest of the matrix into LDS
    auto diag = [&](int K) {
        const int k0 = 16 * K, i = lane & 15;
        double *LK = Linv + K * 16 * 17;
        double row[16], li[16];   // li: column i of L_kk^-1
        if (K == 0) {
            // tile 0 through LDS: each load covers 4 rows x 16 columns (a row per 16-lane row), 4 loads
            // per lane (row i per lane straight from global memory was 16 loads of 16 lines each, and
            // the hand-off's sc1 loads all miss L2: 7.6k cycles against 4.5k for the rest of the matrix)
            double hb[4][2];
            const int cc = lane & 15;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = (lane >> 4) + 4 * q;
                sys_ld(r, cc, cc <= r, hb[q][0], hb[q][1]);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = (lane >> 4) + 4 * q;
                if (cc <= r) A[r * LDA + cc] = sys_val(r, cc, true, hb[q][0], hb[q][1]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // this wave's LDS stores before its reads
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        {
#pragma unroll
            for (int c = 0; c < 16; c++) row[c] = A[(k0 + i) * LDA + k0 + c];   // the upper part (never written:
            // any bits) only ever meets lane i's own columns > i, which no broadcast reads
        }
#ifdef LBA_PROFILE
        long long pa = 0, pb = 0;
        if (K == 0) {
#pragma unroll
            for (int c = 0; c < 16; c++) asm volatile("" : "+v"(row[c]));
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            pa = clock64();
        }
#endif
#pragma unroll
        for (int r = 0; r < 16; r++) li[r] = r == i ? 1.0 : 0.0;
        bool bad = false;
        chol16_pipe(row, li, n - k0, bad);
#ifdef LBA_PROFILE
        if (K == 0) {
#pragma unroll
            for (int c = 0; c < 16; c++) asm volatile("" : "+v"(row[c]), "+v"(li[c]));
            pb = clock64();
            if (lane == 0) { prof_d[0] = pa - t0; prof_d[1] = pb - pa; }
        }
#endif
        // every 16-lane row computed the same tile: all lanes store (same values), so the
        // compiler cannot sink the li chain into a lane < 16 branch and keep every broadcast
        // live until there
#pragma unroll
        for (int c = 0; c < 16; c++) A[(k0 + i) * LDA + k0 + c] = row[c];
#pragma unroll
        for (int r = 0; r < 16; r++) LK[r * 17 + i] = li[r];
        if (lane == 0 && bad) fail = 1;
    };
#ifdef LBA_PROFILE
    __shared__ long long prof_w[2];
#endif
    if (wv == 0) {
        diag(0);
#ifdef LBA_PROFILE
        if (lane == 0) prof_w[0] = clock64() - t0;
#endif
    } else {   // waves 1..: the lower triangle of rows 16.. (N2 <= kSmallNP = 128), all loads in flight
        constexpr int RU = (128 - 16 + kCW - 2) / (kCW - 1);
        double v[RU][2][2];
#pragma unroll
        for (int u = 0; u < RU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int r = 16 + wv - 1 + (kCW - 1) * u, c = lane + 64 * h;
                sys_ld(r, c, r < N2 && c <= r, v[u][h][0], v[u][h][1]);
            }
#pragma unroll
        for (int u = 0; u < RU; u++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int r = 16 + wv - 1 + (kCW - 1) * u, c = lane + 64 * h;
                if (r < N2 && c <= r) A[r * LDA + c] = sys_val(r, c, true, v[u][h][0], v[u][h][1]);
            }
#ifdef LBA_PROFILE
        if (tid == 64) prof_w[1] = clock64() - t0;
#endif
    }
    __syncthreads();
#ifdef LBA_PROFILE
    const long long t_load = prof_w[0] * 1000000LL + prof_w[1];   // wave 0's diag(0) | wave 1's load, cycles
    if (tid == 0) printf("LBAPROF0 loads %lld factor %lld w0 %lld w1 %lld\n", prof_d[0], prof_d[1], prof_w[0], prof_w[1]);
    ta = t0;
#endif
    LBA_T(t_diag);
    // look-ahead: diagonal tile K + 1 is factored by wave 0 right after its own trailing
    // update, while waves 1-7 update the rest of the trailing matrix; 2 barriers per panel
    for (int K = 0; K < NT; K++) {
        if (fail) {   // uniform after the barrier
            if (tid == 0) g.scalars[4] = 0;
            return;
        }
        const int k0 = 16 * K, r0 = k0 + 16, m = NT - K - 1;
        const double *LK = Linv + K * 16 * 17;
        for (int I = wv; I < m; I += kCW) {   // panel: L_ik = A_ik L_kk^-T
            const int ri = r0 + 16 * I;
            double4_t acc = {0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 16; kk += 4) {
                const double a = A[(ri + (lane & 15)) * LDA + k0 + kk + (lane >> 4)];
                const double b = LK[(lane & 15) * 17 + kk + (lane >> 4)];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) A[(ri + (lane >> 4) + 4 * q) * LDA + k0 + (lane & 15)] = acc[q];
        }
        __syncthreads();
        LBA_T(t_trsm);
        if (m == 0) break;
        const int ntile = m * (m + 1) / 2;
        // trailing lower tiles; tile 0 = diagonal tile K + 1 -> wave 0, the rest -> the other waves
        for (int t = wv == 0 ? 0 : wv; t < ntile; t += wv == 0 ? ntile : kCW - 1) {
            int I = 0, u = t;
            while (u > I) { u -= I + 1; I++; }
            const int J = u;
            const int ri = r0 + 16 * I, cj = r0 + 16 * J;
            double4_t acc;
#pragma unroll
            for (int q = 0; q < 4; q++) acc[q] = A[(ri + (lane >> 4) + 4 * q) * LDA + cj + (lane & 15)];
#pragma unroll
            for (int kk = 0; kk < 16; kk += 4) {
                const double a = -A[(ri + (lane & 15)) * LDA + k0 + kk + (lane >> 4)];
                const double b = A[(cj + (lane & 15)) * LDA + k0 + kk + (lane >> 4)];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) A[(ri + (lane >> 4) + 4 * q) * LDA + cj + (lane & 15)] = acc[q];
        }
        if (wv == 0) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // own tile stores before reloading it
            diag(K + 1);
        }
        __syncthreads();
        LBA_T(t_trail);
    }
#ifdef LBA_PROFILE
    const long long ts = clock64();
#endif
    // back substitution L^T x = y, y = row n of the factor, zero past n: the padded rows of
    // the last block then contribute exactly 0 and every block runs fixed 16-term sums
    for (int j = tid; j < N2; j += kCT) yv[j] = j < n ? A[n * LDA + j] : 0.0;
    __syncthreads();
    // Each block step as 4-term partial dot products reduced across lanes (a 16-term dependent
    // FMA chain per step before): x_K by wave 0, lane (column c, quarter p) over rows 4p..4p+3;
    // the rows above by 4 lanes each
    static_assert(kCT / 4 >= kSmallNP, "one pass of row quads");
    // x_K = L_KK^-T y_K on wave 0 (y_K final in yv); the quarter sums added (r0 + r1) + (r2 + r3)
    auto x_block = [&](int K) {
        const int k0 = 16 * K;
        const double *LK = Linv + K * 16 * 17;
        const int c = lane & 15, p4 = 4 * (lane >> 4);
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) s += LK[(p4 + r) * 17 + c] * yv[k0 + p4 + r];   // LK[r][c] = 0 for r < c
        s = rows4_sum(s);
        if (lane < 16) xv[k0 + c] = s;
    };
    // y_j -= L_K^T x_K for row j, by the 4 lanes of a quad (k = 4p .. 4p + 3 each, summed (p0 + p1) + (p2 + p3))
    auto y_update = [&](int k0, int j, int q4) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) s += A[(k0 + q4 + k) * LDA + j] * xv[k0 + q4 + k];
        s = quad_sum(s);
        if ((lane & 3) == 0) yv[j] -= s;
    };
    // One barrier per block: with x_K published, wave 0 updates block K - 1's rows itself and forms
    // x_{K-1} at once (its own LDS accesses are ordered), while waves 1.. update the rows above
    // block K - 1; the barrier then publishes x_{K-1} and those rows. The same sums in the same
    // order as a two-barrier form (x_K, barrier, rows, barrier), so the solution is bit-identical to it.
    {
        int K = (n - 1) / 16;
        if (wv == 0) x_block(K);
        __syncthreads();
        for (; K > 0; K--) {
            const int k0 = 16 * K, kp = k0 - 16;
            if (wv == 0) {
                y_update(k0, kp + (lane >> 2), 4 * (lane & 3));
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // block K - 1's y before x_block reads it
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                x_block(K - 1);
            } else {
                const int j = (tid - 64) >> 2;
                if (j < kp) y_update(k0, j, 4 * (tid & 3));   // a row's 4 lanes are a quad: all in or all out
            }
            __syncthreads();
        }
    }
    for (int j = tid; j < n; j += kCT) g.x[j] = xv[j];
    if (tid == 0) g.scalars[4] = 1;
#ifdef LBA_PROFILE
    if (tid == 0)
        printf("LBAPROF n=%d load=%lld diag=%lld trsm=%lld trail=%lld solve=%lld\n", n, t_load, t_diag, t_trsm, t_trail,
               clock64() - ts);
#endif
}

__global__ __launch_bounds__(kCT) void lba_chol_tiled(Graph g) { chol_tiled_body<false>(g, 0); }

// order a wavefront's LDS writes before its reads (LDS executes a wave's ops in order)
__device__ __forceinline__ void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// 6P > kSmallNP: the Schur system [Hs bs; bs^T 0] factored by one 1024-thread workgroup with the
// matrix in a global work buffer g.W (N2 x N2, lower tiles, L2-resident) instead of LDS: a window of
// 22-88 free keyframes (132 <= 6P <= 528) gets the same one-launch trial tail as a small one (the
// blocked path before: two launches per 32-column panel, 21 launches per trial at 40 free keyframes,
// 0.68 ms per trial). chol_tiled_body's tiles and arithmetic, with the trailing update over two
// 16-column panels per pass (one read-modify-write of a tile per 32 columns: the pass is bound by the
// CU's memory and LDS bandwidth, profiles/r06_lbaprof_global*.txt):
//   * columns K, K + 1 (K even): (B) the panel below L_IK = A_IK L_KK^-T on FP64 MFMA, into W and the
//     LDS panel copy Pc[0]; (C) column K + 1 updated by panel K -- wave 0 takes the diagonal tile
//     (K + 1, K + 1) into LDS (Dt) and factors it (chol16_pipe), the other waves store the rest; (D)
//     its panel L_{I,K+1} into W and Pc[1]; (E) the trailing lower tiles A_IJ -= L_IK L_JK^T +
//     L_{I,K+1} L_{J,K+1}^T (8 MFMAs, operands from Pc) read-modify-write in W, four tiles' loads in
//     flight per wave, wave 0 taking (K + 2, K + 2) into Dt and factoring it;
//   * the first pass (K = 0) reads the handed-over Hs / bs (+ identity rows) directly, so no copy of
//     the system into W; the diagonal tile's factor goes to W (its row n is part of y), its inverse to
//     g.W's inverse area;
//   * the back substitution block by block (chol_tiled_body's, with the inverses copied back into LDS
//     and every row update's W loads issued one block ahead), then the trial poses T_t = exp(x_p) T
//     (lba_lin_points reads them for a large window).
// LDS: Pc [2][N2][17] (after the factor: the inverses [NT][16][17]) | LKs [16][17] | Dt [16][17] | y | x.
__host__ __device__ constexpr size_t chol_global_lds(int n) {
    return sizeof(double) * (2 * (size_t)chol_tiled_dim(n) * 17 + 2 * 16 * 17 + 2 * (size_t)chol_tiled_dim(n));
}
constexpr int kBigNP = 528;   // 6 * 88 free poses: chol_global_lds(528) + the static LDS <= 160 KB
static_assert(chol_global_lds(kBigNP) + 64 <= 160 * 1024, "chol_global_body's LDS");
__host__ __device__ constexpr size_t chol_global_w(int n) {   // doubles of g.W: the matrix, then the inverses
    return (size_t)chol_tiled_dim(n) * chol_tiled_dim(n) + (size_t)(chol_tiled_dim(n) / 16) * 256;
}

template <bool HANDOFF> __device__ __forceinline__ void chol_global_body(Graph &g, int nfb) {
    extern __shared__ double A[];
    __shared__ int fail, tmo;
    if (g.lm->done) return;
    if constexpr (HANDOFF) {   // as chol_tiled_body
        if (threadIdx.x == 0) {
            unsigned spins = 0;
            int to = g.spin_limit == 0;
            while (!to && __hip_atomic_load(g.arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nfb) {
                if (++spins >= g.spin_limit) { to = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (to) {
                __hip_atomic_store(g.arrive + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                g.scalars[4] = 0;
            } else {
                __hip_atomic_store(g.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            tmo = to;
        }
        __syncthreads();
        if (tmo) return;
    }
    const int n = 6 * g.P, N2 = chol_tiled_dim(n), NT = N2 / 16;
    const long long LDW = g.LDW;
    // W and, past it, Lg ([NT][16][16] inverses of the diagonal tiles) through one buffer descriptor with
    // 32-bit element offsets: 64-bit addresses hoisted out of the panel loop spilled VGPRs
    const auto w_rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)g.W, 0, (int)(8 * chol_global_w(n)), 0x00020000);
    const int LG = N2 * (int)LDW;
    auto wld = [&](int e) { return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(w_rsrc, 8 * e, 0, 0)); };
    typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
    auto wst = [&](int e, double v) { __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), w_rsrc, 8 * e, 0, 0); };
    double *Pc0 = A, *Pc1 = A + N2 * 17, *LKs = Pc1 + N2 * 17, *Dt = LKs + 16 * 17, *yv = Dt + 16 * 17, *xv = yv + N2;
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform
    int lr = lane & 15, lq = lane >> 4;   // MFMA operand row / k quarter; C layout: row lq + 4q, column lr
#ifdef LBA_PROFILE
    const long long tg0 = clock64();
    long long tgf = 0, tgb = 0, tgc = 0, tgd = 0, tge = 0, tgx;
#define LBA_TG(acc) do { acc += clock64() - tgx; tgx = clock64(); } while (0)
#else
#define LBA_TG(acc) do {} while (0)
#endif
    const long long NP = g.NP;
    const auto hs_rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)g.Hs, 0, (int)(n * NP * 8), 0x00020000);
    constexpr int kOOR = 0x40000000;
    // bs, the system's row n, staged in LDS (the y area, unused until the back substitution)
    for (int j = tid; j < n; j += kCT) yv[j] = g.bs[j];
    // element (r, c <= r) of the system: the handed-over Hs (sc1 loads; 0 past row n - 1), bs as row n
    // (from LDS), identity past it
    auto hs_ld = [&](int r, int c, bool ok) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(hs_rsrc, ok && r < n ? (r * (int)NP + c) * 8 : kOOR,
                                                                               0, HANDOFF ? 16 : 0));
    };
    auto hs_val = [&](int r, int c, bool ok, double h) -> double {
        return h + (ok && r == n ? yv[c] : 0.0) + (ok && r > n && r == c ? 1.0 : 0.0);
    };
    // the 16 x 16 tile at (r0, c0) in C layout: from Hs (first pass) or from W
    auto tile_ld = [&](bool hs, int r0, int c0, double (&v)[4]) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = r0 + lq + 4 * q, c = c0 + lr;
            v[q] = hs ? hs_ld(r, c, c <= r) : wld(r * (int)LDW + c);
        }
    };
    auto tile_val = [&](bool hs, int r0, int c0, const double (&v)[4]) {
        double4_t acc;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = r0 + lq + 4 * q, c = c0 + lr;
            acc[q] = hs ? hs_val(r, c, c <= r, v[q]) : v[q];
        }
        return acc;
    };
    auto tile_st = [&](int r0, int c0, const double4_t &acc) {
#pragma unroll
        for (int q = 0; q < 4; q++) wst((r0 + lq + 4 * q) * (int)LDW + c0 + lr, acc[q]);
    };
    auto dt_st = [&](const double4_t &acc) {
#pragma unroll
        for (int q = 0; q < 4; q++) Dt[(lq + 4 * q) * 17 + lr] = acc[q];
    };
    // acc -= P_I P_J^T for panel cache P (rows ri, cj of the tile pair)
    auto mm = [&](const double *P, int ri, int cj, double4_t acc) {
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-P[(ri + lr) * 17 + 4 * kk + lq], P[(cj + lr) * 17 + 4 * kk + lq], acc, 0, 0, 0);
        return acc;
    };
    // wave 0: factor + invert the diagonal tile K held in Dt (lane i of each 16-lane row = row i): the
    // inverse into LKs and Lg, the factor's rows into W
    auto diag = [&](int K) {
        const int k0 = 16 * K, i = lr;
        lds_wave_sync();
        double row[16], li[16];
#pragma unroll
        for (int c = 0; c < 16; c++) row[c] = Dt[i * 17 + c];
        // the unit column formed here, from a value the compiler cannot hoist (hoisted out of the panel
        // loop, e_i stayed live across it and spilled 145 VGPRs)
        double one = 1.0;
        asm volatile("" : "+v"(one));
#pragma unroll
        for (int r = 0; r < 16; r++) li[r] = r == i ? one : 0.0;
        bool bad = false;
        chol16_pipe(row, li, n - k0, bad);
#pragma unroll
        for (int r = 0; r < 16; r++) LKs[r * 17 + i] = li[r];
        if (lane < 16) {
#pragma unroll
            for (int r = 0; r < 16; r++) wst(LG + K * 256 + r * 16 + i, li[r]);
#pragma unroll
            for (int c = 0; c < 16; c++) wst((k0 + i) * (int)LDW + k0 + c, row[c]);
        }
        if (lane == 0 && bad) fail = 1;
    };
    // panel of column K: L_IK = A_IK L_KK^-T for tiles I > K (A from Hs in the first pass), into W and P
    auto panel = [&](int K, bool hs, double *P) {
        const int k0 = 16 * K;
        for (int I = K + 1 + wv; I < NT; I += kCW) {
            const int ri = 16 * I;
            double a[4];
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const int r = ri + lr, c = k0 + 4 * kk + lq;
                a[kk] = hs ? hs_ld(r, c, true) : wld(r * (int)LDW + c);
            }
            double4_t acc = {0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const double av = hs ? hs_val(ri + lr, k0 + 4 * kk + lq, true, a[kk]) : a[kk];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, LKs[lr * 17 + 4 * kk + lq], acc, 0, 0, 0);
            }
            tile_st(ri, k0, acc);
#pragma unroll
            for (int q = 0; q < 4; q++) P[(ri + lq + 4 * q) * 17 + lr] = acc[q];
        }
    };
    if (tid == 0) fail = 0;
    __syncthreads();   // bs in LDS
    // tile (0, 0) from Hs into Dt, factored by wave 0
    if (wv == 0) {
        double v[4];
        tile_ld(true, 0, 0, v);
        dt_st(tile_val(true, 0, 0, v));
        diag(0);
    }
    __syncthreads();
#ifdef LBA_PROFILE
    tgf = clock64() - tg0;
    tgx = clock64();
#endif
    // one pass over columns K, K + 1; hs: the first pass, A from the handed-over system. Returns 1 when the factorization is complete, -1 on a non-positive pivot.
    auto pass = [&](int K, bool hs) -> int {
        {   // the lane indices re-derived from an opaque copy: the offsets built from them are formed per pass
            // instead of hoisted out of the loop and kept live (spilled) across it
            int l = lane;
            asm volatile("" : "+v"(l));
            lr = l & 15;
            lq = l >> 4;
        }
        panel(K, hs, Pc0);   // (B)
        __syncthreads();
        LBA_TG(tgb);
        if (K + 1 >= NT) return 1;
        {   // (C) column K + 1 by panel K: wave 0 the diagonal tile (into Dt, factored), the others the rest
            const int k1 = 16 * (K + 1);
            for (int I = K + 1 + wv; I < NT; I += kCW) {
                const int ri = 16 * I;
                double v[4];
                tile_ld(hs, ri, k1, v);
                const double4_t acc = mm(Pc0, ri, k1, tile_val(hs, ri, k1, v));
                if (I == K + 1) dt_st(acc);
                else tile_st(ri, k1, acc);
            }
            if (wv == 0) diag(K + 1);
        }
        __syncthreads();
        LBA_TG(tgc);
        if (fail) return -1;
        panel(K + 1, false, Pc1);   // (D)
        __syncthreads();
        LBA_TG(tgd);
        const int m = NT - K - 2;
        if (m <= 0) return 1;
        // (E) the trailing tiles (I, J), K + 2 <= J <= I: tile 0 = (K + 2, K + 2) -> wave 0 (Dt, factored),
        // the others -> waves 1.., four tiles' loads in flight per batch
        const int r0 = 16 * (K + 2);
        if (wv == 0) {
            double v[4];
            tile_ld(hs, r0, r0, v);
            dt_st(mm(Pc1, r0, r0, mm(Pc0, r0, r0, tile_val(hs, r0, r0, v))));
            diag(K + 2);
        } else {
            const int ntile = m * (m + 1) / 2;
            auto tile_of = [](int t, int &I, int &J) {   // lower tile t of the triangle (row-major, I >= J)
                int i = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
                if ((i + 1) * (i + 2) / 2 <= t) i++;
                if (i * (i + 1) / 2 > t) i--;
                I = i;
                J = t - i * (i + 1) / 2;
            };
            // four tiles' loads in flight per wave: six or eight measured slower (E 354k -> 368k / 380k cycles
            // at 6P = 384, profiles/r06_lbaprof_global_*.txt); so did rows of four tiles per wave sharing their
            // A fragments (485k: fewer tiles in flight)
            constexpr int TB = 4;
            for (int t0 = wv; t0 < ntile; t0 += TB * (kCW - 1)) {
                double v[TB][4];
                int It[TB], Jt[TB];
#pragma unroll
                for (int u = 0; u < TB; u++) {
                    const int t = t0 + u * (kCW - 1);
                    It[u] = Jt[u] = 0;
                    if (t < ntile) tile_of(t, It[u], Jt[u]);
                    tile_ld(hs && t < ntile, r0 + 16 * It[u], r0 + 16 * Jt[u], v[u]);
                }
#pragma unroll
                for (int u = 0; u < TB; u++) {
                    const int t = t0 + u * (kCW - 1);
                    if (t >= ntile) continue;
                    const int ri = r0 + 16 * It[u], cj = r0 + 16 * Jt[u];
                    tile_st(ri, cj, mm(Pc1, ri, cj, mm(Pc0, ri, cj, tile_val(hs, ri, cj, v[u]))));
                }
            }
        }
        __syncthreads();
        LBA_TG(tge);
        return 0;
    };
    for (int K = 0;; K += 2) {
        if (fail) {   // uniform after the barrier
            if (tid == 0) g.scalars[4] = 0;
            return;
        }
        const int st = pass(K, K == 0);
        if (st < 0) {
            if (tid == 0) g.scalars[4] = 0;
            return;
        }
        if (st > 0) break;
    }
#ifdef LBA_PROFILE
    const long long tg2 = clock64();
    long long tgs1 = 0;
#endif
    // back substitution L^T x = y (chol_tiled_body's): the inverses back into LDS (over the panel copies)
    double *Linv = A;
    for (int e = tid; e < NT * 256; e += kCT) {
        const int K = e >> 8, r = (e >> 4) & 15, c = e & 15;
        Linv[K * 272 + r * 17 + c] = wld(LG + e);
    }
    for (int j = tid; j < N2; j += kCT) yv[j] = j < n ? wld(n * (int)LDW + j) : 0.0;
    __syncthreads();
    auto x_block = [&](int K) {
        const int k0 = 16 * K;
        const double *LK = Linv + K * 272;
        const int c = lr, p4 = 4 * lq;
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) s += LK[(p4 + r) * 17 + c] * yv[k0 + p4 + r];
        s = rows4_sum(s);
        if (lane < 16) xv[k0 + c] = s;
    };
    // y_j -= L_K^T x_K by the 4 lanes of a quad; the W values of the row (loaded a block ahead)
    auto y_apply = [&](int k0, int j, int q4, const double (&wr)[4]) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 4; k++) s += wr[k] * xv[k0 + q4 + k];
        s = quad_sum(s);
        if ((lane & 3) == 0) yv[j] -= s;
    };
    auto w_ld = [&](int k0, int j, int q4, bool ok, double (&wr)[4]) {
#pragma unroll
        for (int k = 0; k < 4; k++)   // !ok: an offset past the descriptor's end (the load returns 0), no branch
            wr[k] = wld(((k0 + q4 + k) * (int)LDW + j) | (ok ? 0 : 0x08000000));
    };
    {
        constexpr int NJ = 3;   // rows per thread of waves 1..15: (kBigNP + 15) / 240 + 1
        static_assert((kCT - 64) / 4 * NJ >= kBigNP + 16, "rows of the back substitution");
        const int q4w = 4 * (lane & 3), q4o = 4 * (tid & 3), j0 = (tid - 64) >> 2;
        const int K0 = (n - 1) / 16;
        struct WRows { double v[NJ][4]; };   // the W rows one block's update reads (a value: stays in registers)
        auto issue = [&](int K) __attribute__((always_inline)) {
            WRows wr;
            if (K <= 0) return wr;
            const int k0 = 16 * K, kp = k0 - 16;
            if (wv == 0) w_ld(k0, kp + (lane >> 2), q4w, true, wr.v[0]);
            else
#pragma unroll
                for (int u = 0; u < NJ; u++) w_ld(k0, j0 + 240 * u, q4o, j0 + 240 * u < kp, wr.v[u]);
            return wr;
        };
        // block K (x_K published): rows of block K - 1 and x_{K-1} by wave 0, the rows above by the others
        auto step = [&](int K, WRows wr) __attribute__((always_inline)) {
            const int k0 = 16 * K, kp = k0 - 16;
            if (wv == 0) {
                y_apply(k0, kp + (lane >> 2), q4w, wr.v[0]);
                lds_wave_sync();
                x_block(K - 1);
            } else {
#pragma unroll
                for (int u = 0; u < NJ; u++)
                    if (j0 + 240 * u < kp) y_apply(k0, j0 + 240 * u, q4o, wr.v[u]);
            }
            // LDS-only barrier (fences scoped to LDS): __syncthreads() would also wait for the next
            // block's W loads in flight (vmcnt counts loads and stores alike); the solve reads W only
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        };
        WRows wa = issue(K0);
        if (wv == 0) x_block(K0);
        __syncthreads();
#ifdef LBA_PROFILE
        tgs1 = clock64();
#endif
        // two blocks per iteration, the next block's rows loading while this one's are applied
        for (int K = K0; K > 0; K -= 2) {
            const WRows wb = issue(K - 1);
            step(K, wa);
            if (K - 1 <= 0) break;
            wa = issue(K - 2);
            step(K - 1, wb);
        }
    }
#ifdef LBA_PROFILE
    const long long tgs2 = clock64();
#endif
    for (int j = tid; j < n; j += kCT) g.x[j] = xv[j];
    const bool cur = g.lm->cur;
    for (int t = tid; t < g.P; t += kCT) trial_pose(g, cur, t, (cur ? g.T2 : g.T)[g.hpose[t]], xv);
    if (tid == 0) g.scalars[4] = 1;
#ifdef LBA_PROFILE
    if (tid == 0)
        printf("LBAPROFG n=%d diag0=%lld B=%lld C=%lld D=%lld E=%lld solve=%lld (setup %lld loop %lld poses %lld) total=%lld\n", n,
               tgf, tgb, tgc, tgd, tge, clock64() - tg2, tgs1 - tg2, tgs2 - tgs1, clock64() - tgs2, clock64() - tg0);
#endif
#undef LBA_TG
}

__global__ __launch_bounds__(kCT) void lba_chol_global(Graph g) { chol_global_body<false>(g, 0); }

// lba_schur_finish + lba_chol_tiled in one launch (one kernel boundary fewer per LM trial): blocks
// 0 .. nfb - 1 are finish blocks, four tile pairs each (one 4-wave quad per pair, lba_schur_finish's
// work), storing Hs write-through (sc1); after every wave's stores have drained and a workgroup
// barrier, one lane adds 1 to g.arrive[0]. Block nfb is the Cholesky (chol_tiled_body<true>), which
// waits for nfb arrivals. Every block is resident at once (nfb + 1 <= 10 blocks on 256 CUs), so the
// wait cannot block a producer.
template <bool BIG> __global__ __launch_bounds__(kCT) void lba_finish_chol(Graph g, int nfb) {
    if ((int)blockIdx.x == nfb) {
        if constexpr (BIG) chol_global_body<true>(g, nfb);
        else chol_tiled_body<true>(g, nfb);
        return;
    }
    if (g.lm->done) return;   // the Cholesky block reads the same flag and does not wait
    const int lane = threadIdx.x & 63, q = (threadIdx.x >> 6) & 3, p = 4 * (int)blockIdx.x + (int)(threadIdx.x >> 8);
    if (p < g.npairs) {
        const int2 ij = g.tp_ij[p], nc = g.tp_nch[p];   // (I, J); first chunk, chunk count
        const int I = ij.x, J = ij.y, n6 = 6 * g.P;
        const long long NP = g.NP;
        const double lambda = g.lm->lambda;
        double v = 0;
        const double *tp = g.tp_part + 256LL * nc.x + 64 * q + lane;
        for (int c0 = 0; c0 < nc.y; c0 += 32) {
            double t[32];
#pragma unroll
            for (int u = 0; u < 32; u++) t[u] = c0 + u < nc.y ? tp[256LL * (c0 + u)] : 0.0;
#pragma unroll
            for (int u = 0; u < 32; u++)
                if (c0 + u < nc.y) v += t[u];
        }
        // C/D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * q
        const int row = 16 * I + (lane >> 4) + 4 * q, col = 16 * J + (lane & 15);
        if (row < n6 && col < n6) {
            double h = 0;
            if (row / 6 == col / 6) h = g.Hpp[36 * (row / 6) + 6 * (row % 6) + (col % 6)];
            if (row == col) h += lambda;
            h -= v;
            const unsigned long long hb = (unsigned long long)__double_as_longlong(h);
            __hip_atomic_store((unsigned long long *)(g.Hs + row * NP + col), hb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (I != J)
                __hip_atomic_store((unsigned long long *)(g.Hs + (long long)col * NP + row), hb, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(g.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// n6 > kSmallNP: blocked right-looking Cholesky in place on Hs (lower triangle), panel
// width kCB = 32. Per panel kb: lba_chol_panel factors the diagonal block in LDS (every
// workgroup redundantly; workgroup 0 stores it) and solves 256 rows of the panel below it
// per workgroup (one thread per row, forward substitution against L_kk); lba_chol_update
// subtracts L_panel L_panel^T from the trailing lower tiles on FP64 MFMA (one wave per
// 16 x 16 tile, K = 32 = 8 x v_mfma_f64_16x16x4f64).
__global__ __launch_bounds__(256) void lba_chol_panel(Graph g, int kb) {
    __shared__ double D[kCB][kCB + 1];
    if (g.lm->done) return;
    const int n = 6 * g.P, tid = threadIdx.x;
    const long long NP = g.NP;
    const int nb = min(kCB, n - kb);
    for (int t = tid; t < kCB * kCB; t += 256) {
        const int r = t >> 5, c = t & 31;
        D[r][c] = (r < nb && c < nb && c <= r) ? g.Hs[(kb + r) * NP + kb + c] : 0.0;
    }
    __syncthreads();
    for (int j = 0; j < nb; j++) {      // unblocked factor of the diagonal block
        const double d = D[j][j];       // uniform after the barrier
        if (!(d > 0)) {
            if (tid == 0 && blockIdx.x == 0) g.scalars[4] = 0;
            break;
        }
        const double ljj = sqrt(d);
        __syncthreads();
        if (tid > j && tid < nb) D[tid][j] /= ljj;
        if (tid == j) D[j][j] = ljj;
        __syncthreads();
        if (tid > j && tid < nb) {
            const double v = D[tid][j];
            for (int c = j + 1; c <= tid; c++) D[tid][c] -= v * D[c][j];
        }
        __syncthreads();
    }
    if (blockIdx.x == 0)
        for (int t = tid; t < kCB * kCB; t += 256) {
            const int r = t >> 5, c = t & 31;
            if (r < nb && c <= r) g.Hs[(kb + r) * NP + kb + c] = D[r][c];
        }
    const int row = kb + nb + blockIdx.x * 256 + tid;
    if (row >= n) return;
    double a[kCB];
    double *Ar = g.Hs + row * NP + kb;
#pragma unroll
    for (int c = 0; c < kCB; c++) a[c] = c < nb ? Ar[c] : 0.0;
#pragma unroll
    for (int c = 0; c < kCB; c++) {     // x L_kk^T = a  ->  forward substitution
        if (c < nb) {
            double v = a[c];
#pragma unroll
            for (int k = 0; k < c; k++) v -= a[k] * D[c][k];
            a[c] = v / D[c][c];
        }
    }
#pragma unroll
    for (int c = 0; c < kCB; c++) if (c < nb) Ar[c] = a[c];
}

__global__ __launch_bounds__(64) void lba_chol_update(Graph g, int kb, int ntile) {
    if (g.lm->done) return;
    // lower 16 x 16 tiles (I >= J) of the trailing matrix, rows / cols >= kb + kCB
    const int lane = threadIdx.x;
    int t = blockIdx.x, I = 0;
    while (t > I) { t -= I + 1; I++; }
    const int J = t;
    const long long NP = g.NP;
    const int base = kb + kCB;
    const double *la = g.Hs + (base + 16 * I + (lane & 15)) * NP + kb;
    const double *lb = g.Hs + (base + 16 * J + (lane & 15)) * NP + kb;
    double4_t acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < kCB; k += 4) {
        const int kk = k + (lane >> 4);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(la[kk], lb[kk], acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; r++) {
        const int row = base + 16 * I + (lane >> 4) + 4 * r, c = base + 16 * J + (lane & 15);
        if (c <= row) g.Hs[row * NP + c] -= acc[r];
    }
}

// triangular solves on the blocked factor: one 1024-thread workgroup, rhs in LDS; wave 0
// solves each 32-row diagonal block serially, then every thread updates the remaining rows.
__global__ __launch_bounds__(1024) void lba_chol_solve_blocked(Graph g) {
    extern __shared__ double y[];
    if (g.lm->done) return;
    const int n = 6 * g.P, tid = threadIdx.x;
    const long long NP = g.NP;
    const double *L = g.Hs;
    for (int i = tid; i < n; i += 1024) y[i] = g.bs[i];
    __syncthreads();
    for (int kb = 0; kb < n; kb += kCB) {
        const int nb = min(kCB, n - kb);
        if (tid < 64) {
            double v = tid < nb ? y[kb + tid] : 0.0;
            for (int k = 0; k < nb; k++) {
                const double yk = __shfl(v, k) / L[(kb + k) * NP + kb + k];
                if (tid == k) v = yk;
                else if (tid > k && tid < nb) v -= L[(kb + tid) * NP + kb + k] * yk;
            }
            if (tid < nb) y[kb + tid] = v;
        }
        __syncthreads();
        for (int r = kb + nb + tid; r < n; r += 1024) {
            double v = y[r];
            const double *Lr = L + r * NP + kb;
            for (int k = 0; k < nb; k++) v -= Lr[k] * y[kb + k];
            y[r] = v;
        }
        __syncthreads();
    }
    for (int kb = ((n - 1) / kCB) * kCB; kb >= 0; kb -= kCB) {
        const int nb = min(kCB, n - kb);
        if (tid < 64) {
            double v = tid < nb ? y[kb + tid] : 0.0;
            for (int k = nb - 1; k >= 0; k--) {
                const double xk = __shfl(v, k) / L[(kb + k) * NP + kb + k];
                if (tid == k) v = xk;
                else if (tid < k) v -= L[(kb + k) * NP + kb + tid] * xk;
            }
            if (tid < nb) y[kb + tid] = v;
        }
        __syncthreads();
        for (int r = tid; r < kb; r += 1024) {
            double v = y[r];
            for (int k = 0; k < nb; k++) v -= L[(kb + k) * NP + r] * y[kb + k];
            y[r] = v;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += 1024) g.x[i] = y[i];
    const bool cur = g.lm->cur;
    for (int t = tid; t < g.P; t += 1024) trial_pose(g, cur, t, (cur ? g.T2 : g.T)[g.hpose[t]], y);
}

__global__ void lba_set_ok(Graph g) {
    if (!g.lm->done) g.scalars[4] = 1;
}

// SparseOptimizer::terminate(): *_forceStopFlag (sparse_optimizer.h), read live from the mapped word
// the host keeps equal to the caller's pbStopFlag, or the deterministic test hook
__device__ inline bool stop_raised(const Graph &g, const LMState &s) {
    return __hip_atomic_load(g.stopf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u || s.trials >= s.stop_at;
}

// SparseOptimizer::optimize(iterations) start: lambda / nu / nBad reset (levenberg.cpp:66-72), and
// the loop's first `i < iterations && !terminate()` check (sparse_optimizer.cpp:376)
__global__ void lba_lm_init(Graph g, int iterations, int stop_at) {
    LMState s{};
    s.cur = g.lm->cur;   // which buffer holds the estimate carries over between optimize() calls
    s.ni = 2;
    s.iterations = iterations;
    s.newiter = 1;
    s.stop_at = stop_at;
    s.done = iterations <= 0;
    if (!s.done && stop_raised(g, s)) s.seen = s.done = 1;
    *g.lm = s;
}

// The second optimize()'s start, reading the first one's final state p1 on the device, so it can be
// enqueued behind the first one's chunk without a host round trip (lba_solve): `spec` and p1 not
// yet done -> deferred (every launch of the enqueued phase-2 chunk is a no-op, the host re-enqueues
// the phase after the first one's retries); bDoMore false -- pbStopFlag raised, or the test hook's
// trial reached in the first optimize() (Optimizer.cc:913-917) -> skipped; else lba_lm_init's reset
// and first terminate() check, with the estimate buffer carried over (p1->cur).
__global__ void lba_phase2_begin(Graph g, const LMState *p1, int iterations, int stop_at, int spec) {
    const LMState s1 = *p1;
    LMState s{};
    s.cur = s1.cur;
    s.ni = 2;
    s.iterations = iterations;
    s.newiter = 1;
    s.stop_at = stop_at;
    if (s1.fault) {
        s.done = 1;
        s.fault = 1;
    } else if (spec && !s1.done) {
        s.done = 1;
        s.gate = 1;
    } else if (__hip_atomic_load(g.stopf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u || s1.trials >= s1.stop_at) {
        s.done = 1;
        s.gate = 2;
    } else {
        s.done = iterations <= 0;
        if (!s.done && stop_raised(g, s)) s.seen = s.done = 1;
    }
    *g.lm = s;
}

// End of one LM trial (optimization_algorithm_levenberg.cpp:96-164 + the ORB-SLAM2 stop rule
// :155-161): wave 0 sums the update's computeScale block sums and the trial chi2 block sums,
// thread 0 decides and advances the state; an accepted trial becomes the current estimate by
// swapping the estimate buffers (LMState::cur).
// The decision's two sums (wave 0): the trial's computeScale block sums and chi2 block sums (nbt
// each, scalars[8..]) in a fixed order -- lane k: blocks k, k + 64, ... in order, then an xor
// butterfly (a serial sum on one thread was ~3 us on the trial's critical path)
__device__ inline void decide_sums(const Graph &g, int nbt, double *sums_s) {
    if (threadIdx.x < 64) {
        const int k = threadIdx.x;
        const double *pp = g.scalars + 8;
        double a = 0, b = 0;
        for (int i = k; i < nbt; i += 64) a += pp[i];
        for (int i = k; i < nbt; i += 64) b += pp[nbt + i];
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
            a += __shfl_xor(a, m);
            b += __shfl_xor(b, m);
        }
        if (k == 0) { sums_s[0] = a; sums_s[1] = b; }
    }
}

// End of one LM trial (optimization_algorithm_levenberg.cpp:96-164 + the ORB-SLAM2 stop rule
// :155-161) as a pure function of the state before it: rho, lambda / nu, the retry / new-iteration
// choice, nBad; an accepted trial becomes the current estimate by swapping the roles of the two
// estimate buffers (LMState::cur). currentChi at an iteration's first trial: the first
// iteration's comes from the linearisation (scalars[0], lba_prep_slots), every later one is the
// accepted trial's chi2 itself -- the value g2o's activeRobustChi2() recomputes there.
__device__ LMState lm_next(const Graph &g, LMState s, double sc_sum, double chi_sum) {
    const double *sc = g.scalars;
    if (g.arrive[1] != 0u) {   // written by an earlier launch of this call: every workgroup reads the same
        s.fault = 1;
        s.done = 1;
        return s;
    }
    if (s.qmax == 0) {
        if (s.it == 0) s.currentChi = sc[0];
        s.iniChi = s.currentChi;
    }
    const double tempChi = sc[4] != 0 ? chi_sum : DBL_MAX;
    double rho = s.currentChi - tempChi;
    const double scale = sc_sum + 1e-3;
    rho /= scale;
    int a = 0;
    if (rho > 0 && isfinite(tempChi)) {   // good step: discardTop
        double alpha = 1. - pow((2 * rho - 1), 3.0);
        alpha = fmin(alpha, 2. / 3.);
        s.lambda *= fmax(1. / 3., alpha);
        s.ni = 2;
        s.currentChi = tempChi;
        a = 1;
    } else {                               // bad step: pop
        s.lambda *= s.ni;
        s.ni *= 2;
    }
    s.qmax++;
    s.trials++;
    s.rho = rho;
    s.accepted = a;
    // pbStopFlag, read where g2o reads it: the trial loop's `rho < 0 && qmax < max && !terminate()`
    // (levenberg.cpp:149, evaluated only after a rejected trial) and the iteration loop's
    // `i < iterations && !terminate() && ok` (sparse_optimizer.cpp:376, before `ok`). The flag is
    // the snapshot lba_lin_points took at the end of this trial (scalars[6]): one value for every
    // workgroup of a deciding launch.
    const bool raised = sc[6] != 0.0 || s.trials >= s.stop_at;
    bool retry = false;
    if (rho < 0 && s.qmax < 10) {
        if (raised) s.seen = 1;
        else retry = true;
    }
    if (retry) {
        s.newiter = 0;                     // retry the same linearisation
    } else {
        s.it++;
        s.final_chi = s.currentChi;
        bool ok = true;
        if (s.qmax == 10 || rho == 0) ok = false;
        else {
            if ((s.iniChi - s.currentChi) * 1e3 < s.iniChi) s.nBad++; else s.nBad = 0;
            if (s.nBad >= 3) ok = false;
        }
        s.newiter = 1;
        s.qmax = 0;
        bool term = false;
        if (s.it < s.iterations && raised) term = s.seen = 1;
        if (!ok || s.it >= s.iterations || term) s.done = 1;
    }
    if (a) s.cur ^= 1;   // the trial buffers become the current estimate (no copy)
    return s;
}

// The decision as a launch of its own: after the last trial slot of a chunk (the state the host
// reads back). Inside a chunk the next slot's lba_reduce_points decides instead.
__global__ __launch_bounds__(64) void lba_decide(Graph g, int nbt) {
    __shared__ double sums_s[2];
    const LMState s0 = *g.lm_src;
    if (s0.done) {
        if (threadIdx.x == 0) *g.lm = s0;
        return;
    }
    decide_sums(g, nbt, sums_s);
    __syncthreads();
    if (threadIdx.x == 0) *g.lm = lm_next(g, s0, sums_s[0], sums_s[1]);
}

// the EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ records of Optimizer.cc:750-848 from the
// caller's arrays: observation (stereo iff ur >= 0), information inv_sigma2 * I, Huber delta
// sqrt(5.991) / sqrt(7.815) (float, as the reference's thHuberMono / thHuberStereo), the
// keyframe's camera
__global__ __launch_bounds__(256) void lba_build_edges(EdgeDev *E, int ne, const int *ep, const int *eq, const float *obs,
                                                       const float *isg, const float *cam, float thMono, float thStereo) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= ne) return;
    EdgeDev d;
    const float *ob = obs + 3 * k;
    d.point = eq[k];
    d.pose = ep[k];
    d.stereo = ob[2] >= 0;
    d.obs[0] = ob[0]; d.obs[1] = ob[1]; d.obs[2] = d.stereo ? ob[2] : 0;
    d.info = isg[k];
    d.robust = 1;
    d.delta = d.stereo ? thStereo : thMono;
    d.dsqr = d.delta * d.delta;
    const float *c = cam + 5 * d.pose;
    d.fx = c[0]; d.fy = c[1]; d.cx = c[2]; d.cy = c[3]; d.bf = c[4];
    E[k] = d;
}

// outlier test of Optimizer.cc:925-962 / 977-1008: chi2 (stale _error) + depth sign
// the call's results packed for one download: the estimate's poses (nT doubles), points (nX
// doubles) and the erase flags of every edge, each thread one double of T, one of X and one flag
// The estimate buffers of the call's final state: (T, X) or (T2, X2) by st->cur (the last optimize()'s
// state, read on the device: the launch can be enqueued before the host knows it).
__global__ __launch_bounds__(256) void lba_outliers(const EdgeDev *E, const double *err, const Pose *T0,
                                                    const Pose *T1, const double *X0, const double *X1,
                                                    const LMState *st, int ne, int nT, int nX, double *outT,
                                                    double *outX, uint8_t *flag) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const bool c = st->cur;
    const Pose *T = c ? T1 : T0;
    const double *X = c ? X1 : X0;
    if (k < nT) outT[k] = ((const double *)T)[k];
    if (k < nX) outX[k] = X[k];
    if (k >= ne) return;
    const EdgeDev e = E[k];
    const double *er = err + 3 * k;
    const double chi = edge_chi2(e, er);
    double p[3];
    pose_map(T[e.pose], X + 3 * e.point, p);
    const double th = e.stereo ? 7.815 : 5.991;
    flag[k] = (chi > th || !(p[2] > 0.0)) ? 1 : 0;
}

// The per-call buffer initialisation in one launch (was seven memsets and two device copies, each
// a launch of its own on the path to the first LM trial): range r = blockIdx.y fills `bytes` bytes
// at dst with the byte `value`, or copies them from src. dst / src 16-byte aligned (hipMalloc /
// 256-byte arena offsets); the tail past the last 16-byte chunk byte by byte.
struct InitRange { void *dst; const void *src; unsigned long long bytes; int value, pad; };
constexpr int kInitRanges = 10;
struct InitRanges { InitRange r[kInitRanges]; };
__global__ __launch_bounds__(256) void lba_init_buffers(InitRanges R) {
    // fields read with constant indices only (a dynamic index copies the argument to scratch)
    void *dst = nullptr;
    const void *src = nullptr;
    unsigned long long bytes = 0;
    int value = 0;
    switch (blockIdx.y) {
#define LBA_INIT_CASE(i) \
    case i: dst = R.r[i].dst; src = R.r[i].src; bytes = R.r[i].bytes; value = R.r[i].value; break;
        LBA_INIT_CASE(0) LBA_INIT_CASE(1) LBA_INIT_CASE(2) LBA_INIT_CASE(3) LBA_INIT_CASE(4)
        LBA_INIT_CASE(5) LBA_INIT_CASE(6) LBA_INIT_CASE(7) LBA_INIT_CASE(8) LBA_INIT_CASE(9)
#undef LBA_INIT_CASE
        default: return;
    }
    static_assert(kInitRanges == 10, "one case per range");
    const InitRange q = {dst, src, bytes, value, 0};
    const unsigned long long n16 = q.bytes >> 4;
    const unsigned v8 = (unsigned)(q.value & 0xFF) * 0x01010101u;
    const uint4 fill = make_uint4(v8, v8, v8, v8);
    // two loops, not a select: `src ? src[i] : fill` becomes a load through a pointer select, and
    // `fill` a private (scratch) variable
    const unsigned long long i0 = (unsigned long long)blockIdx.x * 256 + threadIdx.x, di = (unsigned long long)gridDim.x * 256;
    if (q.src) {
        for (unsigned long long i = i0; i < n16; i += di) ((uint4 *)q.dst)[i] = ((const uint4 *)q.src)[i];
    } else {
        for (unsigned long long i = i0; i < n16; i += di) ((uint4 *)q.dst)[i] = fill;
    }
    if (blockIdx.x == 0 && threadIdx.x < (q.bytes & 15)) {
        const unsigned long long b = (n16 << 4) + threadIdx.x;
        ((uint8_t *)q.dst)[b] = q.src ? ((const uint8_t *)q.src)[b] : (uint8_t)q.value;
    }
}

// Optimizer.cc:925-962 between the two optimize() calls, on the device: the outlier test of every
// active edge against the current estimate (stale _error, depth sign) moves it to level 1 (on = 0)
// and every edge drops its robust kernel. The second optimize() then runs over the same slots,
// hessian indices and Schur tile lists: a level-1 slot contributes zeros (lba_linearize) and no
// chi2 (lba_errors), and a vertex left without level-0 edges keeps a zero Hessian block and a zero
// update -- the results g2o gives by leaving it out of initializeOptimization(0).
__global__ __launch_bounds__(256) void lba_phase2_mark(Graph g, EdgeDev *E, uint8_t *on, int ne) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (g.lm->gate != 0) return;   // lba_phase2_begin: the second optimize() does not run (now)
    if (s < g.nact) {
        const int k = s;   // every edge is active in slot order (build_active)
        const bool cur = g.lm->cur;
        const EdgeDev e = E[k];
        const double chi = edge_chi2(e, g.err + 3 * k);
        double p[3];
        pose_map((cur ? g.T2 : g.T)[e.pose], (cur ? g.X2 : g.X) + 3 * e.point, p);
        const double th = e.stereo ? 7.815 : 5.991;
        const int lpos = g.slot_lpos[s];
        if (chi > th || !(p[2] > 0.0)) { on[s] = 0; g.on_lm[lpos] = 0; }
        g.E_lm[lpos].robust = 0;
    }
    if (s < ne) E[s].robust = 0;
}

// the landmark-major copy of the edge records (lba_lin_points), once per LocalBA call
__global__ __launch_bounds__(256) void lba_gather_edges(EdgeDev *E_lm, uint8_t *on_lm, const EdgeDev *E, const int *pt_items,
                                                        int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    E_lm[i] = E[pt_items[i]];
    on_lm[i] = 1;
}

// b vector in hessian order for computeScale: [b_p (6P) | b_l (3Lm)]

}  // namespace lbaamd

using namespace lbaamd;

struct DBuf {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n && p) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, std::max<size_t>(bytes, 64)) != hipSuccess) return -1;
        n = std::max<size_t>(bytes, 64);
        return 0;
    }
    template <class T> T *as() { return (T *)p; }
    ~DBuf() { if (p) (void)hipFree(p); }
};

struct lba_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    DBuf T, T2, X, X2, E, E_lm, on_lm, err, act, pose_hidx, point_hidx, hpose, hpoint, pt_start, pt_items,
        ps_start, ps_items, slot_pt, slot_ph, con, hpl, Hll, bl, Hpp, bp, Dinv, Lc, Y, ywp, on, tp_part, Hs, bs, x, partial,
        scalars, flags, lm, arrive, arenaA, arenaB, arenaC, Wm;
    double *h_scalars = nullptr;  // pinned
    LMState *h_lm = nullptr;      // pinned, one per optimize() of a call
    void *h_stage[3] = {nullptr, nullptr, nullptr};   // pinned upload staging per arena (grow-only)
    size_t h_stage_bytes[3] = {0, 0, 0};
    hipEvent_t ev_stage[3] = {nullptr, nullptr, nullptr};   // the last DMA out of each staging buffer
    bool stage_rec[3] = {false, false, false};
    void *h_down = nullptr;       // pinned download staging of the results (grow-only)
    size_t h_down_bytes = 0;
    // pbStopFlag as the device sees it: a page-locked, device-mapped, coherent word the host loop
    // keeps equal to the caller's flag while a chunk of trials runs (lba_optimize)
    unsigned *h_stop = nullptr;
    unsigned *d_stop = nullptr;
    hipEvent_t ev_chunk[2] = {nullptr, nullptr};   // per optimize(): its last chunk's state readback
    int hook_phase = 0, hook_trial = 0;   // lba_set_stop_hook
    int chunks_seen = 0;                  // chunk readbacks of the current call (hook phase 3)
    bool hook_raised = false;             // hook phase 3 fired in this call: ORed into the mirrored flag
    // lba_set_test_option: the two-launch finish + Cholesky path instead of lba_finish_chol, and the
    // hand-off wait's poll bound
    bool fuse_finish = true;
    unsigned spin_limit = kSpinLimit;
    // per-kernel hipEvent timing on the engine stream (lba_profile; bench.py localba roofline)
    bool prof = false;
    struct ProfRec { const char *name; hipEvent_t a, b; };
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
};

static int lprof_begin(lba_engine *e) {
    if (!e->prof) return -1;
    if (e->used + 2 > e->pool.size())
        for (int k = 0; k < 256; k++) {
            hipEvent_t ev;
            if (hipEventCreate(&ev) != hipSuccess) return -1;
            e->pool.push_back(ev);
        }
    const int h = (int)e->used;
    e->used += 2;
    (void)hipEventRecord(e->pool[h], e->stream);
    return h;
}
static void lprof_end(lba_engine *e, int h, const char *name) {
    if (h < 0) return;
    (void)hipEventRecord(e->pool[h + 1], e->stream);
    e->recs.push_back({name, e->pool[h], e->pool[h + 1]});
}

namespace {

using namespace lbaamd_host;

// The host arrays of one upload step packed into the engine's page-locked staging buffer and
// sent to one device arena in ONE DMA (one pageable copy per array before: ~40 staged copies per
// LocalBA call). add() returns the array's byte offset inside the arena.
struct UploadSet {
    struct Item { const void *src; size_t bytes, off; };
    std::vector<Item> items;
    size_t total = 0;
    template <class T> size_t add(const std::vector<T> &v) { return add(v.data(), sizeof(T) * v.size()); }
    // arena space only (filled on the device)
    template <class T> size_t reserve(const std::vector<T> &v) { return add(nullptr, sizeof(T) * v.size()); }
    size_t add(const void *src, size_t bytes) {
        const size_t off = total;
        items.push_back({src, bytes, off});
        total += (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
        return off;
    }
};
// Two staging buffers (one per arena): an upload waits only for the previous DMA out of its own
// buffer (an event), not for the stream -- the second upload of a call no longer stalls on the first.
int upload_set(lba_engine *e, int k, DBuf &arena, const UploadSet &u, hipStream_t s) {
    if (e->stage_rec[k] && hipEventSynchronize(e->ev_stage[k]) != hipSuccess) return -1;
    if (u.total > e->h_stage_bytes[k]) {
        if (e->h_stage[k]) (void)hipHostFree(e->h_stage[k]);
        e->h_stage[k] = nullptr;
        e->h_stage_bytes[k] = 0;
        if (hipHostMalloc(&e->h_stage[k], u.total, hipHostMallocDefault) != hipSuccess) return -1;
        e->h_stage_bytes[k] = u.total;
    }
    for (const auto &it : u.items)
        if (it.bytes && it.src) std::memcpy((char *)e->h_stage[k] + it.off, it.src, it.bytes);
    if (u.total > arena.n && hipStreamSynchronize(s) != hipSuccess) return -1;   // the old arena may be in use
    if (arena.ensure(u.total)) return -1;
    if (hipMemcpyAsync(arena.p, e->h_stage[k], u.total, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipEventRecord(e->ev_stage[k], s) != hipSuccess)
        return -1;
    e->stage_rec[k] = true;
    return 0;
}
template <class T> T *at(DBuf &arena, size_t off) { return (T *)((char *)arena.p + off); }

int nblk(int n) { return std::max(1, (n + 255) / 256); }

}  // namespace

// One SparseOptimizer::optimize(iterations) on the device (LmPhase): trial slots (linearisation +
// setLambda/Schur/solve/update/errors, each decided inside the next slot's lba_reduce_points) are
// enqueued in chunks without host synchronisation; the device LM state turns the slots after the
// last trial into no-ops. Each chunk ends with a one-block lba_decide, an async readback of the
// state and an event; the host polls the event. pbStopFlag is read by the device itself, at every
// point where g2o reads it (the optimize() start, lm_next): while a chunk runs, the host loop copies
// *stop into the mapped word the kernels load with system scope, so a flag raised mid-call ends the
// optimisation after the trial in flight, as SparseOptimizer::terminate() does.
// stop_at: the test hook's trial count for this optimize() (INT_MAX: none).
struct LmPhase {
    lba_engine *e;
    Graph &g;
    const ActiveSet &A;
    int iterations;
    const volatile uint8_t *stop;
    int stop_at;
    LMState *h_state;     // pinned readback of this phase's state
    hipEvent_t ev;        // end of the last chunk's readback
    hipStream_t s;
    int nact = 0, n6 = 0, nbl = 0, nbt = 0, slots = 0, rc = 0;
    LmPhase(lba_engine *e_, Graph &g_, const ActiveSet &A_, int iterations_, const volatile uint8_t *stop_, int stop_at_,
            LMState *h_state_, hipEvent_t ev_)
        : e(e_), g(g_), A(A_), iterations(iterations_), stop(stop_), stop_at(stop_at_), h_state(h_state_), ev(ev_),
          s(e_->stream) {
        if (A.P + A.Lm == 0) { rc = -1; return; }
        if (A.P > kMaxPoses) { rc = -2; return; }
        if ((A.Lm + kRPL - 1) / kRPL > kRedBlocks) { rc = -2; return; }   // partial regions
        nact = (int)A.act.size();
        n6 = 6 * A.P;
        // lba_lin_points workgroups: landmarks (kLPB each), then free poses (256 each); its chi2 and
        // computeScale block sums are the partials every reduction of the LM state reads (nbt of each)
        nbl = std::max(1, (A.Lm + kLPB - 1) / kLPB);
        nbt = nbl + nblk(A.P);
        if (nbt > kRedBlocks) rc = -2;
    }
    void mirror() {
        if (stop) __atomic_store_n(e->h_stop, (unsigned)(*stop != 0 || e->hook_raised), __ATOMIC_RELAXED);
    }
    // the LM state ping-pongs between g.lm_buf[0 / 1] at every decision: a deciding launch reads one
    // buffer and writes the other, and every later launch reads the new one
    void advance(Graph &gd) {
        gd = g;
        gd.lm_src = g.lm;
        gd.lm = g.lm == g.lm_buf[0] ? g.lm_buf[1] : g.lm_buf[0];
        g.lm = gd.lm;
    }
    void slot(bool first, bool decide) {
        slot_head(first, decide);
        slot_tail();
    }
    // a trial slot up to the Schur step: the linearisation (an iteration's first slot) and the
    // landmark reductions; `decide`: the previous trial of this chunk is undecided, this slot's
    // lba_reduce_points decides it
    void slot_head(bool first, bool decide) {
        int ph;
        if (first) {   // later iterations start from the linearisation of the accepted trial
            ph = lprof_begin(e);
            lba_lin_points<false><<<nbt, 256, 0, s>>>(g, nullptr, g.scalars + 8 + nbt, nbl);
            lprof_end(e, ph, "lba_linearize");
        }
        ph = lprof_begin(e);
        const int nrp = std::max(1, (A.Lm + kRPL - 1) / kRPL);
        // lambda init (levenberg.cpp:179-191) in an optimize()'s first slot: the maxDiagonal needs
        // Hpp before the Schur step (the pose workgroups of lba_reduce_points)
        const int npw = first && A.P > 0 ? (27 * A.P + 3) / 4 : 0;
        if (decide) {
            Graph gd;
            advance(gd);
            lba_reduce_points<<<nrp + npw, 256, 0, s>>>(gd, nbt, nbt, npw);
        } else {
            lba_reduce_points<<<nrp + npw, 256, 0, s>>>(g, nbt, nbt, npw);
        }
        lprof_end(e, ph, "lba_reduce_points");
        if (first) {
            ph = lprof_begin(e);
            lba_prep_slots<<<nblk(nact + A.Lm), 256, 0, s>>>(g, nbt, nrp, 6 * A.P);
            lprof_end(e, ph, "lba_prep_slots");
        }
    }
    // the rest of a trial slot: Schur complement, solve, update + the trial's residuals
    void slot_tail() {
        int ph;
        if (A.P > 0) {
            ph = lprof_begin(e);
            // chunk workgroups, then b_p / b_schur rows (one wave each), then Hpp (one wave per
            // (pose, upper component))
            lba_schur_tiles<<<g.nchunks + (n6 + 3) / 4 + (21 * A.P + 3) / 4, 256, 0, s>>>(g);
            lprof_end(e, ph, "lba_schur_tiles");
            const bool big = n6 > kSmallNP && n6 <= kBigNP;
            if (e->fuse_finish && (n6 <= kSmallNP || big)) {
                ph = lprof_begin(e);
                const int nfb = (g.npairs + 3) / 4;
                if (big)
                    lba_finish_chol<true><<<nfb + 1, kCT, chol_global_lds(n6), s>>>(g, nfb);
                else
                    lba_finish_chol<false><<<nfb + 1, kCT, chol_tiled_lds(n6), s>>>(g, nfb);
                lprof_end(e, ph, "lba_finish_chol");
            } else {
            ph = lprof_begin(e);
            lba_schur_finish<<<g.npairs, 256, 0, s>>>(g);
            lprof_end(e, ph, "lba_schur_finish");
            if (n6 <= kSmallNP) {
                ph = lprof_begin(e);
                lba_chol_tiled<<<1, kCT, chol_tiled_lds(n6), s>>>(g);
                lprof_end(e, ph, "lba_chol_tiled");
            } else if (big) {
                ph = lprof_begin(e);
                lba_chol_global<<<1, kCT, chol_global_lds(n6), s>>>(g);
                lprof_end(e, ph, "lba_chol_global");
            } else {   // every launch its own profile record: lba_profile_read's counts are launches
                ph = lprof_begin(e);
                lba_set_ok<<<1, 1, 0, s>>>(g);
                lprof_end(e, ph, "lba_set_ok");
                for (int kb = 0; kb < n6; kb += kCB) {
                    const int rows = n6 - kb - kCB;
                    ph = lprof_begin(e);
                    lba_chol_panel<<<std::max(1, (rows + 255) / 256), 256, 0, s>>>(g, kb);
                    lprof_end(e, ph, "lba_chol_panel");
                    if (rows > 0) {
                        const int nt = (rows + 15) / 16;
                        ph = lprof_begin(e);
                        lba_chol_update<<<nt * (nt + 1) / 2, 64, 0, s>>>(g, kb, nt);
                        lprof_end(e, ph, "lba_chol_update");
                    }
                }
                ph = lprof_begin(e);
                lba_chol_solve_blocked<<<1, 1024, sizeof(double) * n6, s>>>(g);
                lprof_end(e, ph, "lba_chol_solve_blocked");
            }
            }
        } else {
            lba_set_ok<<<1, 1, 0, s>>>(g);
        }
        // scalars[8..): the trial's computeScale block sums, then its chi2 block sums (nbt each)
        ph = lprof_begin(e);
        lba_lin_points<true><<<nbt, kLinThreads, 0, s>>>(g, g.scalars + 8, g.scalars + 8 + nbt, nbl);
        lprof_end(e, ph, "lba_update_errors");
    }
    // optimize() start (levenberg.cpp:66-72 reset, the first terminate() check)
    void init() {
        mirror();
        lba_lm_init<<<1, 1, 0, s>>>(g, iterations, stop_at);
    }
    // k trial slots of the open chunk (`chunk0`: the first slot of the chunk's enqueue)
    int chunk0 = 0;
    void enqueue_slots(int k) {
        for (int i = 0; i < k; i++) slot(slots + i == 0, slots + i > chunk0);
        slots += k;
    }
    // k trial slots, the chunk's last decision, the state readback and the chunk's event
    int enqueue_chunk(int k) {
        chunk0 = slots;
        enqueue_slots(k);
        return close_chunk();
    }
    // the first chunk of an optimize() in two parts: the first slot's head (first_head), then its
    // tail and the chunk's k - 1 other slots
    void first_head() {
        slots = chunk0 = 0;
        slot_head(true, false);
    }
    int complete_first_chunk(int k) {
        slot_tail();
        slots = 1;
        enqueue_slots(k - 1);
        return close_chunk();
    }
    int close_chunk() {
        {
            const int ph = lprof_begin(e);
            Graph gd;
            advance(gd);
            lba_decide<<<1, 64, 0, s>>>(gd, nbt);
            lprof_end(e, ph, "lba_decide");
        }
        if (hipMemcpyAsync(h_state, g.lm, sizeof(LMState), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(ev, s) != hipSuccess)
            return -3;
        return 0;
    }
    // wait for the last chunk's readback, keeping the device's copy of the flag current. The poll
    // gives its core away: a short pause-spin (a chunk often ends within it), then sched_yield()
    // between queries -- free when the core is idle, and the Tracking threads' extractor calls
    // (Frame.cc:144-153) run first when they want the core -- and, past 2 ms (only an unusually
    // long chunk), 20 us sleeps. The flag is still mirrored at every query.
    int wait(LMState &st) {
        if (!stop) {
            if (hipEventSynchronize(ev) != hipSuccess) return -3;
        } else {
            const auto t0 = std::chrono::steady_clock::now();
            for (int it = 0;; it++) {
                mirror();
                const hipError_t q = hipEventQuery(ev);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) return -3;
                if (it < 16) {
                    for (int k = 0; k < 64; k++) __builtin_ia32_pause();
                } else if (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2)) {
                    sched_yield();
                } else {
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                }
            }
        }
        st = *h_state;
        if (st.fault) {   // a hand-off wait timed out (lba_finish_chol): the results are not the oracle's
            (void)hipStreamSynchronize(s);
            fprintf(stderr, "orbslam2_amd lba: Schur hand-off wait timed out\n");
            return -4;
        }
        // test hook (lba_set_stop_hook phase 3): once the call's hook_trial-th chunk is read back, the
        // mirrored flag reads as raised from then on (an engine-owned flag ORed into it: the caller's
        // const flag is never written) -- a mid-call raise at a deterministic point
        if (stop && e->hook_phase == 3 && ++e->chunks_seen == e->hook_trial) {
            e->hook_raised = true;
            mirror();
        }
        return 0;
    }
    // two slots per chunk while retries remain (the first chunk holds one trial per iteration: the
    // common case, every first trial accepted)
    int finish(LMState &st) {
        while (!st.done) {
            if (slots > 10 * iterations + 1) return -3;   // cannot happen: <= 10 trials per iteration
            if (enqueue_chunk(2) || wait(st)) return -3;
        }
        return 0;
    }
};

extern "C" {

int lba_create(lba_engine **out) {
    if (!out) return ORBX_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORBX_EDEVICE;
    lba_engine *e = new lba_engine();
    // the engine stream at the device's highest priority: LocalMapping's LocalBA beside Tracking's
    // extraction (Frame.cc:144-153 on other threads) -- beside a saturating C2 stream 34 -> 8.7 ms per
    // call (profiles/r06_lba_concurrent.log); alone no difference
    int prio_least = 0, prio_greatest = 0;
    if (hipGetDevice(&e->device) != hipSuccess || hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, prio_greatest) != hipSuccess ||
        hipHostMalloc((void **)&e->h_scalars, (8 + 2 * kRedBlocks) * sizeof(double)) != hipSuccess ||
        hipHostMalloc((void **)&e->h_lm, 2 * sizeof(LMState)) != hipSuccess ||
        hipHostMalloc((void **)&e->h_stop, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&e->d_stop, e->h_stop, 0) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_chunk[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_chunk[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_stage[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_stage[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_stage[2], hipEventDisableTiming) != hipSuccess) {
        delete e;
        return ORBX_EDEVICE;
    }
    *out = e;
    return ORBX_OK;
}

void lba_destroy(lba_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) { (void)hipStreamSynchronize(e->stream); (void)hipStreamDestroy(e->stream); }
    if (e->h_scalars) (void)hipHostFree(e->h_scalars);
    if (e->h_lm) (void)hipHostFree(e->h_lm);
    if (e->h_stop) (void)hipHostFree(e->h_stop);
    for (hipEvent_t ev : e->ev_chunk) if (ev) (void)hipEventDestroy(ev);
    for (int k = 0; k < 3; k++) {
        if (e->h_stage[k]) (void)hipHostFree(e->h_stage[k]);
        if (e->ev_stage[k]) (void)hipEventDestroy(e->ev_stage[k]);
    }
    if (e->h_down) (void)hipHostFree(e->h_down);
    for (hipEvent_t ev : e->pool) (void)hipEventDestroy(ev);
    delete e;
}

// host-phase wall clock of lba_solve (ORBX_LBA_HOSTPROF=1: one line per call on stderr)
struct HostProf {
    bool on;
    std::chrono::steady_clock::time_point t0, t;
    std::string line;
    HostProf() : on(std::getenv("ORBX_LBA_HOSTPROF") != nullptr), t0(std::chrono::steady_clock::now()), t(t0) {}
    void mark(const char *what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        line += std::string(" ") + what + "=" + std::to_string(std::chrono::duration<double, std::micro>(n - t).count());
        t = n;
    }
    ~HostProf() {
        if (on)
            fprintf(stderr, "LBAHOST total=%.1f%s\n", std::chrono::duration<double, std::micro>(t - t0).count(), line.c_str());
    }
};

int lba_solve(lba_engine *e, const lba_problem *p, lba_result *r, const volatile uint8_t *stop) {
    if (!e || !p || !r || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0) return ORBX_EINVAL;
    HostProf hp;
    LBA_CHK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    const int np = p->n_poses, nq = p->n_points, ne = p->n_edges;
    r->iterations[0] = r->iterations[1] = 0;
    r->trials[0] = r->trials[1] = 0;
    r->chi2[0] = r->chi2[1] = 0;
    r->stopped = 0;
    if (stop && *stop) {  // Optimizer.cc:902-904: return before optimising, nothing written back
        r->stopped = 2;
        std::memcpy(r->pose_Tcw, p->pose_Tcw, sizeof(float) * 16 * np);
        std::memcpy(r->point_Xw, p->point_Xw, sizeof(float) * 3 * nq);
        std::memset(r->edge_erase, 0, ne);
        return ORBX_OK;
    }
    // vertices (Converter::toSE3Quat / toVector3d)
    std::vector<Pose> T(np);
    for (int i = 0; i < np; i++) {
        const float *m = p->pose_Tcw + 16 * i;
        const double R[9] = {m[0], m[1], m[2], m[4], m[5], m[6], m[8], m[9], m[10]};
        quat_from_R_norm(R, T[i].q);
        T[i].t[0] = m[3]; T[i].t[1] = m[7]; T[i].t[2] = m[11];
        T[i].pad = 0;
    }
    std::vector<double> X(3 * (size_t)nq);
    for (int i = 0; i < 3 * nq; i++) X[i] = p->point_Xw[i];
    HostGraph h;
    h.np = np; h.nq = nq; h.ne = ne;
    h.pose_id = p->pose_id; h.point_id = p->point_id; h.fixed = p->pose_fixed;
    h.edge_point = p->edge_point;
    h.edge_pose = p->edge_pose;
    for (int k = 0; k < ne; k++)
        if (h.edge_point[k] < 0 || h.edge_point[k] >= nq || h.edge_pose[k] < 0 || h.edge_pose[k] >= np) return ORBX_EINVAL;
    hp.mark("build");
    // the caller's edge arrays go up as they are (24 B per edge); lba_build_edges forms the device
    // edge records (112 B) there
    UploadSet ua;
    // the trial buffers T2 / X2 are set equal to T / X by setup's lba_init_buffers
    const size_t oT = ua.add(T), oT2 = ua.reserve(T), oX = ua.add(X), oX2 = ua.reserve(X);
    const size_t oep = ua.add(p->edge_pose, sizeof(int32_t) * ne), oeq = ua.add(p->edge_point, sizeof(int32_t) * ne),
                 oobs = ua.add(p->edge_obs, sizeof(float) * 3 * ne), oisg = ua.add(p->edge_inv_sigma2, sizeof(float) * ne),
                 ocam = ua.add(p->pose_cam, sizeof(float) * 5 * np);
    if (upload_set(e, 0, e->arenaA, ua, s) || e->E.ensure(sizeof(EdgeDev) * std::max(ne, 1)) ||
        e->err.ensure(sizeof(double) * 3 * std::max(ne, 1)) ||
        e->flags.ensure(sizeof(Pose) * np + sizeof(double) * 3 * nq + ne + 16) || e->scalars.ensure((8 + 2 * kRedBlocks) * sizeof(double)) ||
        e->partial.ensure(sizeof(double) * 4 * kRedBlocks) || e->lm.ensure(4 * sizeof(LMState)) || e->arrive.ensure(64))
        return ORBX_EDEVICE;
    // err, arrive and the LM state (cur = 0: (T, X) hold the estimate) are zeroed by setup's
    // lba_init_buffers, before any kernel reads them
    int cur = 0;
    *e->h_stop = 0u;
    e->chunks_seen = 0;
    e->hook_raised = false;
    Graph g{};
    g.stopf = e->d_stop;
    g.spin_limit = e->spin_limit;
    g.T = at<Pose>(e->arenaA, oT); g.T2 = at<Pose>(e->arenaA, oT2);
    g.X = at<double>(e->arenaA, oX); g.X2 = at<double>(e->arenaA, oX2);
    if (ne > 0)
        lba_build_edges<<<nblk(ne), 256, 0, s>>>(e->E.as<EdgeDev>(), ne, at<int>(e->arenaA, oep), at<int>(e->arenaA, oeq),
                                                 at<float>(e->arenaA, oobs), at<float>(e->arenaA, oisg),
                                                 at<float>(e->arenaA, ocam), (float)std::sqrt(5.991), (float)std::sqrt(7.815));   // thHuberMono / Stereo
    LBA_CHK(hipGetLastError());
    g.E = e->E.as<EdgeDev>();
    g.arrive = e->arrive.as<unsigned>();
    g.err = e->err.as<double>();
    g.scalars = e->scalars.as<double>();
    g.partial = e->partial.as<double>();
    g.lm_buf[0] = e->lm.as<LMState>();
    g.lm_buf[1] = g.lm_buf[0] + 1;
    g.lm = g.lm_buf[0];
    g.lm_src = nullptr;
    // the active-set index arrays in one upload, the call's buffers, their initialisation and the
    // landmark-major edge records (the Schur tile lists follow in setup_tiles)
    auto setup = [&](ActiveSet &A) -> int {
        const int Kpad = std::max(4, ((3 * A.Lm + 3) / 4) * 4);
        UploadSet ub;
        const size_t o_pose_hidx = ub.add(A.pose_hidx), o_point_hidx = ub.add(A.point_hidx),
                     o_hpose = ub.add(A.hpose), o_hpoint = ub.add(A.hpoint), o_pt_start = ub.add(A.pt_start),
                     o_pt_items = ub.add(A.pt_items), o_ps_start = ub.add(A.ps_start), o_ps_items = ub.add(A.ps_items),
                     o_slot_pt = ub.add(A.slot_pt), o_slot_ph = ub.add(A.slot_ph);
        // landmark-major slot order (the common case): the lpos arrays are the slot arrays
        const size_t o_slot_ppos = ub.add(A.slot_ppos), o_slot_lpos = ub.add(A.slot_lpos),
                     o_lpos_ph = A.mono ? o_slot_ph : ub.add(A.lpos_ph), o_lpos_ppos = A.mono ? o_slot_ppos : ub.add(A.lpos_ppos);
        if (upload_set(e, 1, e->arenaB, ub, s)) return -1;
        hp.mark("stage");
        const int nact = (int)A.act.size();
        g.nact = nact;
        if (e->on.ensure(std::max(nact, 1))) return -1;
        g.on = e->on.as<uint8_t>();
        // landmark-major slot order (A.mono): the landmark-major records and level flags are the
        // slot ones themselves, no gathered copy
        if (A.mono) {
            g.E_lm = const_cast<EdgeDev *>(g.E);
            g.on_lm = e->on.as<uint8_t>();
        } else {
            if (e->E_lm.ensure(sizeof(EdgeDev) * std::max(nact, 1)) || e->on_lm.ensure(std::max(nact, 1))) return -1;
            g.E_lm = e->E_lm.as<EdgeDev>();
            g.on_lm = e->on_lm.as<uint8_t>();
        }
        g.pose_hidx = at<int>(e->arenaB, o_pose_hidx); g.point_hidx = at<int>(e->arenaB, o_point_hidx);
        g.hpose = at<int>(e->arenaB, o_hpose); g.hpoint = at<int>(e->arenaB, o_hpoint);
        g.P = A.P; g.Lm = A.Lm;
        g.pt_start = at<int>(e->arenaB, o_pt_start); g.pt_items = at<int>(e->arenaB, o_pt_items);
        g.ps_start = at<int>(e->arenaB, o_ps_start); g.ps_items = at<int>(e->arenaB, o_ps_items);
        g.slot_pt = at<int>(e->arenaB, o_slot_pt); g.slot_ph = at<int>(e->arenaB, o_slot_ph);
        g.slot_ppos = at<int>(e->arenaB, o_slot_ppos);
        g.slot_lpos = at<int>(e->arenaB, o_slot_lpos);
        g.lpos_ph = at<int>(e->arenaB, o_lpos_ph);
        g.lpos_ppos = at<int>(e->arenaB, o_lpos_ppos);
        g.Kpad = Kpad;
        g.NP = std::max(kCB, ((6 * A.P + kCB - 1) / kCB) * kCB);
        const size_t NP = (size_t)g.NP, NPW = NP + 16;
        g.NPW = (int)NPW;
        g.wrow = 16 * std::max(1, (6 * A.P + 15) / 16);
        const size_t nl = std::max(nact, 1), npp = std::max<size_t>(1, A.ps_items.size());
        if (e->con.ensure(sizeof(double) * 2 * (9 * nl + 27 * npp)) || e->hpl.ensure(sizeof(double) * 2 * 18 * nl) ||
            e->Hll.ensure(sizeof(double) * 9 * std::max(A.Lm, 1)) || e->bl.ensure(sizeof(double) * 3 * std::max(A.Lm, 1)) ||
            e->Hpp.ensure(sizeof(double) * 36 * std::max(A.P, 1)) || e->bp.ensure(sizeof(double) * 6 * std::max(A.P, 1)) ||
            e->Dinv.ensure(sizeof(double) * 9 * std::max(A.Lm, 1)) || e->Lc.ensure(sizeof(double) * 6 * std::max(A.Lm, 1)) ||
            e->Y.ensure(sizeof(double) * NPW * (size_t)(g.Kpad + 4)) || e->Hs.ensure(sizeof(double) * NP * NP) ||
            e->ywp.ensure(sizeof(double) * 6 * std::max<size_t>(1, A.ps_items.size())) ||
            e->bs.ensure(sizeof(double) * NP) || e->x.ensure(sizeof(double) * (6 * A.P + 3 * A.Lm + 8)))
            return -1;
        g.conl[0] = e->con.as<double>(); g.conl[1] = g.conl[0] + 9 * nl;
        g.conp[0] = g.conl[1] + 9 * nl; g.conp[1] = g.conp[0] + 27 * npp;
        g.hpl[0] = e->hpl.as<double>(); g.hpl[1] = g.hpl[0] + 18 * nl;
        g.Hll = e->Hll.as<double>(); g.bl = e->bl.as<double>();
        g.Hpp = e->Hpp.as<double>(); g.bp = e->bp.as<double>();
        g.Dinv = e->Dinv.as<double>(); g.Lc = e->Lc.as<double>(); g.Y = e->Y.as<double>();
        g.w = g.Y + g.wrow;
        g.Hs = e->Hs.as<double>(); g.bs = e->bs.as<double>(); g.ywp = e->ywp.as<double>();
        g.x = e->x.as<double>();
        g.W = nullptr;
        g.LDW = 0;
        if (6 * A.P > kSmallNP && 6 * A.P <= kBigNP) {   // chol_global_body's work matrix (fully rewritten per trial)
            const int N2 = chol_tiled_dim(6 * A.P);
            if (e->Wm.ensure(sizeof(double) * chol_global_w(6 * A.P))) return -1;
            g.W = e->Wm.as<double>();
            g.LDW = N2;
        }
        {   // zeroed / filled / copied in one launch: err, arrive, the LM state, the level flags (1),
            // Y, Hs, x, and the trial buffers set equal to the current estimate (inactive vertices
            // never change)
            InitRanges R{};
            const InitRange rr[kInitRanges] = {
                {e->err.p, nullptr, sizeof(double) * 3 * (unsigned long long)std::max(ne, 1), 0, 0},
                {e->arrive.p, nullptr, 64, 0, 0},
                {e->lm.p, nullptr, 4 * sizeof(LMState), 0, 0},
                {e->on.p, nullptr, (unsigned long long)std::max(nact, 1), 1, 0},
                {g.Y, nullptr, sizeof(double) * NPW * (unsigned long long)(g.Kpad + 4), 0, 0},
                {g.Hs, nullptr, sizeof(double) * NP * NP, 0, 0},
                {g.x, nullptr, sizeof(double) * (unsigned long long)(6 * A.P + 3 * A.Lm + 8), 0, 0},
                {cur ? g.T : g.T2, cur ? g.T2 : g.T, sizeof(Pose) * (unsigned long long)std::max(np, 1), 0, 0},
                {cur ? g.X : g.X2, cur ? g.X2 : g.X, sizeof(double) * 3 * (unsigned long long)std::max(nq, 1), 0, 0},
                {nullptr, nullptr, 0, 0, 0}};
            unsigned long long most = 0;
            for (int i = 0; i < kInitRanges; i++) { R.r[i] = rr[i]; most = std::max(most, rr[i].bytes); }
            const unsigned gx = (unsigned)std::max<unsigned long long>(1, std::min<unsigned long long>(1024, (most / 16 + 255) / 256));
            lba_init_buffers<<<dim3(gx, kInitRanges), 256, 0, s>>>(R);
            if (hipGetLastError() != hipSuccess) return -1;
        }
        if (nact > 0 && !A.mono) lba_gather_edges<<<nblk(nact), 256, 0, s>>>(g.E_lm, g.on_lm, g.E, g.pt_items, nact);
        return 0;
    };
    // the block structure of the Schur product (build_schur_tiles) in an upload of its own: built on
    // the host while the first trial slot's linearisation and landmark reductions run on the device
    // (nothing before lba_schur_tiles reads it)
    auto setup_tiles = [&](ActiveSet &A) -> int {
        build_schur_tiles(A, g.Kpad, kSCH);
        UploadSet uc;
        const size_t o_tp_ij = uc.add(A.tp_ij), o_tp_start = uc.add(A.tp_start), o_tp_rows = uc.add(A.tp_rows),
                     o_tp_chunk = uc.add(A.tp_chunk), o_tp_nch = uc.add(A.tp_nch);
        if (upload_set(e, 2, e->arenaC, uc, s)) return -1;
        g.tp_ij = at<int2>(e->arenaC, o_tp_ij);
        g.tp_start = at<int>(e->arenaC, o_tp_start);
        g.tp_rows = at<int>(e->arenaC, o_tp_rows);
        g.npairs = (int)A.tp_ij.size();
        g.tp_chunk = at<int4>(e->arenaC, o_tp_chunk);
        g.tp_nch = at<int2>(e->arenaC, o_tp_nch);
        g.nchunks = (int)A.tp_chunk.size();
        if (e->tp_part.ensure(sizeof(double) * 256 * std::max(g.nchunks, 1))) return -1;
        g.tp_part = e->tp_part.as<double>();
        return 0;
    };
    hp.mark("upload");
    static thread_local ActiveSet A;
    build_active(h, A);
    hp.mark("active1");
    if (setup(A)) return ORBX_EDEVICE;
    hp.mark("setup1");
    // the two optimize() calls (Optimizer.cc:900-917 and 964-966). -1 iterations = the pre-LM error
    // evaluation failed (g2o's optimize() returning -1, a valid outcome). Phase 1's LM state
    // ping-pongs in lm[0..1], phase 2's in lm[2..3]: phase 2's start and first chunk are enqueued
    // right behind phase 1's first chunk, gated on the device by
    // lba_phase2_begin, so the common call (phase 1 done in its first chunk) has no host round trip
    // between the optimizations; when phase 1 needs retry slots, that enqueued chunk is a no-op and
    // phase 2 is enqueued again after them.
    // the three results packed by lba_outliers into one device buffer, one DMA into one page-locked
    // staging buffer (three copies before: D2H copies into the caller's pageable arrays were staged
    // and serialised by the runtime). Enqueued right behind the last optimize()'s chunk, before its
    // state is read back: the kernel takes the estimate buffer from that state on the device. When
    // the chunk turns out not to be the last one, it is enqueued again after the retries.
    const size_t oTd = 0, oXd = sizeof(Pose) * np, oFd = oXd + sizeof(double) * 3 * nq, down = oFd + ne + 16;
    if (down > e->h_down_bytes) {
        if (e->h_down) (void)hipHostFree(e->h_down);
        e->h_down = nullptr;
        e->h_down_bytes = 0;
        LBA_CHK(hipHostMalloc(&e->h_down, down, hipHostMallocDefault));
        e->h_down_bytes = down;
    }
    auto enqueue_final = [&](const LMState *stp) -> int {
        char *dd = (char *)e->flags.p;   // `down` bytes, allocated with the call's other buffers
        const int nT = (int)(sizeof(Pose) / sizeof(double)) * np, nX = 3 * nq;
        lba_outliers<<<nblk(std::max(ne, std::max(nT, nX))), 256, 0, s>>>(
            g.E, g.err, g.T, g.T2, g.X, g.X2, stp, ne, nT, nX, (double *)(dd + oTd), (double *)(dd + oXd),
            (uint8_t *)(dd + oFd));
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(e->h_down, e->flags.p, oFd + ne, hipMemcpyDeviceToHost, s) != hipSuccess)
            return -3;
        return 0;
    };
    const int hook1 = e->hook_phase == 1 ? e->hook_trial : INT_MAX, hook2 = e->hook_phase == 2 ? e->hook_trial : INT_MAX;
    LmPhase p1(e, g, A, 5, stop, hook1, e->h_lm, e->ev_chunk[0]);
    if (p1.rc == -2) return ORBX_EINVAL;
    if (p1.rc == -1) {   // no vertex to optimise: both optimize() calls return -1
        r->iterations[0] = -1;
        if (!(stop && *stop)) r->iterations[1] = -1;
        else r->stopped = 1;
        if (enqueue_final(g.lm)) return ORBX_EDEVICE;   // lm zeroed: cur = 0
    } else {
        // phase 1's first slot up to the Schur step, then the tile lists (host work that overlaps
        // it), then the rest of the slot and of the chunk
        p1.init();
        p1.first_head();
        if (setup_tiles(A)) return ORBX_EDEVICE;
        hp.mark("tiles");
        Graph g2 = g;
        g2.lm_buf[0] = g.lm_buf[0] + 2;
        g2.lm_buf[1] = g.lm_buf[0] + 3;
        g2.lm = g2.lm_buf[0];
        g2.lm_src = nullptr;
        LmPhase p2(e, g2, A, 10, stop, hook2, e->h_lm + 1, e->ev_chunk[1]);
        // phase 2's start and its first `k` trial slots (the rest of its first chunk follows)
        auto phase2_start = [&](bool spec, int k) -> int {
            lba_phase2_begin<<<1, 1, 0, s>>>(g2, g.lm, 10, hook2, spec ? 1 : 0);
            // phase 1 ran with every edge at level 0 (its slots are all edges): the level-1 moves and
            // the robust-kernel drop stay on the device
            lba_phase2_mark<<<nblk(std::max(ne, (int)A.act.size())), 256, 0, s>>>(g2, const_cast<EdgeDev *>(g.E),
                                                                                   e->on.as<uint8_t>(), ne);
            if (hipGetLastError() != hipSuccess) return -3;
            p2.slots = p2.chunk0 = 0;
            p2.enqueue_slots(k);
            return 0;
        };
        LMState st1{}, st2{};
        if (p1.complete_first_chunk(5)) return ORBX_EDEVICE;
        // one phase-2 slot behind phase 1's first chunk: it keeps the GPU busy while the host reads
        // phase 1's state back; a deferred one costs its few empty launches
        const bool spec = true;
        if (spec && phase2_start(true, 1)) return ORBX_EDEVICE;
        if (p1.wait(st1)) return ORBX_EDEVICE;
        const bool first_chunk = st1.done;   // the speculative phase-2 start finds phase 1 done
        if (p1.finish(st1)) return ORBX_EDEVICE;
        hp.mark("opt1");
        r->iterations[0] = st1.it;
        r->chi2[0] = st1.final_chi;
        r->trials[0] = st1.trials;
        cur = st1.cur;
        if (!spec || !first_chunk) {
            if (phase2_start(false, 10) || p2.close_chunk()) return ORBX_EDEVICE;
        } else {
            p2.enqueue_slots(9);
            if (p2.close_chunk()) return ORBX_EDEVICE;
        }
        if (enqueue_final(g2.lm)) return ORBX_EDEVICE;
        const int slots2 = p2.slots;
        if (p2.wait(st2) || p2.finish(st2)) return ORBX_EDEVICE;
        if (p2.slots != slots2 && enqueue_final(g2.lm)) return ORBX_EDEVICE;   // retries ran after it
        if (st2.gate == 2) {   // if(pbStopFlag) if(*pbStopFlag) bDoMore = false: no second optimize()
            r->stopped = 1;
        } else {
            r->iterations[1] = st2.it;
            r->chi2[1] = st2.final_chi;
            r->trials[1] = st2.trials;
            cur = st2.cur;
            if (st2.seen) r->stopped = 1;   // phase 2 cut short by the flag
        }
        hp.mark("opt2");
    }
    LBA_CHK(hipStreamSynchronize(s));   // the enqueued final copy (enqueue_final) has landed
    char *hd = (char *)e->h_down;
    std::memcpy(T.data(), hd + oTd, sizeof(Pose) * np);
    std::memcpy(X.data(), hd + oXd, sizeof(double) * 3 * nq);
    std::memcpy(r->edge_erase, hd + oFd, ne);
    hp.mark("final_wait");
    for (int i = 0; i < np; i++) {  // Converter::toCvMat(SE3Quat)
        double R[9];
        quat_to_R(T[i].q, R);
        float *o = r->pose_Tcw + 16 * i;
        for (int a = 0; a < 3; a++) {
            for (int c = 0; c < 3; c++) o[4 * a + c] = (float)R[3 * a + c];
            o[4 * a + 3] = (float)T[i].t[a];
        }
        o[12] = 0; o[13] = 0; o[14] = 0; o[15] = 1;
    }
    for (int i = 0; i < 3 * nq; i++) r->point_Xw[i] = (float)X[i];
    hp.mark("convert");
    return ORBX_OK;
}

int lba_set_test_option(lba_engine *e, int option, long long value) {
    if (!e) return ORBX_EINVAL;
    switch (option) {
        case LBA_OPT_FUSE_FINISH: e->fuse_finish = value != 0; return ORBX_OK;
        case LBA_OPT_STREAM_PRIORITY: {   // the engine stream recreated at the device's lowest (0) / highest (1) priority
            int least = 0, greatest = 0;
            if (hipSetDevice(e->device) != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess ||
                hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
                return ORBX_EDEVICE;
            hipStream_t ns = nullptr;
            if (hipStreamCreateWithPriority(&ns, hipStreamNonBlocking, value ? greatest : least) != hipSuccess) return ORBX_EDEVICE;
            (void)hipStreamDestroy(e->stream);
            e->stream = ns;
            return ORBX_OK;
        }
        case LBA_OPT_SPIN_LIMIT:   // < 0: the default; 0: every hand-off wait times out (fault injection)
            if (value > 0xFFFFFFFFLL) return ORBX_EINVAL;
            e->spin_limit = value < 0 ? kSpinLimit : (unsigned)value;
            return ORBX_OK;
        default: return ORBX_EINVAL;
    }
}

int lba_set_stop_hook(lba_engine *e, int phase, int trial) {
    if (!e || phase < 0 || phase > 3 || trial < 0 || (phase == 3 && trial < 1)) return ORBX_EINVAL;
    e->hook_phase = phase;
    e->hook_trial = trial;
    return ORBX_OK;
}

int lba_profile(lba_engine *e, int enable) {
    if (!e) return ORBX_EINVAL;
    for (auto &r : e->recs) (void)hipEventSynchronize(r.b);
    e->prof = enable != 0;
    e->recs.clear();
    e->used = 0;
    return ORBX_OK;
}

int lba_profile_read(lba_engine *e, int idx, char *name, int name_cap, double *total_ms, int *launches) {
    if (!e || idx < 0) return ORBX_EINVAL;
    std::vector<std::string> names;
    for (auto &r : e->recs) {
        LBA_CHK(hipEventSynchronize(r.b));
        if (std::find(names.begin(), names.end(), std::string(r.name)) == names.end()) names.push_back(r.name);
    }
    if (idx >= (int)names.size()) return ORBX_ESTATE;
    double tot = 0;
    int cnt = 0;
    for (auto &r : e->recs) {
        if (names[idx] != r.name) continue;
        float ms = 0;
        LBA_CHK(hipEventElapsedTime(&ms, r.a, r.b));
        tot += ms;
        cnt++;
    }
    if (name && name_cap > 0) std::snprintf(name, (size_t)name_cap, "%s", names[idx].c_str());
    if (total_ms) *total_ms = tot;
    if (launches) *launches = cnt;
    return ORBX_OK;
}

}  // extern "C"
