// MI355X-native BoW-guided matchers:
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)   ORBmatcher.cc:236-353
//   ORBmatcher::SearchForTriangulation(KF1, KF2, F12, pairs, bOnlyStereo)  ORBmatcher.cc:915-1089
//   ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)  ORBmatcher.cc:760-903
//
// Both walk the FeatureVector nodes the two frames share; a keypoint belongs to exactly one
// node, so the greedy claims (vpMapPointMatches / vbMatched2) never cross nodes and every
// shared node is an independent task: one wavefront per (pair, node) keeps the reference's
// sequential order over the first frame's features of the node, with the second frame's
// features of the node spread over the lanes (distance, filters, then a wave reduction to the
// reference's winner: SearchByBoW = first minimum + second-smallest distance,
// SearchForTriangulation = minimum distance among candidates passing the epipolar checks,
// ties to the last). The rotation-consistency histogram is global per pair and applied by a
// finishing workgroup, which also emits SearchForTriangulation's pairs in idx1 order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "orb_device.h"
#include "orb_engine.h"
#include "orbslam2_amd.h"

using namespace orbamd;

#define BM_CHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd bowmatch: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace orbbm {

constexpr int TH_LOW = 50, HISTO_LENGTH = 30;   // ORBmatcher.cc:56-58
constexpr int kMaxKp = 4096;

struct PairHdr {
    int nA, nB, n_nodes;
    float fxB, fyB, cxB, cyB;
    float sfB[16], s2B[16];
    float F12[9], Cw1[3], T2w[12];
};

struct Slots {
    const PairHdr *hdr;
    const orbx_kp *kA, *kB;     // [S][cap]
    const float *uA, *uB;
    const uint8_t *dA, *dB;     // [S][cap][32]
    const int *mpA, *mpB;
    const uint8_t *badA, *badB;
    const int *fA, *fB;         // FeatureVector features in node order [S][cap]
    const int4 *nodes;          // [S][cap] shared node ranges (a0, a1, b0, b1)
    int cap;
};

struct Work {
    int *out;          // [S][cap]: SearchByBoW matches[nB] / SearchForTriangulation m12[nA]
    int *hist_idx;     // [S][cap]
    int8_t *hist_bin;  // [S][cap]
    int *hist_n;       // [S]
    int *counts;       // [S][30]
    int *nmatch;       // [S]
    int *pairs;        // [S][cap][2]
};


__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}

// two smallest keys over the wave (a <= b per lane on entry)
__device__ inline void wave_min2_u64(unsigned long long &a, unsigned long long &b) {
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long oa = __shfl_xor(a, off), ob = __shfl_xor(b, off);
        const unsigned long long lo = oa < a ? oa : a, hi = oa < a ? a : oa;
        const unsigned long long mb = ob < b ? ob : b;
        a = lo;
        b = hi < mb ? hi : mb;
    }
}

__device__ inline int rot_bin(float a1, float a2) {
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * (HISTO_LENGTH / 360.0f));
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// R * X + t with cv::Mat CV_32F semantics
__device__ inline void mat_rx_t(const float *T, const float *X, float o[3]) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float s = T[4 * i] * X[0];
        s = s + T[4 * i + 1] * X[1];
        s = s + T[4 * i + 2] * X[2];
        o[i] = s + T[4 * i + 3];
    }
}

__global__ __launch_bounds__(256) void bm_init_kernel(Slots S, int tri, Work W) {
    const int s = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const PairHdr &h = S.hdr[s];
    const int n = tri ? h.nA : h.nB;   // tri != 0: output indexed by A's keypoints
    if (i < n) W.out[(long long)s * S.cap + i] = -1;
    if (i < HISTO_LENGTH) W.counts[s * HISTO_LENGTH + i] = 0;
    if (i == 0) { W.hist_n[s] = 0; W.nmatch[s] = 0; }
}

// one wavefront per (slot, shared node); blockIdx.x = node.
// kMode 0 = SearchByBoW(KF, F), 1 = SearchForTriangulation, 2 = SearchByBoW(KF1, KF2)
enum { BM_BOW = 0, BM_TRI = 1, BM_BOWKF = 2 };
template <int kMode>
__global__ __launch_bounds__(64) void bm_node_kernel(Slots S, float nnratio, int only_stereo, int check_ori, Work W) {
    extern __shared__ uint8_t claimed[];   // B positions of this node (vbMatched2 / vpMapPointMatches)
    constexpr bool kTri = kMode == BM_TRI;
    const int s = blockIdx.y, node = blockIdx.x, lane = threadIdx.x;
    const PairHdr &h = S.hdr[s];
    if (node >= h.n_nodes) return;
    const long long kb = (long long)s * S.cap;
    const int4 r = S.nodes[kb + node];
    const int nb = r.w - r.z;
    for (int p = lane; p < nb; p += 64) claimed[p] = 0;
    float ex = 0.f, ey = 0.f;
    if (kTri) {   // epipole of KF1's centre in KF2 (ORBmatcher.cc:925-934)
        float C2[3];
        mat_rx_t(h.T2w, h.Cw1, C2);
        const float invz = 1.0f / C2[2];
        ex = h.fxB * C2[0] * invz + h.cxB;
        ey = h.fyB * C2[1] * invz + h.cyB;
    }
    wave_lds_sync();
    int nm = 0;
    for (int u = r.x; u < r.y; u++) {
        const int ia = S.fA[kb + u];
        const long long ga = kb + ia;
        if (!kTri) {
            if (S.mpA[ga] < 0 || (S.badA && S.badA[ga])) continue;
        } else {
            if (S.mpA[ga] >= 0) continue;                        // GetMapPoint(idx1) != NULL
            if (only_stereo && !(S.uA[ga] >= 0)) continue;
        }
        const uint8_t *da = S.dA + ga * 32;
        const orbx_kp kp1 = S.kA[ga];
        const bool st1 = S.uA[ga] >= 0;
        unsigned long long k1 = ~0ull, k2 = ~0ull;
        for (int p = lane; p < nb; p += 64) {
            if (claimed[p]) continue;
            const int ib = S.fB[kb + r.z + p];
            const long long gb = kb + ib;
            if (!kTri) {
                if (kMode == BM_BOWKF && (S.mpB[gb] < 0 || S.badB[gb])) continue;   // :822-826
                const unsigned long long key = ((unsigned long long)hamming32(da, S.dB + gb * 32) << 32) | (unsigned)p;
                if (key < k1) { k2 = k1; k1 = key; } else if (key < k2) k2 = key;
            } else {
                if (S.mpB[gb] >= 0) continue;
                const bool st2 = S.uB[gb] >= 0;
                if (only_stereo && !st2) continue;
                const int dist = hamming32(da, S.dB + gb * 32);
                if (dist > TH_LOW) continue;
                const orbx_kp kp2 = S.kB[gb];
                if (!st1 && !st2) {
                    const float distex = ex - kp2.x, distey = ey - kp2.y;
                    if (distex * distex + distey * distey < 100 * h.sfB[kp2.octave]) continue;
                }
                // CheckDistEpipolarLine (ORBmatcher.cc:211-231)
                const float *F = h.F12;
                const float a = kp1.x * F[0] + kp1.y * F[3] + F[6];
                const float b = kp1.x * F[1] + kp1.y * F[4] + F[7];
                const float c = kp1.x * F[2] + kp1.y * F[5] + F[8];
                const float num = a * kp2.x + b * kp2.y + c;
                const float den = a * a + b * b;
                if (den == 0) continue;
                const float dsqr = num * num / den;
                if (!((double)dsqr < 3.84 * (double)h.s2B[kp2.octave])) continue;
                // minimum distance, ties to the last position (ORBmatcher.cc:990-1000)
                const unsigned long long key = ((unsigned long long)dist << 32) | (0xFFFFFFFFu - (unsigned)p);
                if (key < k1) k1 = key;
            }
        }
        int win = -1;
        if (!kTri) {
            wave_min2_u64(k1, k2);
            const int d1 = k1 == ~0ull ? 256 : (int)(k1 >> 32), d2 = k2 == ~0ull ? 256 : (int)(k2 >> 32);
            const bool gate = kMode == BM_BOWKF ? d1 < TH_LOW : d1 <= TH_LOW;   // :845 strict for (KF, KF)
            if (gate && (float)d1 < nnratio * (float)d2) win = (int)(unsigned)k1;
        } else {
            k1 = wave_min_u64(k1);
            if (k1 != ~0ull) win = (int)(0xFFFFFFFFu - (unsigned)k1);
        }
        if (win < 0) continue;
        const int ib = S.fB[kb + r.z + win];
        if (lane == 0) {
            claimed[win] = 1;
            if (kMode == BM_BOW) W.out[kb + ib] = S.mpA[ga];      // vpMapPointMatches[bestIdxF] = pMP
            else if (kMode == BM_TRI) W.out[kb + ia] = ib;       // vMatches12[idx1] = bestIdx2
            else W.out[kb + ia] = S.mpB[kb + ib];                 // vpMatches12[idx1] = vpMapPoints2[bestIdx2]
            if (check_ori) {
                const int bin = rot_bin(kp1.angle, S.kB[kb + ib].angle);
                const int slot = atomicAdd(&W.hist_n[s], 1);
                W.hist_idx[kb + slot] = kMode == BM_BOW ? ib : ia;
                W.hist_bin[kb + slot] = (int8_t)bin;
                atomicAdd(&W.counts[s * HISTO_LENGTH + bin], 1);
            }
        }
        nm++;
        wave_lds_sync();
    }
    if (lane == 0 && nm) atomicAdd(&W.nmatch[s], nm);
}

// rotation consistency (ComputeThreeMaxima, ORBmatcher.cc:2076-2118) + pair emission
__global__ __launch_bounds__(256) void bm_finish_kernel(Slots S, int tri, int check_ori, Work W) {
    __shared__ int top[3], s_removed, part[256];
    const int s = blockIdx.x, tid = threadIdx.x;
    const PairHdr &h = S.hdr[s];
    const long long kb = (long long)s * S.cap;
    if (tid == 0) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        if (check_ori) {
            int max1 = 0, max2 = 0, max3 = 0;
            for (int i = 0; i < HISTO_LENGTH; i++) {
                const int v = W.counts[s * HISTO_LENGTH + i];
                if (v > max1) { max3 = max2; max2 = max1; max1 = v; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (v > max2) { max3 = max2; max2 = v; ind3 = ind2; ind2 = i; }
                else if (v > max3) { max3 = v; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
        }
        top[0] = ind1; top[1] = ind2; top[2] = ind3;
        s_removed = 0;
    }
    __syncthreads();
    if (check_ori) {
        const int nh = W.hist_n[s];
        int rem = 0;
        for (int k = tid; k < nh; k += 256) {
            const int b = W.hist_bin[kb + k];
            if (b == top[0] || b == top[1] || b == top[2]) continue;
            W.out[kb + W.hist_idx[kb + k]] = -1;
            rem++;
        }
        atomicAdd(&s_removed, rem);
    }
    __syncthreads();
    if (tid == 0) W.nmatch[s] -= s_removed;
    if (tri != 1) return;
    // vMatchedPairs in idx1 order: exclusive scan of (m12[i] >= 0)
    const int n = h.nA, per = (n + 255) / 256, lo = tid * per;
    int cnt = 0;
    for (int i = lo; i < min(n, lo + per); i++) cnt += W.out[kb + i] >= 0;
    part[tid] = cnt;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const int v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int rk = part[tid] - cnt;
    for (int i = lo; i < min(n, lo + per); i++) {
        const int m = W.out[kb + i];
        if (m >= 0) { W.pairs[(kb + rk) * 2] = i; W.pairs[(kb + rk) * 2 + 1] = m; rk++; }
    }
}

}  // namespace orbbm

using namespace orbbm;

struct orbb_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;          // end of the last run (fetch waits on it only)
    hipStream_t done_stream = nullptr;
    int nslots = 0, cap = 0;
    DevBuf hdr, kA, kB, uA, uB, dA, dB, mpA, mpB, badA, badB, fA, fB, nodes;
    DevBuf out, hidx, hbin, hn, counts, nmatch, pairs;
    std::vector<PairHdr> h;
};

namespace {

Slots make_slots(orbb_engine *e) {
    Slots S;
    S.hdr = e->hdr.as<PairHdr>();
    S.kA = e->kA.as<orbx_kp>(); S.kB = e->kB.as<orbx_kp>(); S.uA = e->uA.as<float>(); S.uB = e->uB.as<float>();
    S.dA = e->dA.as<uint8_t>(); S.dB = e->dB.as<uint8_t>(); S.mpA = e->mpA.as<int>(); S.mpB = e->mpB.as<int>();
    S.badA = e->badA.as<uint8_t>(); S.badB = e->badB.as<uint8_t>(); S.fA = e->fA.as<int>(); S.fB = e->fB.as<int>(); S.nodes = e->nodes.as<int4>();
    S.cap = e->cap;
    return S;
}

Work make_work(orbb_engine *e) {
    Work W;
    W.out = e->out.as<int>(); W.hist_idx = e->hidx.as<int>(); W.hist_bin = e->hbin.as<int8_t>();
    W.hist_n = e->hn.as<int>(); W.counts = e->counts.as<int>(); W.nmatch = e->nmatch.as<int>();
    W.pairs = e->pairs.as<int>();
    return W;
}

int validate(const orbb_keyframe *k, int cap) {
    if (!k || k->n < 0 || k->n > cap || k->n_fv < 0 || k->nlevels < 1 || k->nlevels > 16) return ORBX_EINVAL;
    if (k->n > 0 && (!k->keys_un || !k->u_right || !k->desc || !k->mp)) return ORBX_EINVAL;
    if (k->n_fv > 0 && (!k->fv_nodes || !k->fv_start || !k->fv_features)) return ORBX_EINVAL;
    if (k->n_fv > 0 && (k->fv_start[0] != 0 || k->fv_start[k->n_fv] > k->n)) return ORBX_EINVAL;
    for (int j = 0; j < k->n_fv; j++) {
        if (k->fv_start[j + 1] < k->fv_start[j] || (j && k->fv_nodes[j] <= k->fv_nodes[j - 1])) return ORBX_EINVAL;
    }
    for (int j = 0; k->n_fv > 0 && j < k->fv_start[k->n_fv]; j++)
        if (k->fv_features[j] < 0 || k->fv_features[j] >= k->n) return ORBX_EINVAL;
    for (int i = 0; i < k->n; i++)
        if (k->keys_un[i].octave < 0 || k->keys_un[i].octave >= k->nlevels) return ORBX_EINVAL;
    return ORBX_OK;
}

}  // namespace

extern "C" {

int orbb_create(orbb_engine **out) {
    if (!out) return ORBX_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return ORBX_EDEVICE;
    orbb_engine *e = new orbb_engine();
    if (hipGetDevice(&e->device) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        !(e->done = make_done_event())) {
        delete e;
        return ORBX_EDEVICE;
    }
    *out = e;
    return ORBX_OK;
}

void orbb_destroy(orbb_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) { (void)hipStreamSynchronize(e->stream); (void)hipStreamDestroy(e->stream); }
    if (e->done) { (void)hipEventSynchronize(e->done); (void)hipEventDestroy(e->done); }
    DevBuf *bufs[] = {&e->hdr, &e->kA, &e->kB, &e->uA, &e->uB, &e->dA, &e->dB, &e->mpA, &e->mpB, &e->badA, &e->badB, &e->fA,
                      &e->fB, &e->nodes, &e->out, &e->hidx, &e->hbin, &e->hn, &e->counts, &e->nmatch, &e->pairs};
    for (DevBuf *b : bufs) b->release();
    delete e;
}

int orbb_reserve(orbb_engine *e, int n_slots, int cap_kp) {
    if (!e || n_slots <= 0 || cap_kp <= 0 || cap_kp > kMaxKp) return ORBX_EINVAL;
    BM_CHK(hipSetDevice(e->device));
    const size_t S = (size_t)n_slots, C = (size_t)cap_kp;
    if (e->hdr.ensure(sizeof(PairHdr) * S) || e->kA.ensure(sizeof(orbx_kp) * S * C) || e->kB.ensure(sizeof(orbx_kp) * S * C) ||
        e->uA.ensure(4 * S * C) || e->uB.ensure(4 * S * C) || e->dA.ensure(32 * S * C) || e->dB.ensure(32 * S * C) ||
        e->mpA.ensure(4 * S * C) || e->mpB.ensure(4 * S * C) || e->badA.ensure(S * C) || e->badB.ensure(S * C) || e->fA.ensure(4 * S * C) ||
        e->fB.ensure(4 * S * C) || e->nodes.ensure(16 * S * C) || e->out.ensure(4 * S * C) || e->hidx.ensure(4 * S * C) ||
        e->hbin.ensure(S * C) || e->hn.ensure(4 * S) || e->counts.ensure(4 * S * HISTO_LENGTH) || e->nmatch.ensure(4 * S) ||
        e->pairs.ensure(8 * S * C))
        return ORBX_EDEVICE;
    e->nslots = n_slots;
    e->cap = cap_kp;
    e->h.assign(n_slots, PairHdr{});
    return ORBX_OK;
}

int orbb_stage(orbb_engine *e, int slot, const orbb_keyframe *a, const orbb_keyframe *b, const float F12[9],
               const float Cw1[3], const float T2w[12]) {
    if (!e || slot < 0 || slot >= e->nslots) return ORBX_EINVAL;
    int rc = validate(a, e->cap);
    if (!rc) rc = validate(b, e->cap);
    if (rc) return rc;
    BM_CHK(hipSetDevice(e->device));
    PairHdr &h = e->h[slot];
    h = PairHdr{};
    h.nA = a->n; h.nB = b->n;
    h.fxB = b->fx; h.fyB = b->fy; h.cxB = b->cx; h.cyB = b->cy;
    std::memcpy(h.sfB, b->scale_factors, sizeof h.sfB);
    std::memcpy(h.s2B, b->level_sigma2, sizeof h.s2B);
    if (F12) std::memcpy(h.F12, F12, sizeof h.F12);
    if (Cw1) std::memcpy(h.Cw1, Cw1, sizeof h.Cw1);
    if (T2w) std::memcpy(h.T2w, T2w, sizeof h.T2w);
    // shared FeatureVector nodes (the reference's merge loop with lower_bound)
    std::vector<int4> nodes;
    for (int i = 0, j = 0; i < a->n_fv && j < b->n_fv;) {
        if (a->fv_nodes[i] == b->fv_nodes[j]) {
            nodes.push_back(make_int4(a->fv_start[i], a->fv_start[i + 1], b->fv_start[j], b->fv_start[j + 1]));
            i++; j++;
        } else if (a->fv_nodes[i] < b->fv_nodes[j]) i++;
        else j++;
    }
    h.n_nodes = (int)nodes.size();
    const size_t C = (size_t)e->cap, s = (size_t)slot;
    hipStream_t st = e->stream;
    BM_CHK(order_after_done(e, st));
    auto up = [&](DevBuf &bf, size_t off, const void *src, size_t bytes) -> bool {
        return bytes == 0 || !src || hipMemcpyAsync((char *)bf.p + off, src, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
    };
    const size_t na = (size_t)a->n, nbk = (size_t)b->n;
    const size_t fa = a->n_fv ? (size_t)a->fv_start[a->n_fv] : 0, fb = b->n_fv ? (size_t)b->fv_start[b->n_fv] : 0;
    bool ok = up(e->hdr, sizeof(PairHdr) * s, &h, sizeof h) && up(e->kA, sizeof(orbx_kp) * s * C, a->keys_un, sizeof(orbx_kp) * na) &&
              up(e->kB, sizeof(orbx_kp) * s * C, b->keys_un, sizeof(orbx_kp) * nbk) && up(e->uA, 4 * s * C, a->u_right, 4 * na) &&
              up(e->uB, 4 * s * C, b->u_right, 4 * nbk) && up(e->dA, 32 * s * C, a->desc, 32 * na) &&
              up(e->dB, 32 * s * C, b->desc, 32 * nbk) && up(e->mpA, 4 * s * C, a->mp, 4 * na) &&
              up(e->mpB, 4 * s * C, b->mp, 4 * nbk) && up(e->fA, 4 * s * C, a->fv_features, 4 * fa) &&
              up(e->fB, 4 * s * C, b->fv_features, 4 * fb) && up(e->nodes, 16 * s * C, nodes.data(), 16 * nodes.size());
    if (ok) {
        if (a->mp_bad) ok = up(e->badA, s * C, a->mp_bad, na);
        else ok = hipMemsetAsync((char *)e->badA.p + s * C, 0, na, st) == hipSuccess;
    }
    if (ok) {
        if (b->mp_bad) ok = up(e->badB, s * C, b->mp_bad, nbk);
        else ok = hipMemsetAsync((char *)e->badB.p + s * C, 0, nbk, st) == hipSuccess;
    }
    if (!ok) return ORBX_EDEVICE;
    BM_CHK(hipStreamSynchronize(st));
    return ORBX_OK;
}

static int run(orbb_engine *e, int n_slots, int mode, float nnratio, int only_stereo, int check_ori, void *stream) {
    if (!e || n_slots <= 0 || n_slots > e->nslots) return ORBX_EINVAL;
    BM_CHK(hipSetDevice(e->device));
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    BM_CHK(order_after_done(e, st));
    int maxn = 1, maxnodes = 1;
    for (int s = 0; s < n_slots; s++) {
        maxn = std::max(maxn, std::max(e->h[s].nA, e->h[s].nB));
        maxnodes = std::max(maxnodes, e->h[s].n_nodes);
    }
    const Slots S = make_slots(e);
    const Work W = make_work(e);
    bm_init_kernel<<<dim3((std::max(maxn, HISTO_LENGTH) + 255) / 256, n_slots), 256, 0, st>>>(S, mode, W);
    const dim3 grid(maxnodes, n_slots);
    if (mode == BM_TRI) bm_node_kernel<BM_TRI><<<grid, 64, e->cap, st>>>(S, nnratio, only_stereo, check_ori, W);
    else if (mode == BM_BOWKF) bm_node_kernel<BM_BOWKF><<<grid, 64, e->cap, st>>>(S, nnratio, only_stereo, check_ori, W);
    else bm_node_kernel<BM_BOW><<<grid, 64, e->cap, st>>>(S, nnratio, only_stereo, check_ori, W);
    bm_finish_kernel<<<n_slots, 256, 0, st>>>(S, mode, check_ori, W);
    BM_CHK(hipGetLastError());
    BM_CHK(mark_done(e, st));
    return ORBX_OK;
}

int orbb_run_bow_batch(orbb_engine *e, int n_slots, float nnratio, int check_ori, void *stream) {
    return run(e, n_slots, BM_BOW, nnratio, 0, check_ori, stream);
}

int orbb_run_tri_batch(orbb_engine *e, int n_slots, int only_stereo, int check_ori, void *stream) {
    return run(e, n_slots, BM_TRI, 0.6f, only_stereo, check_ori, stream);
}

int orbb_run_bowkf_batch(orbb_engine *e, int n_slots, float nnratio, int check_ori, void *stream) {
    return run(e, n_slots, BM_BOWKF, nnratio, 0, check_ori, stream);
}

int orbb_fetch(orbb_engine *e, int slot, int tri, int32_t *out, int32_t *n) {
    if (!e || slot < 0 || slot >= e->nslots || !out || !n) return ORBX_EINVAL;
    BM_CHK(hipSetDevice(e->device));
    BM_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    const size_t C = (size_t)e->cap, s = (size_t)slot;
    BM_CHK(d2h_sync(n, (char *)e->nmatch.p + 4 * s, 4, e->stream));
    if (tri == 0 || tri == 2) {   // matches[b.n] (SearchByBoW(KF, F)) / matches12[a.n] (SearchByBoW(KF1, KF2))
        const size_t m = (size_t)(tri == 0 ? e->h[slot].nB : e->h[slot].nA);
        if (m) BM_CHK(d2h_sync(out, (char *)e->out.p + 4 * s * C, 4 * m, e->stream));
    } else if (*n > 0) {
        BM_CHK(d2h_sync(out, (char *)e->pairs.p + 8 * s * C, 8 * (size_t)*n, e->stream));
    }
    return ORBX_OK;
}

int orbb_search_by_bow(orbb_engine *e, const orbb_keyframe *kf, const orbb_keyframe *f, float nnratio, int check_ori,
                       int32_t *matches, int32_t *nmatches) {
    if (!e || !kf || !f || !matches || !nmatches) return ORBX_EINVAL;
    const int need = std::max(1, std::max(kf->n, f->n));
    if (e->nslots < 1 || e->cap < need) {
        const int rc = orbb_reserve(e, std::max(1, e->nslots), std::max(e->cap, need));
        if (rc) return rc;
    }
    int rc = orbb_stage(e, 0, kf, f, nullptr, nullptr, nullptr);
    if (!rc) rc = orbb_run_bow_batch(e, 1, nnratio, check_ori, nullptr);
    if (!rc) rc = orbb_fetch(e, 0, 0, matches, nmatches);
    return rc;
}

int orbb_search_by_bow_kf(orbb_engine *e, const orbb_keyframe *kf1, const orbb_keyframe *kf2, float nnratio, int check_ori,
                          int32_t *matches12, int32_t *nmatches) {
    if (!e || !kf1 || !kf2 || !matches12 || !nmatches) return ORBX_EINVAL;
    const int need = std::max(1, std::max(kf1->n, kf2->n));
    if (e->nslots < 1 || e->cap < need) {
        const int rc = orbb_reserve(e, std::max(1, e->nslots), std::max(e->cap, need));
        if (rc) return rc;
    }
    int rc = orbb_stage(e, 0, kf1, kf2, nullptr, nullptr, nullptr);
    if (!rc) rc = orbb_run_bowkf_batch(e, 1, nnratio, check_ori, nullptr);
    if (!rc) rc = orbb_fetch(e, 0, 2, matches12, nmatches);
    return rc;
}

int orbb_search_for_triangulation(orbb_engine *e, const orbb_keyframe *kf1, const orbb_keyframe *kf2, const float F12[9],
                                  const float Cw1[3], const float T2w[12], int only_stereo, int check_ori,
                                  int32_t *pairs, int32_t *npairs) {
    if (!e || !kf1 || !kf2 || !F12 || !Cw1 || !T2w || !pairs || !npairs) return ORBX_EINVAL;
    const int need = std::max(1, std::max(kf1->n, kf2->n));
    if (e->nslots < 1 || e->cap < need) {
        const int rc = orbb_reserve(e, std::max(1, e->nslots), std::max(e->cap, need));
        if (rc) return rc;
    }
    int rc = orbb_stage(e, 0, kf1, kf2, F12, Cw1, T2w);
    if (!rc) rc = orbb_run_tri_batch(e, 1, only_stereo, check_ori, nullptr);
    if (!rc) rc = orbb_fetch(e, 0, 1, pairs, npairs);
    return rc;
}

}  // extern "C"
