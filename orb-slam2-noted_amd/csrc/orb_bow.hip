// MI355X-native Frame::ComputeBoW (Frame.cc:704-719): DBoW2 TemplatedVocabulary::transform
// (TemplatedVocabulary.h:1125-1286) of a frame's ORB descriptors into its BowVector and
// FeatureVector.
//
// Vocabulary in HBM: children of every node stored contiguously in push_back (file) order as
// a CSR (child_start / child count) with the children's 32-byte descriptors packed in the same
// order, so one descent level reads k consecutive descriptors.
//   bow_descend_kernel    one thread per (frame, feature): L levels of k Hamming distances
//                         (first minimum, FORB::distance), the leaf's word id / weight and the
//                         node `levelsup` above the leaves
//   bow_aggregate_kernel  one workgroup per frame: (word, feature) and (node, feature) keys
//                         bitonic-sorted in LDS; each word's weight summed in feature order
//                         (BowVector::addWeight order), the L1/L2 norm summed in word order
//                         (BowVector::normalize) -> bit-identical doubles to the reference order
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "orb_engine.h"
#include "orbslam2_amd.h"

using namespace orbamd;

#define BW_CHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd bow: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace orbbow {

constexpr int kMaxFeat = 4096;   // features per frame sorted in LDS

struct VocabDev {
    const int *child_start;    // [n_nodes + 1]
    const int *child_node;     // [n_nodes] CSR order
    const uint4 *child_desc;   // [n_nodes][2] CSR order
    const int *word_id;        // [n_nodes]
    const double *weight;      // [n_nodes]
    int L, scoring, weighting;
};

__device__ inline int hamming(const uint4 a0, const uint4 a1, const uint4 *b) {
    const uint4 b0 = b[0], b1 = b[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(256) void bow_descend_kernel(VocabDev V, const uint8_t *desc, const int *counts, int cap,
                                                          long long frame_stride, int levelsup, int ocap, int *word,
                                                          double *wt, int *nid_out) {
    const int i = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (i >= min(counts[f], cap)) return;
    const uint4 *q = (const uint4 *)(desc + f * frame_stride + (long long)i * 32);
    const uint4 a0 = q[0], a1 = q[1];
    const int nid_level = V.L - levelsup;
    int nid = 0, final_id = 0, level = 0;
    while (true) {                                   // transform(feature, id, w, nid, levelsup)
        ++level;
        const int a = V.child_start[final_id], b = V.child_start[final_id + 1];
        int best = a, best_d = hamming(a0, a1, V.child_desc + 2LL * a);
        for (int c = a + 1; c < b; c++) {
            const int d = hamming(a0, a1, V.child_desc + 2LL * c);
            if (d < best_d) { best_d = d; best = c; }
        }
        final_id = V.child_node[best];
        if (level == nid_level) nid = final_id;
        if (V.child_start[final_id + 1] == V.child_start[final_id]) break;   // isLeaf()
    }
    const long long o = (long long)f * ocap + i;
    word[o] = V.word_id[final_id];
    wt[o] = V.weight[final_id];
    nid_out[o] = nid;
}

__device__ inline void bitonic_u64(unsigned long long *k, int n2) {
    for (int size = 2; size <= n2; size <<= 1)
        for (int j = size >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = k[i], y = k[ixj];
                    const bool asc = (i & size) == 0;
                    if (asc ? (x > y) : (x < y)) { k[i] = y; k[ixj] = x; }
                }
            }
            __syncthreads();
        }
}

struct BowOut {
    uint32_t *words;    // [F][cap]
    double *values;     // [F][cap]
    int *n_words;       // [F]
    uint32_t *fv_nodes; // [F][cap]
    int *fv_start;      // [F][cap + 1]
    int *fv_feat;       // [F][cap]
    int *n_fv;          // [F]
};

// exclusive rank of segment heads (keys sorted, head = first of equal key >> 32) over [0, m)
__device__ inline int head_ranks(const unsigned long long *keys, int m, int sort_cap, int *rank, int *part) {
    const int tid = threadIdx.x, per = sort_cap / 256;   // sort_cap >= 256 (multiple of 256)
    const int lo = tid * per;
    int cnt = 0;
    for (int j = lo; j < lo + per; j++)
        cnt += j < m && (j == 0 || (uint32_t)(keys[j] >> 32) != (uint32_t)(keys[j - 1] >> 32));
    part[tid] = cnt;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {              // inclusive Hillis-Steele scan
        const int v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int r = part[tid] - cnt;
    for (int j = lo; j < lo + per; j++) {
        const bool h = j < m && (j == 0 || (uint32_t)(keys[j] >> 32) != (uint32_t)(keys[j - 1] >> 32));
        rank[j] = h ? r : -1;
        r += h;
    }
    const int total = part[255];
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(256) void bow_aggregate_kernel(VocabDev V, const int *counts, int cap, int sort_cap,
                                                            int ocap, const int *word, const double *wt,
                                                            const int *nid, BowOut O) {
    extern __shared__ unsigned long long keys[];              // [sort_cap]
    double *vals = (double *)(keys + sort_cap);               // [sort_cap]
    int *rank = (int *)(vals + sort_cap);                     // [sort_cap]
    __shared__ int part[256];
    __shared__ int s_m;
    __shared__ double s_norm;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = min(counts[f], cap);
    const long long base = (long long)f * ocap;
    // BowVector: (word << 32 | feature) for features that are not stopped (w > 0)
    for (int i = tid; i < sort_cap; i += 256) {
        unsigned long long k = ~0ull;
        if (i < n && wt[base + i] > 0) k = ((unsigned long long)(uint32_t)word[base + i] << 32) | (uint32_t)i;
        keys[i] = k;
    }
    if (tid == 0) s_m = 0;
    __syncthreads();
    bitonic_u64(keys, sort_cap);
    int cnt = 0;
    for (int i = tid; i < sort_cap; i += 256) cnt += keys[i] != ~0ull;
    atomicAdd(&s_m, cnt);
    __syncthreads();
    const int m = s_m;
    const int nw = head_ranks(keys, m, sort_cap, rank, part);
    const bool tf = V.weighting == 0 || V.weighting == 1;
    uint32_t *W = O.words + base;
    double *Vv = O.values + base;
    for (int j = tid; j < m; j += 256) {
        const int r = rank[j];
        if (r < 0) continue;
        const uint32_t w = (uint32_t)(keys[j] >> 32);
        double acc = wt[base + (uint32_t)keys[j]];
        if (tf)   // BowVector::addWeight in feature order; addIfNotExist keeps the first
            for (int e = j + 1; e < m && (uint32_t)(keys[e] >> 32) == w; e++) acc += wt[base + (uint32_t)keys[e]];
        W[r] = w;
        vals[r] = acc;
    }
    __syncthreads();
    const bool must = V.scoring != 5;
    if (tid == 0) {   // the norm summed in word order (BowVector::normalize)
        double norm = 0.0;
        if (must) {
            if (V.scoring != 1) for (int j = 0; j < nw; j++) norm += fabs(vals[j]);
            else { for (int j = 0; j < nw; j++) norm += vals[j] * vals[j]; norm = sqrt(norm); }
        }
        s_norm = norm;
        O.n_words[f] = nw;
    }
    __syncthreads();
    const double nd = nw;
    for (int j = tid; j < nw; j += 256) {
        double x = vals[j];
        if (tf && !must) x /= nd;
        if (must && s_norm > 0.0) x /= s_norm;
        Vv[j] = x;
    }
    __syncthreads();
    // FeatureVector: (node << 32 | feature)
    for (int i = tid; i < sort_cap; i += 256) {
        unsigned long long k = ~0ull;
        if (i < n && wt[base + i] > 0) k = ((unsigned long long)(uint32_t)nid[base + i] << 32) | (uint32_t)i;
        keys[i] = k;
    }
    __syncthreads();
    bitonic_u64(keys, sort_cap);
    const int nf = head_ranks(keys, m, sort_cap, rank, part);
    uint32_t *FN = O.fv_nodes + base;
    int *FS = O.fv_start + (long long)f * (ocap + 1), *FF = O.fv_feat + base;
    for (int j = tid; j < m; j += 256) {
        FF[j] = (int)(uint32_t)keys[j];
        const int r = rank[j];
        if (r >= 0) { FN[r] = (uint32_t)(keys[j] >> 32); FS[r] = j; }
    }
    if (tid == 0) { FS[nf] = m; O.n_fv[f] = nf; }
}

}  // namespace orbbow

using namespace orbbow;

struct orbv_vocab {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;          // end of the last run (fetch waits on it only)
    hipStream_t done_stream = nullptr;
    int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
    DevBuf child_start, child_node, child_desc, word_id, weight;
    // batch buffers
    int cap = 0, frames = 0;
    DevBuf in_desc, in_counts, word, wt, nid, o_words, o_values, o_nw, o_fvn, o_fvs, o_fvf, o_nfv;
};

namespace {

VocabDev vdev(orbv_vocab *v) {
    VocabDev V;
    V.child_start = v->child_start.as<int>(); V.child_node = v->child_node.as<int>();
    V.child_desc = v->child_desc.as<uint4>(); V.word_id = v->word_id.as<int>(); V.weight = v->weight.as<double>();
    V.L = v->L; V.scoring = v->scoring; V.weighting = v->weighting;
    return V;
}

int ensure_batch(orbv_vocab *v, int frames, int cap) {
    if (frames <= v->frames && cap <= v->cap) return 0;
    frames = std::max(frames, v->frames);
    cap = std::max(cap, v->cap);
    const size_t F = (size_t)frames, C = (size_t)cap;
    if (v->word.ensure(4 * F * C) || v->wt.ensure(8 * F * C) || v->nid.ensure(4 * F * C) || v->o_words.ensure(4 * F * C) ||
        v->o_values.ensure(8 * F * C) || v->o_nw.ensure(4 * F) || v->o_fvn.ensure(4 * F * C) ||
        v->o_fvs.ensure(4 * F * (C + 1)) || v->o_fvf.ensure(4 * F * C) || v->o_nfv.ensure(4 * F))
        return -1;
    v->frames = frames;
    v->cap = cap;
    return 0;
}

int launch(orbv_vocab *v, const uint8_t *d_desc, const int32_t *d_counts, int n_frames, int cap, size_t stride,
           int levelsup, hipStream_t st) {
    if (order_after_done(v, st) != hipSuccess) return -1;
    int sc = 256;
    while (sc < cap) sc <<= 1;
    bow_descend_kernel<<<dim3((cap + 255) / 256, n_frames), 256, 0, st>>>(vdev(v), d_desc, d_counts, cap, (long long)stride,
                                                                          levelsup, v->cap, v->word.as<int>(),
                                                                          v->wt.as<double>(), v->nid.as<int>());
    BowOut O;
    O.words = v->o_words.as<uint32_t>(); O.values = v->o_values.as<double>(); O.n_words = v->o_nw.as<int>();
    O.fv_nodes = v->o_fvn.as<uint32_t>(); O.fv_start = v->o_fvs.as<int>(); O.fv_feat = v->o_fvf.as<int>();
    O.n_fv = v->o_nfv.as<int>();
    bow_aggregate_kernel<<<n_frames, 256, (8 + 8 + 4) * (size_t)sc, st>>>(vdev(v), d_counts, cap, sc, v->cap,
                                                                                 v->word.as<int>(), v->wt.as<double>(),
                                                                                 v->nid.as<int>(), O);
    if (hipGetLastError() != hipSuccess) return -1;
    return mark_done(v, st) == hipSuccess ? 0 : -1;
}

}  // namespace

extern "C" {

int orbv_create(int k, int L, int scoring, int weighting, int n_nodes, const int32_t *parent, const uint8_t *is_leaf,
                const uint8_t *desc, const double *weight, orbv_vocab **out) {
    if (!out || n_nodes < 1 || !parent || !is_leaf || !desc || !weight || scoring < 0 || scoring > 5 || weighting < 0 ||
        weighting > 3 || L < 1)
        return ORBX_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ORBX_EDEVICE;
    // loadFromTextFile order: children pushed back in node order, words to leaves in node order
    std::vector<int> cs(n_nodes + 1, 0), cn(std::max(1, n_nodes - 1)), wid(n_nodes, 0), fill(n_nodes, 0);
    for (int i = 1; i < n_nodes; i++) {
        if (parent[i] < 0 || parent[i] >= i) return ORBX_EINVAL;
        cs[parent[i] + 1]++;
    }
    for (int i = 0; i < n_nodes; i++) cs[i + 1] += cs[i];
    for (int i = 1; i < n_nodes; i++) cn[cs[parent[i]] + fill[parent[i]]++] = i;
    if (cs[1] == 0) return ORBX_EINVAL;              // root without children
    std::vector<uint8_t> cd(32 * (size_t)std::max(1, n_nodes - 1));
    for (int c = 0; c < n_nodes - 1; c++) std::memcpy(&cd[32 * (size_t)c], desc + 32 * (size_t)cn[c], 32);
    int nw = 0;
    std::vector<double> w(n_nodes);
    for (int i = 0; i < n_nodes; i++) {
        wid[i] = (i > 0 && is_leaf[i]) ? nw++ : 0;
        w[i] = i == 0 ? 0.0 : weight[i];
    }
    orbv_vocab *v = new orbv_vocab();
    if (hipGetDevice(&v->device) != hipSuccess || hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess ||
        !(v->done = make_done_event())) {
        delete v;
        return ORBX_EDEVICE;
    }
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting; v->n_nodes = n_nodes; v->n_words = nw;
    auto up = [&](DevBuf &b, const void *src, size_t bytes) -> bool {
        return b.ensure(std::max<size_t>(bytes, 16)) == 0 &&
               hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!up(v->child_start, cs.data(), 4 * cs.size()) || !up(v->child_node, cn.data(), 4 * cn.size()) ||
        !up(v->child_desc, cd.data(), cd.size()) || !up(v->word_id, wid.data(), 4 * wid.size()) ||
        !up(v->weight, w.data(), 8 * w.size())) {
        orbv_destroy(v);
        return ORBX_EDEVICE;
    }
    *out = v;
    return ORBX_OK;
}

int orbv_load_text(const char *path, orbv_vocab **out) {
    if (!path || !out) return ORBX_EINVAL;
    FILE *f = fopen(path, "r");
    if (!f) return ORBX_EINVAL;
    int k, L, n1, n2;
    std::vector<char> line(1 << 16);
    if (!fgets(line.data(), (int)line.size(), f) || sscanf(line.data(), "%d %d %d %d", &k, &L, &n1, &n2) != 4 || k < 0 ||
        k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
        fclose(f);
        return ORBX_EINVAL;
    }
    std::vector<int32_t> par{-1};
    std::vector<uint8_t> leaf{0}, desc(32, 0);
    std::vector<double> w{0.0};
    while (fgets(line.data(), (int)line.size(), f)) {
        char *p = line.data();
        while (*p == ' ' || *p == '\t') p++;
        if (*p == '\n' || *p == '\r' || *p == 0) continue;   // trailing empty line
        char *end;
        par.push_back((int32_t)strtol(p, &end, 10)); p = end;
        leaf.push_back(strtol(p, &end, 10) > 0); p = end;
        for (int j = 0; j < 32; j++) { desc.push_back((uint8_t)strtol(p, &end, 10)); p = end; }
        w.push_back(strtod(p, &end));
    }
    fclose(f);
    return orbv_create(k, L, n1, n2, (int)par.size(), par.data(), leaf.data(), desc.data(), w.data(), out);
}

void orbv_destroy(orbv_vocab *v) {
    if (!v) return;
    (void)hipSetDevice(v->device);
    if (v->stream) { (void)hipStreamSynchronize(v->stream); (void)hipStreamDestroy(v->stream); }
    if (v->done) { (void)hipEventSynchronize(v->done); (void)hipEventDestroy(v->done); }
    DevBuf *bufs[] = {&v->child_start, &v->child_node, &v->child_desc, &v->word_id, &v->weight, &v->in_desc,
                      &v->in_counts, &v->word, &v->wt, &v->nid, &v->o_words, &v->o_values, &v->o_nw, &v->o_fvn,
                      &v->o_fvs, &v->o_fvf, &v->o_nfv};
    for (DevBuf *b : bufs) b->release();
    delete v;
}

int orbv_info(const orbv_vocab *v, int *n_nodes, int *n_words, int *k, int *L) {
    if (!v) return ORBX_EINVAL;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    if (k) *k = v->k;
    if (L) *L = v->L;
    return ORBX_OK;
}

int orbv_transform_batch_device(orbv_vocab *v, const uint8_t *d_desc, const int32_t *d_counts, int n_frames, int cap,
                                size_t frame_stride, int levelsup, void *stream) {
    if (!v || !d_desc || !d_counts || n_frames <= 0 || cap <= 0 || cap > kMaxFeat) return ORBX_EINVAL;
    BW_CHK(hipSetDevice(v->device));
    if (ensure_batch(v, n_frames, cap)) return ORBX_EDEVICE;
    if (v->n_words == 0) return ORBX_EINVAL;
    if (launch(v, d_desc, d_counts, n_frames, cap, frame_stride, levelsup, stream ? (hipStream_t)stream : v->stream))
        return ORBX_EDEVICE;
    return ORBX_OK;
}

int orbv_batch_fetch(orbv_vocab *v, int frame, uint32_t *words, double *values, int32_t *n_words, uint32_t *fv_nodes,
                     int32_t *fv_start, int32_t *fv_features, int32_t *n_fv) {
    if (!v || frame < 0 || frame >= v->frames || !n_words || !n_fv) return ORBX_EINVAL;
    BW_CHK(hipSetDevice(v->device));
    BW_CHK(hipStreamWaitEvent(v->stream, v->done, 0));
    const size_t C = (size_t)v->cap, f = (size_t)frame;
    BW_CHK(d2h_sync(n_words, (char *)v->o_nw.p + 4 * f, 4, v->stream));
    BW_CHK(d2h_sync(n_fv, (char *)v->o_nfv.p + 4 * f, 4, v->stream));
    int32_t m = 0;
    BW_CHK(d2h_sync(&m, (char *)v->o_fvs.p + 4 * (f * (C + 1) + (size_t)*n_fv), 4, v->stream));
    if (words && *n_words) BW_CHK(d2h_sync(words, (char *)v->o_words.p + 4 * f * C, 4 * (size_t)*n_words, v->stream));
    if (values && *n_words) BW_CHK(d2h_sync(values, (char *)v->o_values.p + 8 * f * C, 8 * (size_t)*n_words, v->stream));
    if (fv_nodes && *n_fv) BW_CHK(d2h_sync(fv_nodes, (char *)v->o_fvn.p + 4 * f * C, 4 * (size_t)*n_fv, v->stream));
    if (fv_start) BW_CHK(d2h_sync(fv_start, (char *)v->o_fvs.p + 4 * f * (C + 1), 4 * ((size_t)*n_fv + 1), v->stream));
    if (fv_features && m) BW_CHK(d2h_sync(fv_features, (char *)v->o_fvf.p + 4 * f * C, 4 * (size_t)m, v->stream));
    return ORBX_OK;
}

int orbv_transform(orbv_vocab *v, const uint8_t *desc, int n, int levelsup, uint32_t *words, double *values,
                   int32_t *n_words, uint32_t *fv_nodes, int32_t *fv_start, int32_t *fv_features, int32_t *n_fv) {
    if (!v || n < 0 || n > kMaxFeat || !n_words || !n_fv || (n > 0 && !desc)) return ORBX_EINVAL;
    *n_words = 0;
    *n_fv = 0;
    if (fv_start) fv_start[0] = 0;
    if (n == 0 || v->n_words == 0) return ORBX_OK;        // empty(): outputs cleared
    BW_CHK(hipSetDevice(v->device));
    if (v->in_desc.ensure(32 * (size_t)n) || v->in_counts.ensure(4)) return ORBX_EDEVICE;
    hipStream_t st = v->stream;
    BW_CHK(hipMemcpyAsync(v->in_desc.p, desc, 32 * (size_t)n, hipMemcpyHostToDevice, st));
    const int32_t cnt = n;
    BW_CHK(hipMemcpyAsync(v->in_counts.p, &cnt, 4, hipMemcpyHostToDevice, st));
    if (ensure_batch(v, 1, n)) return ORBX_EDEVICE;
    if (launch(v, v->in_desc.as<uint8_t>(), v->in_counts.as<int32_t>(), 1, n, 32 * (size_t)n, levelsup, st))
        return ORBX_EDEVICE;
    BW_CHK(hipStreamSynchronize(st));
    // results live in frame 0 with stride v->cap
    return orbv_batch_fetch(v, 0, words, values, n_words, fv_nodes, fv_start, fv_features, n_fv);
}

}  // extern "C"
