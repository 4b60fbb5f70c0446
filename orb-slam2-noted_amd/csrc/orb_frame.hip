// MI355X-native per-frame front end around the extractor (C3 config):
//   * Frame::UndistortKeyPoints (Frame.cc:725-776; cv::undistortPoints) +
//     Frame::ComputeStereoFromRGBD (Frame.cc:1131-1169)        -> rgbd_kernel
//   * Frame grid (AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea, Frame.cc:398-698)
//     as a per-frame sorted (cell, index) key list             -> grid_sort_kernel
//   * ORBmatcher::SearchForInitialization (ORBmatcher.cc:580-748) + ComputeThreeMaxima
//     (:2076-2118): windowed candidates and Hamming distances are wave-parallel, the greedy
//     claim / evict order of the reference is kept by walking F1 keypoints in index order
//                                                              -> search_init_kernel
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

#define FR_CHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

namespace orbframe {

constexpr int GRID_COLS = 64, GRID_ROWS = 48;   // Frame.h:55-60
constexpr int GRID_CELLS = GRID_COLS * GRID_ROWS;
// LDS of one search_init_resolve_kernel workgroup: list stage + per-F1 prefix + vMatchedDistance /
// v21 / M12 (u16) + rotation bins (i8). 64 KB holds a 4096-keypoint frame (fixed part 45,076 B,
// stage 5,115 entries >= cap0); two workgroups still fit a CU's 160 KB.
constexpr size_t kSearchLds = 64 * 1024;

struct Camera {
    double fx, fy, cx, cy;
    double k[5];      // k1 k2 p1 p2 k3
    int distorted;    // mDistCoef.at<float>(0) != 0
    float mbf;
};

// cv::undistortPoints(src, dst, K, dist, noArray(), K): 5 fixed iterations in double
__host__ __device__ inline void undistort_point(const Camera &c, float u, float v, float *uo, float *vo) {
    const double ifx = 1. / c.fx, ify = 1. / c.fy;
    double x = u, y = v;
    x = (x - c.cx) * ifx;
    y = (y - c.cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = 1. / (1 + ((c.k[4] * r2 + c.k[1]) * r2 + c.k[0]) * r2);
        const double deltaX = 2 * c.k[2] * x * y + c.k[3] * (r2 + 2 * x * x);
        const double deltaY = c.k[2] * (r2 + 2 * y * y) + 2 * c.k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    *uo = (float)(c.fx * x + c.cx);
    *vo = (float)(c.fy * y + c.cy);
}

// one thread per keypoint of every image in the batch
__global__ __launch_bounds__(256) void rgbd_kernel(Camera cam, const orbx_kp *kps, const int *cnt, int cap,
                                                   const float *depth, long long depth_stride, int dpitch,
                                                   orbx_kp *kun, float *u_right, float *dep_out) {
    const int i = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
    if (i >= cap) return;
    const long long o = (long long)b * cap + i;
    if (i >= cnt[b]) return;
    orbx_kp kp = kps[o];
    orbx_kp ku = kp;
    if (cam.distorted) undistort_point(cam, kp.x, kp.y, &ku.x, &ku.y);
    kun[o] = ku;
    float uR = -1, dd = -1;
    const float d = depth[(long long)b * depth_stride + (long long)(int)kp.y * dpitch + (int)kp.x];
    if (d > 0) {
        dd = d;
        uR = ku.x - cam.mbf / d;
    }
    u_right[o] = uR;
    dep_out[o] = dd;
}

struct GridParams {
    float minX, maxX, minY, maxY, invW, invH;
};

// Per frame: keys (cell << 16 | index) of keypoints that fall in the grid, sorted -> the
// candidate order of GetFeaturesInArea (ix, then iy, then insertion order) -- and the first key
// position of every cell (cstart[c], c = ix * GRID_ROWS + iy; cstart[GRID_CELLS] = the valid key
// count), so a column's cell range [iy0, iy1] is keys [cstart[ix R + iy0], cstart[ix R + iy1 + 1])
// in two loads (a binary search over the keys was ~10 dependent global loads per bound).
__global__ __launch_bounds__(256) void grid_sort_kernel(GridParams gp, const orbx_kp *kun, const int *cnt,
                                                        int cap, int sort_cap, uint32_t *keys, int *nkeys, int *cstart) {
    extern __shared__ uint32_t sk[];
    const int b = blockIdx.x;
    const int n = min(cnt[b], cap);
    for (int i = threadIdx.x; i < sort_cap; i += 256) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n) {
            const orbx_kp k = kun[(long long)b * cap + i];
            const int px = (int)roundf((k.x - gp.minX) * gp.invW);   // PosInGrid (Frame.cc:682-698)
            const int py = (int)roundf((k.y - gp.minY) * gp.invH);
            if (!(px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS))
                key = ((uint32_t)(px * GRID_ROWS + py) << 16) | (uint32_t)i;
        }
        sk[i] = key;
    }
    __syncthreads();
    for (int k = 2; k <= sort_cap; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < sort_cap; i += 256) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t x = sk[i], y = sk[ixj];
                    const bool asc = (i & k) == 0;
                    if (asc ? (x > y) : (x < y)) { sk[i] = y; sk[ixj] = x; }
                }
            }
            __syncthreads();
        }
    __shared__ int valid;
    if (threadIdx.x == 0) valid = 0;
    __syncthreads();
    int mine = 0;
    int *cs = cstart + (long long)b * (GRID_CELLS + 1);
    for (int i = threadIdx.x; i <= sort_cap; i += 256) {
        // cells (cell of key i - 1, cell of key i] start at i (invalid keys: cell GRID_CELLS)
        const int c1 = i < sort_cap ? min((int)(sk[i] >> 16), GRID_CELLS) : GRID_CELLS;
        const int c0 = i > 0 ? min((int)(sk[i - 1] >> 16), GRID_CELLS) : -1;
        for (int c = c0 + 1; c <= c1; c++) cs[c] = i;
        if (i < sort_cap) {
            keys[(long long)b * sort_cap + i] = sk[i];
            mine += sk[i] != 0xFFFFFFFFu;
        }
    }
    atomicAdd(&valid, mine);
    __syncthreads();
    if (threadIdx.x == 0) nkeys[b] = valid;
}



// SearchForInitialization in two phases.
// Phase A (search_init_cand_kernel, one wavefront per F1 keypoint of octave 0, all pairs at
// once): GetFeaturesInArea's candidates in its order (ix, iy, insertion; Frame.cc:631-666),
// level and square-window filtered, with their Hamming distance and rotation bin, compacted
// in order into a per-keypoint list: entry = i2 | dist << 16 | bin << 25. None of this
// depends on the greedy state.
// Phase B (search_init_resolve_kernel, one workgroup per pair): the greedy claim loop over i1
// in index order (ORBmatcher.cc:614-712) on LDS state only -- vMatchedDistance filter, first
// minimum and second distance by a wave min over (dist, position) keys, eviction of the
// previous owner -- then ComputeThreeMaxima pruning (:2076-2118). The lists are staged into LDS
// in chunks by all four wavefronts; wavefront 0 walks them.
struct SearchArgs {
    // F1 = image f1_base + f1_step * p, F2 = image f2_base + f2_step * p
    int f1_base, f1_step, f2_base, f2_step;
    const orbx_kp *kun;
    const uint8_t *desc;
    const int *cnt;
    int cap, sort_cap, cap0;   // cap0: level-0 keypoint capacity (list length bound)
    const uint32_t *keys;      // grid-sorted keys per image
    const int *nkeys;
    const int *cstart;         // per image: first key of every grid cell (GRID_CELLS + 1)
    GridParams gp;
    float r, nnratio;
    int check_ori;
    uint32_t *list;            // [pair][cap0][cap0] candidate entries
    int *lcnt;                 // [pair][cap0] entries per F1 keypoint
    int stage_cap;             // LDS entry budget of phase B
};

__device__ __forceinline__ int rot_bin(float a1, float a2) {   // ORBmatcher.cc:700-707 (factor 30/360)
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (30 / 360.0f));
    if (bin == 30) bin = 0;
    return bin;
}

__global__ __launch_bounds__(256) void search_init_cand_kernel(SearchArgs a, const float *prev_xy) {
    __shared__ int run_pre_s[4][65];
    __shared__ int run_lo_s[4][64];
    const int lane = threadIdx.x & 63, wv = wave_id();
    const int p = blockIdx.y, i1 = blockIdx.x * 4 + wv;
    if (i1 >= a.cap0) return;
    const int i1img = a.f1_base + a.f1_step * p, i2img = a.f2_base + a.f2_step * p;
    const int N1 = min(a.cnt[i1img], a.cap);
    int *cnt_out = a.lcnt + (long long)p * a.cap0 + i1;
    if (i1 >= N1) { if (lane == 0) *cnt_out = 0; return; }
    const orbx_kp *K1 = a.kun + (long long)i1img * a.cap, *K2 = a.kun + (long long)i2img * a.cap;
    const orbx_kp kp1 = K1[i1];
    const float x = prev_xy[((long long)p * a.cap + i1) * 2], y = prev_xy[((long long)p * a.cap + i1) * 2 + 1];
    const float r = a.r;
    // GetFeaturesInArea (Frame.cc:590-671) cell window
    const int nMinCellX = max(0, (int)floorf((x - a.gp.minX - r) * a.gp.invW));
    const int nMaxCellX = min(GRID_COLS - 1, (int)ceilf((x - a.gp.minX + r) * a.gp.invW));
    const int nMinCellY = max(0, (int)floorf((y - a.gp.minY - r) * a.gp.invH));
    const int nMaxCellY = min(GRID_ROWS - 1, (int)ceilf((y - a.gp.minY + r) * a.gp.invH));
    if (kp1.octave > 0 || nMinCellX >= GRID_COLS || nMaxCellX < 0 || nMinCellY >= GRID_ROWS || nMaxCellY < 0) {
        if (lane == 0) *cnt_out = 0;
        return;
    }
    const uint32_t *sk = a.keys + (long long)i2img * a.sort_cap;
    const int *cs = a.cstart + (long long)i2img * (GRID_CELLS + 1);
    int *run_pre = run_pre_s[wv], *run_lo = run_lo_s[wv];
    const int nx = nMaxCellX - nMinCellX + 1;
    int len = 0, lo = 0;
    if (lane < nx) {   // column ix, cells nMinCellY .. nMaxCellY: one key range
        const int ix = nMinCellX + lane;
        lo = cs[ix * GRID_ROWS + nMinCellY];
        len = cs[ix * GRID_ROWS + nMaxCellY + 1] - lo;
    }
    int incl = len;   // exclusive prefix of run lengths over lanes
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    run_pre[lane] = incl - len;
    run_lo[lane] = lo;
    if (lane == 63) run_pre[64] = incl;
    wave_lds_sync();
    const int total = run_pre[64];
    const uint8_t *d1 = a.desc + ((long long)i1img * a.cap + i1) * 32;
    const uint8_t *D2 = a.desc + (long long)i2img * a.cap * 32;
    uint32_t *out = a.list + ((long long)p * a.cap0 + i1) * a.cap0;
    int n = 0;
    for (int base = 0; base < total; base += 64) {
        const int c = base + lane;
        bool keep = false;
        uint32_t ent = 0;
        if (c < total) {
            int rr = 0, hi = min(nx, 64) - 1;   // run containing c
            while (rr < hi) {
                const int m = (rr + hi + 1) >> 1;
                if (run_pre[m] <= c) rr = m; else hi = m - 1;
            }
            const int i2 = (int)(sk[run_lo[rr] + (c - run_pre[rr])] & 0xFFFFu);
            const orbx_kp kp2 = K2[i2];
            // minLevel = maxLevel = 0 (ORBmatcher.cc:626) and the square window (Frame.cc:655)
            if (!(kp2.octave < 0) && !(kp2.octave > 0) && fabsf(kp2.x - x) < r && fabsf(kp2.y - y) < r) {
                const int dist = hamming32(d1, D2 + (long long)i2 * 32);
                const int bin = a.check_ori ? rot_bin(kp1.angle, kp2.angle) : 0;
                ent = (uint32_t)i2 | (uint32_t)dist << 16 | (uint32_t)bin << 25;
                keep = true;
            }
        }
        const unsigned long long bal = __ballot(keep);
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (keep && n + rank < a.cap0) out[n + rank] = ent;
        n += __popcll(bal);
    }
    if (lane == 0) *cnt_out = min(n, a.cap0);
}

__device__ __forceinline__ void min2_merge(uint32_t &k1, uint32_t &k2, uint32_t o1, uint32_t o2) {
    const uint32_t lo = min(k1, o1), hi = max(k1, o1);
    k1 = lo;
    k2 = min(hi, min(k2, o2));
}
// (k1, k2) = the two smallest keys over the 16 lanes of each row: four DPP merge steps (lane ^ 1,
// lane ^ 2, half-row mirror, row mirror) -- VALU latency per step instead of a ds_bpermute round
// trip; every lane of a row ends with its row's pair
template <int CTRL> __device__ __forceinline__ void min2_dpp_step(uint32_t &k1, uint32_t &k2) {
    const uint32_t o1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)k1, CTRL, 0xF, 0xF, false);
    const uint32_t o2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)k2, CTRL, 0xF, 0xF, false);
    min2_merge(k1, k2, o1, o2);
}
__device__ __forceinline__ void min2_row(uint32_t &k1, uint32_t &k2) {
    min2_dpp_step<0xB1>(k1, k2);    // quad_perm [1, 0, 3, 2]
    min2_dpp_step<0x4E>(k1, k2);    // quad_perm [2, 3, 0, 1]
    min2_dpp_step<0x141>(k1, k2);   // row_half_mirror
    min2_dpp_step<0x140>(k1, k2);   // row_mirror
}

// (Measured and not kept: speculative 64-keypoint windows in this walk -- bit-exact, but the kernel
// alone 166 against 150 us per 256-frame batch and the C3 leg +1.2 %: profiles/r05_ab_c3_spec.log,
// tools/archive/pruned_r06.patch.)
__global__ __launch_bounds__(256) void search_init_resolve_kernel(SearchArgs a, float *prev_xy, int *m12, int *nmatch) {
    extern __shared__ uint32_t rs_lds[];
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    const int i1img = a.f1_base + a.f1_step * p, i2img = a.f2_base + a.f2_step * p;
    const int N1 = min(a.cnt[i1img], a.cap);
    const int n1s = min(N1, a.cap0);   // F1 keypoints with a list (octave 0 is a prefix)
    // LDS: stage[stage_cap] u32 | pre[cap0 + 1] i32 | vst[cap] u32 (vMatchedDistance u16 | vnMatches21
    // i16 << 16: one load gives a candidate's both) | M12[cap] i16 | bin[cap] i8
    uint32_t *stage = rs_lds;
    int *pre = (int *)(stage + a.stage_cap);
    uint32_t *vst = (uint32_t *)(pre + a.cap0 + 1);
    int16_t *M12 = (int16_t *)(vst + a.cap);
    int8_t *bin_of = (int8_t *)(M12 + a.cap);
    for (int i = tid; i < a.cap; i += 256) { vst[i] = 0xFFFFFFFFu; M12[i] = -1; bin_of[i] = -1; }
    const int *lc = a.lcnt + (long long)p * a.cap0;
    if (wv == 0) {   // exclusive prefix of list lengths
        int carry = 0;
        for (int b0 = 0; b0 < n1s; b0 += 64) {
            const int v = b0 + lane < n1s ? lc[b0 + lane] : 0;
            int incl = v;
            for (int off = 1; off < 64; off <<= 1) {
                const int t = __shfl_up(incl, off, 64);
                if (lane >= off) incl += t;
            }
            if (b0 + lane < n1s) pre[b0 + lane] = carry + incl - v;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) pre[n1s] = carry;
    }
    __syncthreads();
    const uint32_t *L = a.list + (long long)p * a.cap0 * a.cap0;
    int nmatches = 0;
    for (int s0 = 0; s0 < n1s;) {
        // chunk [s0, e0): as many lists as fit the stage (every list fits: cap0 <= stage_cap)
        int lo = s0 + 1, hi = n1s;
        while (lo < hi) {
            const int m = (lo + hi + 1) >> 1;
            if (pre[m] - pre[s0] <= a.stage_cap) lo = m; else hi = m - 1;
        }
        const int e0 = lo;
        for (int i1 = s0 + wv; i1 < e0; i1 += 4) {
            const int n = pre[i1 + 1] - pre[i1], o = pre[i1] - pre[s0];
            for (int j = lane; j < n; j += 64) stage[o + j] = L[(long long)i1 * a.cap0 + j];
        }
        __syncthreads();
        if (wv == 0) {
            // The walk is one wave's dependent chain and shares its CU with other engines'
            // VALU-bound extraction waves (C3 runs batches on three streams): issue priority keeps
            // each of its instructions from queueing behind theirs
            __builtin_amdgcn_s_setprio(3);
            // The greedy walk, one F1 keypoint after another, as a software pipeline: the next
            // keypoint's list entries and the (vMatchedDistance, vnMatches21) word of each of its
            // candidates are loaded while this one is decided; the loads are issued after every
            // earlier state write (in-order LDS), and the one write they can miss -- this
            // keypoint's claim -- is patched in by comparing with the claimed index. Lists of up
            // to 64 entries (the common case) reduce their two smallest (dist << 12 | position)
            // keys with DPP inside each 16-lane row and a scalar merge over the rows in use.
            auto load = [&](int i1, uint32_t &ent, uint32_t &st) {
                const int n = i1 < e0 ? pre[i1 + 1] - pre[i1] : 0, o = i1 < e0 ? pre[i1] - pre[s0] : 0;
                ent = lane < n ? stage[o + lane] : 0xFFFFFFFFu;
                st = lane < n ? vst[ent & 0xFFFFu] : 0u;
            };
            uint32_t ent, st;
            load(s0, ent, st);
            for (int i1 = s0; i1 < e0; i1++) {
                const int n = pre[i1 + 1] - pre[i1], o = pre[i1] - pre[s0];
                if (n == 0) {
                    load(i1 + 1, ent, st);
                    continue;
                }
                uint32_t k1 = 0xFFFFFFFFu, k2 = 0xFFFFFFFFu;   // two smallest (dist << 12 | position)
                if (n <= 64) {
                    if (lane < n) {
                        const int dist = (int)((ent >> 16) & 0x1FFu);
                        if (!((int)(st & 0xFFFFu) <= dist)) k1 = (uint32_t)dist << 12 | (uint32_t)lane;
                    }
                    min2_row(k1, k2);
                    uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)k1, 0);
                    uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)k2, 0);
                    for (int row = 1; row < (n + 15) / 16; row++)
                        min2_merge(r1, r2, (uint32_t)__builtin_amdgcn_readlane((int)k1, 16 * row),
                                   (uint32_t)__builtin_amdgcn_readlane((int)k2, 16 * row));
                    k1 = r1;
                    k2 = r2;
                } else {   // long list: per-lane pairs over 64-entry groups, then the butterfly
                    for (int j = lane; j < n; j += 64) {
                        const uint32_t e2 = stage[o + j];
                        const int i2 = (int)(e2 & 0xFFFFu), dist = (int)((e2 >> 16) & 0x1FFu);
                        if (!((int)(vst[i2] & 0xFFFFu) <= dist)) min2_merge(k1, k2, (uint32_t)dist << 12 | (uint32_t)j, 0xFFFFFFFFu);
                    }
                    for (int off = 32; off > 0; off >>= 1) {
                        const uint32_t o1 = (uint32_t)__shfl_xor((int)k1, off, 64), o2 = (uint32_t)__shfl_xor((int)k2, off, 64);
                        min2_merge(k1, k2, o1, o2);
                    }
                    k1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
                    k2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k2);
                }
                // the winner's entry and state word, before the next keypoint's loads replace them
                uint32_t went = 0, wst = 0;
                if (k1 != 0xFFFFFFFFu) {
                    const int jw = (int)(k1 & 0xFFFu);
                    if (n <= 64) {
                        went = (uint32_t)__builtin_amdgcn_readlane((int)ent, jw);
                        wst = (uint32_t)__builtin_amdgcn_readlane((int)st, jw);
                    } else {
                        went = stage[o + jw];
                        wst = vst[went & 0xFFFFu];
                    }
                }
                load(i1 + 1, ent, st);   // issued after every earlier claim's writes
                if (k1 == 0xFFFFFFFFu) continue;
                const int bestDist = (int)(k1 >> 12);
                const int bestDist2 = k2 == 0xFFFFFFFFu ? INT_MAX : (int)(k2 >> 12);
                if (bestDist <= 50 && bestDist < (float)bestDist2 * a.nnratio) {   // TH_LOW, mfNNratio
                    const int bestIdx2 = (int)(went & 0xFFFFu);
                    const int prev = (int)(int16_t)(wst >> 16);
                    if (prev >= 0) nmatches--;
                    nmatches++;
                    const uint32_t nst = (uint32_t)(uint16_t)bestDist | (uint32_t)(uint16_t)(int16_t)i1 << 16;
                    if (lane == 0) {
                        if (prev >= 0) M12[prev] = -1;
                        M12[i1] = (int16_t)bestIdx2;
                        vst[bestIdx2] = nst;   // vMatchedDistance | vnMatches21 << 16
                        if (a.check_ori) bin_of[i1] = (int8_t)(went >> 25);
                    }
                    if ((ent & 0xFFFFu) == (uint32_t)bestIdx2 && ent != 0xFFFFFFFFu) st = nst;   // patch the prefetch
                }
            }
            __builtin_amdgcn_s_setprio(0);
        }
        __syncthreads();
        s0 = e0;
    }
    __shared__ int hist[30];
    __shared__ int ind[3];
    __shared__ int removed;
    if (tid < 30) hist[tid] = 0;
    if (tid == 0) removed = 0;
    __syncthreads();
    if (a.check_ori) {   // ComputeThreeMaxima over the acceptance events, prune other bins
        for (int i = tid; i < n1s; i += 256)
            if (bin_of[i] >= 0) atomicAdd(&hist[bin_of[i]], 1);
        __syncthreads();
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < 30; i++) {
                const int s = hist[i];
                if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
                else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
                else if (s > max3) { max3 = s; ind3 = i; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            ind[0] = ind1; ind[1] = ind2; ind[2] = ind3;
        }
        __syncthreads();
        int mine = 0;
        for (int i = tid; i < n1s; i += 256) {
            const int bb = bin_of[i];
            if (bb < 0 || bb == ind[0] || bb == ind[1] || bb == ind[2]) continue;
            if (M12[i] >= 0) { M12[i] = -1; mine++; }
        }
        if (mine) atomicAdd(&removed, mine);
        __syncthreads();
    }
    if (tid == 0) nmatch[p] = nmatches - removed;
    const orbx_kp *K2 = a.kun + (long long)i2img * a.cap;
    float *pxy = prev_xy + (long long)p * a.cap * 2;
    int *out = m12 + (long long)p * a.cap;
    for (int i = tid; i < N1; i += 256) {
        const int m = i < n1s ? (int)M12[i] : -1;
        out[i] = m;
        if (m >= 0) { pxy[2 * i] = K2[m].x; pxy[2 * i + 1] = K2[m].y; }
    }
}

__global__ __launch_bounds__(256) void init_prev_xy(const orbx_kp *kun, const int *cnt, int cap, int f1_base,
                                                    int f1_step, float *prev_xy) {
    const int i = blockIdx.x * 256 + threadIdx.x, p = blockIdx.y;
    if (i >= cap) return;
    const int img = f1_base + f1_step * p;
    float *o = prev_xy + ((long long)p * cap + i) * 2;
    if (i < cnt[img]) {
        const orbx_kp k = kun[(long long)img * cap + i];
        o[0] = k.x; o[1] = k.y;   // mvbPrevMatched[i] = mvKeysUn[i].pt (Tracking.cc)
    }
}

static Camera make_camera(const float K[4], const float dist[5], float mbf) {
    Camera c;
    c.fx = K[0]; c.fy = K[1]; c.cx = K[2]; c.cy = K[3];
    for (int i = 0; i < 5; i++) c.k[i] = dist[i];
    c.distorted = dist[0] != 0.0f;
    c.mbf = mbf;
    return c;
}

// Frame::ComputeImageBounds (Frame.cc:780-830) + grid element inverses (Frame.cc:183-185)
static GridParams make_grid(const Camera &c, int cols, int rows) {
    GridParams g;
    if (c.distorted) {
        float u[4], v[4];
        const float in[8] = {0.f, 0.f, (float)cols, 0.f, 0.f, (float)rows, (float)cols, (float)rows};
        for (int i = 0; i < 4; i++) undistort_point(c, in[2 * i], in[2 * i + 1], &u[i], &v[i]);
        g.minX = std::min(u[0], u[2]);
        g.maxX = std::max(u[1], u[3]);
        g.minY = std::min(v[0], v[1]);
        g.maxY = std::max(v[2], v[3]);
    } else {
        g.minX = 0.0f; g.maxX = (float)cols; g.minY = 0.0f; g.maxY = (float)rows;
    }
    g.invW = (float)GRID_COLS / (g.maxX - g.minX);
    g.invH = (float)GRID_ROWS / (g.maxY - g.minY);
    return g;
}

}  // namespace orbframe

using namespace orbframe;

// Per-engine Frame buffers, owned by the engine (freed by orbx_destroy). kun / uR / dep are
// valid for the extraction generation `kun_gen` (n images x `kun_cap` keypoints); m12 / prev
// for `si_pairs` pairs of the SearchForInitialization run that followed.
struct orbf_state {
    DevBuf kun, uR, dep, keys, nkeys, cstart, prev, m12, nmatch, depth_in, list, lcnt;
    long long kun_gen = -1;
    int kun_n = 0, kun_cap = 0, si_pairs = 0;
};

static orbf_state &fstate(orbx_engine *e) {
    if (!e->fs) e->fs = new orbf_state();
    return *e->fs;
}

namespace orbamd {
void frame_state_free(orbx_engine *e) {
    if (!e->fs) return;
    orbf_state *S = e->fs;
    DevBuf *bufs[] = {&S->kun, &S->uR, &S->dep, &S->keys, &S->nkeys, &S->cstart, &S->prev, &S->m12, &S->nmatch,
                      &S->depth_in, &S->list, &S->lcnt};
    for (DevBuf *b : bufs) b->release();
    delete S;
    e->fs = nullptr;
}
}  // namespace orbamd

extern "C" {

int orbf_rgbd_batch_device(orbx_engine *e, const float *d_depth, size_t depth_stride, int dpitch,
                           const float K[4], const float dist[5], float mbf, void *stream) {
    if (!e || !d_depth || !K || !dist) return ORBX_EINVAL;
    if (e->last_n < 1) return ORBX_ESTATE;
    orbf_state &S = fstate(e);
    const int cap = e->g.out_base[e->g.nlevels], n = e->last_n;
    if (S.kun.ensure(sizeof(orbx_kp) * (size_t)n * cap) || S.uR.ensure(4 * (size_t)n * cap) || S.dep.ensure(4 * (size_t)n * cap))
        return ORBX_EDEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const Camera cam = make_camera(K, dist, mbf);
    FR_CHK(order_after_done(e, s));
    int ph = prof_begin(e, s);
    rgbd_kernel<<<dim3((cap + 255) / 256, n), 256, 0, s>>>(cam, e->d_kps.as<orbx_kp>(), e->d_cnt.as<int>(), cap, d_depth,
                                                           (long long)depth_stride, dpitch, S.kun.as<orbx_kp>(),
                                                           S.uR.as<float>(), S.dep.as<float>());
    prof_end(e, s, ph, "rgbd_kernel");
    FR_CHK(hipGetLastError());
    FR_CHK(mark_done(e, s));
    S.kun_gen = e->gen;
    S.kun_n = n;
    S.kun_cap = cap;
    S.si_pairs = 0;
    return ORBX_OK;
}

int orbf_rgbd(orbx_engine *e, const float *depth, int dpitch, const float K[4], const float dist[5], float mbf,
              orbx_kp *keys_un, float *u_right, float *depth_out, int n) {
    if (!e || !depth || n < 0) return ORBX_EINVAL;
    if (e->last_n < 1) return ORBX_ESTATE;
    if (dpitch < e->W) return ORBX_EINVAL;
    orbf_state &S = fstate(e);
    if (S.depth_in.ensure(sizeof(float) * (size_t)dpitch * e->H)) return ORBX_EDEVICE;
    // the previous launch on this stream may still read depth_in: stream order covers it
    FR_CHK(hipStreamWaitEvent(e->stream, e->done, 0));
    FR_CHK(hipMemcpyAsync(S.depth_in.p, depth, sizeof(float) * (size_t)dpitch * e->H, hipMemcpyHostToDevice, e->stream));
    int rc = orbf_rgbd_batch_device(e, S.depth_in.as<float>(), 0, dpitch, K, dist, mbf, e->stream);
    if (rc) return rc;
    int cnt = 0;
    {
        HostCopy hc(e->stream, nullptr);
        hc.d2h(&cnt, e->d_cnt.p, sizeof(int));
        if (hc.finish()) return ORBX_EDEVICE;
    }
    if (cnt != n) return ORBX_EINVAL;
    if (n > 0) {
        HostCopy hc(e->stream, nullptr);
        hc.d2h(keys_un, S.kun.p, sizeof(orbx_kp) * n);
        hc.d2h(u_right, S.uR.p, 4 * (size_t)n);
        hc.d2h(depth_out, S.dep.p, 4 * (size_t)n);
        if (hc.finish()) return ORBX_EDEVICE;
    }
    return ORBX_OK;
}

int orbm_search_init_batch_device(orbx_engine *e, int n_pairs, int f1_base, int f1_step, int f2_base, int f2_step,
                                  const float K[4], const float dist[5], int window, float nnratio, int check_ori,
                                  void *stream) {
    if (!e || n_pairs <= 0 || !K || !dist) return ORBX_EINVAL;
    orbf_state &S = fstate(e);
    const int n = e->last_n, cap = e->g.out_base[e->g.nlevels];
    // needs the undistorted keypoints (orbf_rgbd*) of the engine's current extraction
    if (!S.kun.p || S.kun_gen != e->gen || S.kun_n != n || S.kun_cap != cap) return ORBX_ESTATE;
    if (f1_base < 0 || f2_base < 0 || f1_step < 0 || f2_step < 0 ||
        f1_base + f1_step * (n_pairs - 1) >= n || f2_base + f2_step * (n_pairs - 1) >= n) return ORBX_EINVAL;
    int sort_cap = 1;
    while (sort_cap < cap) sort_cap <<= 1;
    if (cap > 4096 || sort_cap > 4096 || cap > 32767) return ORBX_EINVAL;
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const Camera cam = make_camera(K, dist, 0.f);
    FR_CHK(order_after_done(e, s));
    const GridParams gp = make_grid(cam, e->W, e->H);
    if (S.keys.ensure(4 * (size_t)n * sort_cap) || S.nkeys.ensure(4 * (size_t)n) ||
        S.cstart.ensure(4 * (size_t)n * (GRID_CELLS + 1)) ||
        S.prev.ensure(8 * (size_t)n_pairs * cap) || S.m12.ensure(4 * (size_t)n_pairs * cap) ||
        S.nmatch.ensure(4 * (size_t)n_pairs))
        return ORBX_EDEVICE;
    int ph = prof_begin(e, s);
    grid_sort_kernel<<<n, 256, 4 * sort_cap, s>>>(gp, S.kun.as<orbx_kp>(), e->d_cnt.as<int>(), cap, sort_cap,
                                                  S.keys.as<uint32_t>(), S.nkeys.as<int>(), S.cstart.as<int>());
    prof_end(e, s, ph, "grid_sort_kernel");
    init_prev_xy<<<dim3((cap + 255) / 256, n_pairs), 256, 0, s>>>(S.kun.as<orbx_kp>(), e->d_cnt.as<int>(), cap, f1_base,
                                                                  f1_step, S.prev.as<float>());
    const int cap0 = e->g.out_cap[0];
    if (S.list.ensure(4 * (size_t)n_pairs * cap0 * cap0) || S.lcnt.ensure(4 * (size_t)n_pairs * cap0)) return ORBX_EDEVICE;
    SearchArgs a;
    a.f1_base = f1_base; a.f1_step = f1_step; a.f2_base = f2_base; a.f2_step = f2_step;
    a.kun = S.kun.as<orbx_kp>();
    a.desc = e->d_desc.as<uint8_t>();
    a.cnt = e->d_cnt.as<int>();
    a.cap = cap;
    a.sort_cap = sort_cap;
    a.cap0 = cap0;
    a.keys = S.keys.as<uint32_t>();
    a.nkeys = S.nkeys.as<int>();
    a.cstart = S.cstart.as<int>();
    a.gp = gp;
    a.r = (float)window;
    a.nnratio = nnratio;
    a.check_ori = check_ori;
    a.list = S.list.as<uint32_t>();
    a.lcnt = S.lcnt.as<int>();
    // phase B LDS: stage + prefix + vMD/v21/M12 (u16) + bins (i8); stage gets the rest of kSearchLds
    const size_t fixed = 4 * ((size_t)cap0 + 1) + 7 * (size_t)cap + 16;
    a.stage_cap = (int)std::min<size_t>(16384, (kSearchLds - fixed) / 4);
    if (a.stage_cap < cap0) return ORBX_EINVAL;
    const size_t lds = 4 * (size_t)a.stage_cap + fixed;
    ph = prof_begin(e, s);
    search_init_cand_kernel<<<dim3((cap0 + 3) / 4, n_pairs), 256, 0, s>>>(a, S.prev.as<float>());
    search_init_resolve_kernel<<<n_pairs, 256, lds, s>>>(a, S.prev.as<float>(), S.m12.as<int>(), S.nmatch.as<int>());
    prof_end(e, s, ph, "search_init_cand+resolve_kernel", 2);
    FR_CHK(hipGetLastError());
    FR_CHK(mark_done(e, s));
    S.si_pairs = n_pairs;
    return ORBX_OK;
}

int orbm_search_init_fetch(orbx_engine *e, int pair, int *matches12, float *prev_xy, int cap, int *nmatches) {
    if (!e) return ORBX_EINVAL;
    orbf_state &S = fstate(e);
    if (!S.m12.p || S.si_pairs == 0 || S.kun_gen != e->gen) return ORBX_ESTATE;
    if (pair < 0 || pair >= S.si_pairs) return ORBX_EINVAL;
    const int kc = e->g.out_base[e->g.nlevels];
    if (cap < kc) return ORBX_ECAP;
    FR_CHK(hipSetDevice(e->device));
    HostCopy hc(e->stream, e->done);
    hc.d2h(matches12, S.m12.as<int>() + (size_t)pair * kc, 4 * (size_t)kc);
    hc.d2h(prev_xy, S.prev.as<float>() + (size_t)pair * kc * 2, 8 * (size_t)kc);
    hc.d2h(nmatches, S.nmatch.as<int>() + pair, 4);
    return hc.finish();
}

int orbf_rgbd_fetch(orbx_engine *e, int image, orbx_kp *keys_un, float *u_right, float *depth_out, int cap) {
    if (!e) return ORBX_EINVAL;
    orbf_state &S = fstate(e);
    if (!S.kun.p || S.kun_gen != e->gen) return ORBX_ESTATE;
    if (image < 0 || image >= S.kun_n) return ORBX_EINVAL;
    const int kc = e->g.out_base[e->g.nlevels];
    if (cap < kc) return ORBX_ECAP;
    FR_CHK(hipSetDevice(e->device));
    HostCopy hc(e->stream, e->done);
    hc.d2h(keys_un, S.kun.as<orbx_kp>() + (size_t)image * kc, sizeof(orbx_kp) * kc);
    hc.d2h(u_right, S.uR.as<float>() + (size_t)image * kc, 4 * (size_t)kc);
    hc.d2h(depth_out, S.dep.as<float>() + (size_t)image * kc, 4 * (size_t)kc);
    return hc.finish();
}

// ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) on two
// host Frames (ORBmatcher.h:169, ORBmatcher.cc:580-748), as Tracking::MonocularInitialization
// calls it frame after frame against a fixed initial frame (Tracking.cc:893-897, 929-933):
// vbPrevMatched is the window centre per F1 keypoint on input (:627) and is rewritten with the
// matched F2 positions on output (:742-745), so consecutive calls chain exactly as in the
// reference. Same two-phase kernels as the batched form, F1 / F2 = images 0 / 1 of the matcher's
// buffers.
int orbm_search_for_initialization(orbm_matcher *m, const orbm_frame *F1, const orbm_frame *F2, float *prev_matched,
                                   int32_t *matches12, int window, int32_t *nmatches) {
    if (!m || !F1 || !F2 || !nmatches) return ORBX_EINVAL;
    *nmatches = 0;
    if (F1->n < 0 || F2->n < 0) return ORBX_EINVAL;
    if (F1->n == 0) return ORBX_OK;   // vnMatches12 = vector<int>(0)
    if (!prev_matched || !matches12 || !F1->keys_un || !F1->desc) return ORBX_EINVAL;
    if (F2->n > 0 && (!F2->keys_un || !F2->desc)) return ORBX_EINVAL;
    if (!(F2->max_x > F2->min_x) || !(F2->max_y > F2->min_y) || window < 0) return ORBX_EINVAL;
    const int cap = std::max(std::max(F1->n, F2->n), 1);
    int sort_cap = 1;
    while (sort_cap < cap) sort_cap <<= 1;
    if (sort_cap > 4096) return ORBX_EINVAL;   // one workgroup's LDS sort of F2's grid keys
    const int cap0 = cap;                     // every F1 keypoint may be of octave 0
    const size_t fixed = 4 * ((size_t)cap0 + 1) + 7 * (size_t)cap + 16;
    if (fixed >= kSearchLds) return ORBX_EINVAL;
    SearchArgs a;
    a.stage_cap = (int)std::min<size_t>(16384, (kSearchLds - fixed) / 4);
    if (a.stage_cap < cap0) return ORBX_EINVAL;
    FR_CHK(hipSetDevice(m->device));
    const hipStream_t s = m->stream;
    FR_CHK(order_after_done(m, s));
    FR_CHK(hipStreamWaitEvent(s, m->done, 0));
    if (m->kun.ensure(sizeof(orbx_kp) * 2 * (size_t)cap) || m->desc.ensure(64 * (size_t)cap) || m->cnt.ensure(8) ||
        m->keys.ensure(8 * (size_t)sort_cap) || m->nkeys.ensure(8) || m->cstart.ensure(8 * (size_t)(GRID_CELLS + 1)) ||
        m->prev.ensure(8 * (size_t)cap) ||
        m->m12.ensure(4 * (size_t)cap) || m->nmatch.ensure(4) || m->list.ensure(4 * (size_t)cap0 * cap0) ||
        m->lcnt.ensure(4 * (size_t)cap0))
        return ORBX_EDEVICE;
    const int counts[2] = {F1->n, F2->n};
    HostCopy up(s, nullptr);
    up.h2d(m->kun.p, F1->keys_un, sizeof(orbx_kp) * (size_t)F1->n);
    up.h2d((char *)m->kun.p + sizeof(orbx_kp) * (size_t)cap, F2->keys_un, sizeof(orbx_kp) * (size_t)F2->n);
    up.h2d(m->desc.p, F1->desc, 32 * (size_t)F1->n);
    up.h2d((char *)m->desc.p + 32 * (size_t)cap, F2->desc, 32 * (size_t)F2->n);
    up.h2d(m->cnt.p, counts, sizeof counts);
    up.h2d(m->prev.p, prev_matched, 8 * (size_t)F1->n);
    if (up.finish()) return ORBX_EDEVICE;   // host arrays (counts) go out of scope
    GridParams gp;
    gp.minX = F2->min_x; gp.maxX = F2->max_x; gp.minY = F2->min_y; gp.maxY = F2->max_y;
    gp.invW = (float)GRID_COLS / (gp.maxX - gp.minX);   // Frame.cc:183-184
    gp.invH = (float)GRID_ROWS / (gp.maxY - gp.minY);
    a.f1_base = 0; a.f1_step = 0; a.f2_base = 1; a.f2_step = 0;
    a.kun = m->kun.as<orbx_kp>();
    a.desc = m->desc.as<uint8_t>();
    a.cnt = m->cnt.as<int>();
    a.cap = cap;
    a.sort_cap = sort_cap;
    a.cap0 = cap0;
    a.keys = m->keys.as<uint32_t>();
    a.nkeys = m->nkeys.as<int>();
    a.cstart = m->cstart.as<int>();
    a.gp = gp;
    a.r = (float)window;
    a.nnratio = m->nnratio;
    a.check_ori = m->check_ori;
    a.list = m->list.as<uint32_t>();
    a.lcnt = m->lcnt.as<int>();
    grid_sort_kernel<<<2, 256, 4 * sort_cap, s>>>(gp, a.kun, a.cnt, cap, sort_cap, m->keys.as<uint32_t>(), m->nkeys.as<int>(),
                                                  m->cstart.as<int>());
    search_init_cand_kernel<<<dim3((cap0 + 3) / 4, 1), 256, 0, s>>>(a, m->prev.as<float>());
    search_init_resolve_kernel<<<1, 256, 4 * (size_t)a.stage_cap + fixed, s>>>(a, m->prev.as<float>(), m->m12.as<int>(),
                                                                              m->nmatch.as<int>());
    FR_CHK(hipGetLastError());
    FR_CHK(mark_done(m, s));
    HostCopy dn(s, nullptr);
    dn.d2h(matches12, m->m12.p, 4 * (size_t)F1->n);
    dn.d2h(prev_matched, m->prev.p, 8 * (size_t)F1->n);
    dn.d2h(nmatches, m->nmatch.p, 4);
    return dn.finish();
}

}  // extern "C"
