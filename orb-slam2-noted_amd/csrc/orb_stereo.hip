// MI355X-native Frame::ComputeStereoMatches (Frame.cc:831-1128) and the ORBmatcher
// Hamming core (ORBmatcher.cc:2123-2143).
//
// Three kernels per batch of stereo pairs:
//   S1 stereo_sort_right  one workgroup per pair: right keypoints sorted by y (counting sort)
//                         -> replaces the vRowIndices row buckets (:858-888); a second
//                         workgroup per pair buckets the left keypoints by row
//   S2 stereo_match_staged  one workgroup per 32 left keypoints of nearby rows: the union of
//                         their row bands (sorted right records + right descriptors) staged in
//                         LDS once, then per keypoint on one wavefront: 64-wide popcount Hamming
//                         + (dist, index) min-reduce (= first minimum in right-index order,
//                         :912-978), the 11x11 SAD over incR in [-5, 5] (:981-1063), parabola
//                         fit and depth
//   S3 stereo_median_cut  one workgroup per pair: median of the SAD distances and the
//                         1.5*1.4*median rejection (:1112-1127)
#include <hip/hip_runtime.h>

#include <cstring>

#include <algorithm>
#include <climits>
#include <cstdio>

#include "orb_device.h"
#include "orb_engine.h"

using namespace orbamd;

namespace orbamd {

#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

// One side (left or right) of a batch of stereo pairs: where image p's keypoints,
// descriptors, counts and pyramid live.
struct StereoSide {
    const orbx_kp *kps;
    const uint8_t *desc;
    const int *cnt;
    const uint8_t *in;       // level 0
    const uint8_t *pyr;      // levels >= 1
    long long in_stride;
    int in_pitch;
    int img_base, img_step;  // image index of pair p = img_base + img_step * p
};

struct StereoArgs {
    StereoSide L, R;
    int cap;                 // keypoint slots per image
    int sort_cap;            // pow2 >= cap
    float mbf, mb;
    float rmax;              // 2 * max scale factor (row-band half-width bound)
    int nrows;               // row table entries per pair (image height + 2)
    int *rowtab;             // [pair][nrows]: first sorted right keypoint with y >= row
    float maxD;              // mbf / minZ (Frame.cc:897-899), divided once on the host
};

__device__ __forceinline__ const uint8_t *side_level(const ExtractGeom &g, const StereoSide &s, int img,
                                                     int l, int *pitch) {
    if (l == 0) { *pitch = s.in_pitch; return s.in + (long long)img * s.in_stride; }
    *pitch = g.bp[l];
    return s.pyr + (long long)img * g.pyr_stride + g.pyr_off[l];
}


// ---- S1: right keypoints of each pair in (y, index) order, as 16-byte records
// The scan of S2 reads one 16-byte record per right keypoint in y order: {y, x (float bits),
// minr | maxr << 16 (the row band of Frame.cc:869-888, int16 each), iR | octave << 16}, so the
// band / octave / disparity filter needs no dependent gather of the keypoint itself.
// Counting sort on the image row floor(y) (y >= 0): row histogram, block scan -- whose exclusive
// prefix IS the row table of S2 (first record with y >= r) -- scatter into row buckets, then each
// keypoint's final slot = bucket start + its rank among the bucket's few members by (y, index).
// Replaces a 4096-key bitonic sort in LDS (86 -> ~10 us for one pair: the single-frame latency).
#define ST_THREADS 512
// Workgroups n_pairs .. 2 n_pairs - 1 bucket the LEFT keypoints of pair
// blockIdx.x - n_pairs by image row into lidx (any order inside a row: S2 writes each result to
// the keypoint's own slot, so the order only groups keypoints of nearby rows into workgroups).
__global__ __launch_bounds__(ST_THREADS) void stereo_sort_right(ExtractGeom g, StereoArgs a, uint4 *sorted,
                                                                int n_pairs, int *lidx) {
    extern __shared__ int st_lds[];
    int *cnt = st_lds;                       // [nrows] bucket sizes, then fill counters
    int *start = cnt + a.nrows;              // [nrows] exclusive prefix = row table
    int *mem = start + a.nrows;              // [cap] bucket members (keypoint index)
    float *yk = (float *)(mem + a.cap);      // [cap] y of keypoint i
    __shared__ int wsum[ST_THREADS / 64];
    const bool left = (int)blockIdx.x >= n_pairs;
    const int p = left ? blockIdx.x - n_pairs : blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    const StereoSide &sd = left ? a.L : a.R;
    const int imgR = sd.img_base + sd.img_step * p;
    const int nR = min(sd.cnt[imgR], a.cap);
    const orbx_kp *kR = sd.kps + (long long)imgR * a.cap;
    const int nrows = a.nrows;
    for (int r = tid; r < nrows; r += ST_THREADS) cnt[r] = 0;
    __syncthreads();
    for (int i = tid; i < nR; i += ST_THREADS) {
        const float y = kR[i].y;
        yk[i] = y;
        atomicAdd(&cnt[min(max((int)y, 0), nrows - 1)], 1);
    }
    __syncthreads();
    // block exclusive scan of cnt: thread t owns rows [t*per, (t+1)*per)
    const int per = (nrows + ST_THREADS - 1) / ST_THREADS;
    const int r0 = tid * per, r1 = min(r0 + per, nrows);
    int local = 0;
    for (int r = r0; r < r1; r++) local += cnt[r];
    int incl = local;
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int run = incl - local;
    for (int w = 0; w < wv; w++) run += wsum[w];
    for (int r = r0; r < r1; r++) {
        const int c = cnt[r];
        start[r] = run;
        if (!left) a.rowtab[(long long)p * nrows + r] = run;
        run += c;
    }
    __syncthreads();
    for (int r = tid; r < nrows; r += ST_THREADS) cnt[r] = 0;
    __syncthreads();
    if (left) {
        for (int i = tid; i < nR; i += ST_THREADS) {
            const int b = min(max((int)yk[i], 0), nrows - 1);
            lidx[(long long)p * a.sort_cap + start[b] + atomicAdd(&cnt[b], 1)] = i;
        }
        return;
    }
    for (int i = tid; i < nR; i += ST_THREADS) {
        const int b = min(max((int)yk[i], 0), nrows - 1);
        mem[start[b] + atomicAdd(&cnt[b], 1)] = i;
    }
    __syncthreads();
    for (int i = tid; i < nR; i += ST_THREADS) {
        const float y = yk[i];
        const int b = min(max((int)y, 0), nrows - 1), s0 = start[b], nb = cnt[b];
        int rank = 0;
        for (int q = 0; q < nb; q++) {
            const int j = mem[s0 + q];
            const float yj = yk[j];
            rank += (yj < y) || (yj == y && j < i);
        }
        const orbx_kp kp = kR[i];
        const float r = 2.0f * g.scale[kp.octave];
        const int maxr = (int)ceilf(kp.y + r), minr = (int)floorf(kp.y - r);
        sorted[(long long)p * a.sort_cap + s0 + rank] =
            make_uint4(__float_as_uint(kp.y), __float_as_uint(kp.x), (uint32_t)(minr & 0xFFFF) | (uint32_t)maxr << 16,
                       (uint32_t)i | (uint32_t)kp.octave << 16);
    }
}

// SAD refinement of one left keypoint given its best Hamming candidate (Frame.cc:979-1063), on one
// wavefront: 11x11 window SAD over incR in [-5, 5], parabola fit, disparity and depth; lane 0
// writes slot o (uR, depth, SAD distance or -1 each). The caller passes the level-dependent
// values (level images and pitches, width, scale, inverse scale of the keypoint's octave) as
// scalars: indexing the geometry structs by reference here made the compiler copy them to scratch.
__device__ __forceinline__ void stereo_refine(const orbx_kp &kpL, bool matched, float uR0, const uint8_t *imL,
                                              int pitchL, const uint8_t *imR, int pitchR, int lw, float scale,
                                              float sf, float mbf, float maxD, int lane, long long o,
                                              float *u_right, float *depth, int *sad) {
    float outU = -1.0f, outD = -1.0f;
    int outS = -1;
    const float uL = kpL.x;
    const float minD = 0;
    bool ok = matched;
    float scaleduR0 = 0, scaledvL = 0, scaleduL = 0;
    if (ok) {
        scaleduL = roundf(kpL.x * sf);   // sf = mvInvScaleFactors[octave] (ORBextractor.cc:503)
        scaledvL = roundf(kpL.y * sf);
        scaleduR0 = roundf(uR0 * sf);
        const float iniu = scaleduR0 - 5 - 5, endu = scaleduR0 + 5 + 5 + 1;
        if (iniu < 0 || endu >= lw) ok = false;
    }
    if (ok) {
        // SAD of (IL - IL(w, w)) and (IR - IR(w, w + incR)) over the 11 x 11 window (:989-1011):
        // |(L + cr) - (R + cl)| per pixel, on packed u16 pairs with v_sad_u16 (a = L + cr - cl + 256,
        // b = R + 256, both in [0, 766]). Lane 16 s + rr, pass p: window row rr (< 11), incR =
        // 4 p + s - 5 (<= 5); the 16 lanes of a DPP row sum their rows, lane 15 holds incR's total.
        const int r0 = (int)scaledvL - 5, cL0 = (int)scaleduL - 5, cR = (int)scaleduR0;
        const int rr = lane & 15, sgrp = lane >> 4, rrc = min(rr, 10);
        uint32_t LD[3];
        __builtin_memcpy(LD, imL + (long long)(r0 + rrc) * pitchL + cL0, 12);   // 11 pixels + 1 (in the level)
        // the lane's right-window bytes of all three passes in one 20-byte load: pass p reads cols
        // cR + 4 p + s - 10 .. + 11, i.e. dwords p .. p + 2 of the block at cR + s - 10 (its last
        // bytes reach at most one column past the reference's window, still inside the level's
        // row storage: the window's rows end >= 14 rows above the level's last). The centre
        // pixels IL(w, w) and IR(w, w + incR) are bytes of window row 5: taken from lane 16 s + 5
        // by ds_bpermute instead of four more byte loads.
        uint32_t WR[5];
        __builtin_memcpy(WR, imR + (long long)(r0 + rrc) * pitchR + cR - 10 + sgrp, 20);
        const int c5 = ((lane & ~15) | 5) << 2;
        const int cl = (int)((__builtin_amdgcn_ds_bpermute(c5, (int)LD[1]) >> 8) & 0xFF);   // col cL0 + 5
        const uint32_t Lp[6] = {__builtin_amdgcn_perm(0u, LD[0], 0x0c010c00u), __builtin_amdgcn_perm(0u, LD[0], 0x0c030c02u),
                                __builtin_amdgcn_perm(0u, LD[1], 0x0c010c00u), __builtin_amdgcn_perm(0u, LD[1], 0x0c030c02u),
                                __builtin_amdgcn_perm(0u, LD[2], 0x0c010c00u), __builtin_amdgcn_perm(0u, LD[2], 0x0c0c0c02u)};
        const uint32_t ONES = 0x01010101u;
        int sums[12];
#pragma unroll
        for (int pss = 0; pss < 3; pss++) {
            const int inc = 4 * pss + sgrp - 5;
            const uint32_t RD[3] = {WR[pss], WR[pss + 1], WR[pss + 2]};
            const int kc = (int)((__builtin_amdgcn_ds_bpermute(c5, (int)WR[pss + 1]) >> 8) & 0xFF);   // col cR + inc
            const uint32_t KA = (uint32_t)(kc - cl + 256), KA2 = KA * 0x10001u;
            uint32_t acc = __builtin_amdgcn_sad_u16(Lp[0] + KA2, __builtin_amdgcn_perm(ONES, RD[0], 0x04010400u), 0u);
            acc = __builtin_amdgcn_sad_u16(Lp[1] + KA2, __builtin_amdgcn_perm(ONES, RD[0], 0x04030402u), acc);
            acc = __builtin_amdgcn_sad_u16(Lp[2] + KA2, __builtin_amdgcn_perm(ONES, RD[1], 0x04010400u), acc);
            acc = __builtin_amdgcn_sad_u16(Lp[3] + KA2, __builtin_amdgcn_perm(ONES, RD[1], 0x04030402u), acc);
            acc = __builtin_amdgcn_sad_u16(Lp[4] + KA2, __builtin_amdgcn_perm(ONES, RD[2], 0x04010400u), acc);
            acc = __builtin_amdgcn_sad_u16(Lp[5] + KA, __builtin_amdgcn_perm(ONES, RD[2], 0x0c0c0402u), acc);
            int v = (rr < 11 && inc <= 5) ? (int)acc : 0;
            v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
            v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
            v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
            v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
#pragma unroll
            for (int k = 0; k < 4; k++) sums[4 * pss + k] = __builtin_amdgcn_readlane(v, 16 * k + 15);
        }
        // wave-uniform tail (:1013-1063): first minimum over incR, parabola, disparity
        int bestS = INT_MAX, bestinc = 0;
#pragma unroll
        for (int inc = -5; inc <= 5; inc++)
            if (sums[inc + 5] < bestS) { bestS = sums[inc + 5]; bestinc = inc; }
        if (bestinc != -5 && bestinc != 5) {
            const float d1 = (float)sums[5 + bestinc - 1], d2 = (float)sums[5 + bestinc], d3 = (float)sums[5 + bestinc + 1];
            const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
            if (!(deltaR < -1 || deltaR > 1)) {
                float bestuR = scale * ((float)scaleduR0 + (float)bestinc + deltaR);
                float disparity = uL - bestuR;
                if (disparity >= minD && disparity < maxD) {
                    if (disparity <= 0) {
                        disparity = (float)0.01;
                        bestuR = (float)((double)uL - 0.01);
                    }
                    outD = mbf / disparity;
                    outU = bestuR;
                    outS = bestS;
                }
            }
        }
    }
    if (lane == 0) {
        u_right[o] = outU;
        depth[o] = outD;
        sad[o] = outS;
    }
}

// ---- S2: one workgroup per ST_NK left keypoints of nearby rows
// (S1's row buckets), whose candidate bands overlap: the union of their bands -- the sorted right
// records and the right descriptors they index -- is staged in LDS once (one global round trip
// per workgroup instead of a record and a descriptor load per keypoint), then each wavefront scans
// ORBX_ST_KPW keypoints from LDS (201 -> 177 us per 128 pairs alone against one keypoint per wavefront
// reading global memory; 1, 2, 4 or 16 keypoints per wavefront measured slower). The
// candidate set is band [first record with y >= floor(row - rmax - 2), first with
// y >= floor(row + rmax + 2) + 1) with the reference's per-record test (:912-978); a union wider than
// ST_SCAP records scans global memory instead.
#define ORBX_ST_KPW 8
#define ST_NW 4
#define ST_NK (ST_NW * ORBX_ST_KPW)
#define ST_SCAP 256

__device__ __forceinline__ int hamming_v(const uint4 &x0, const uint4 &x1, const uint4 &y0, const uint4 &y1) {
    return __popc(x0.x ^ y0.x) + __popc(x0.y ^ y0.y) + __popc(x0.z ^ y0.z) + __popc(x0.w ^ y0.w) +
           __popc(x1.x ^ y1.x) + __popc(x1.y ^ y1.y) + __popc(x1.z ^ y1.z) + __popc(x1.w ^ y1.w);
}

__global__ __launch_bounds__(ST_NW * 64) void stereo_match_staged(ExtractGeom g, StereoArgs a, const uint4 *sorted,
                                                                  const int *lidx, float *u_right, float *depth,
                                                                  int *sad) {
    __shared__ uint4 s_rec[ST_SCAP], s_d0[ST_SCAP], s_d1[ST_SCAP];
    __shared__ int s_kp[ST_NK][3];   // left keypoint index (-1: none), band [lo, hi)
    // each slot's left keypoint (x, y, octave) and descriptor, loaded once by the prologue with its
    // row: the wavefront's keypoint loop then starts each keypoint without a global round trip
    __shared__ float s_kx[ST_NK], s_ky[ST_NK];
    __shared__ int s_ko[ST_NK];
    __shared__ uint4 s_q[ST_NK][2];
    __shared__ int s_lo, s_hi;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    int bxr, p;
    xcd_remap2(bxr, p);
    const int imgL = a.L.img_base + a.L.img_step * p, imgR = a.R.img_base + a.R.img_step * p;
    const int s0 = bxr * ST_NK;
    // the slot's lidx entry goes out with the keypoint counts (inside the pair's sort_cap row; used
    // only below nL)
    const int iLs = tid < ST_NK && s0 + tid < a.sort_cap ? lidx[(long long)p * a.sort_cap + s0 + tid] : -1;
    const int nL = min(a.L.cnt[imgL], a.cap), nR = min(a.R.cnt[imgR], a.cap);
    if (s0 >= nL) return;   // workgroup-uniform, before any barrier
    const orbx_kp *kL = a.L.kps + (long long)imgL * a.cap;
    const orbx_kp *kR = a.R.kps + (long long)imgR * a.cap;
    const uint4 *srt = sorted + (long long)p * a.sort_cap;
    const int *rowtab = a.rowtab + (long long)p * a.nrows;
    if (tid == 0) { s_lo = INT_MAX; s_hi = INT_MIN; }
    __syncthreads();
    if (tid < ST_NK) {
        int iL = -1, lo = 0, hi = 0;
        if (s0 + tid < nL) {
            iL = iLs;
            const orbx_kp k = kL[iL];
            const uint4 *dq = (const uint4 *)(a.L.desc + ((long long)imgL * a.cap + iL) * 32);
            s_q[tid][0] = dq[0];
            s_q[tid][1] = dq[1];
            s_kx[tid] = k.x;
            s_ky[tid] = k.y;
            s_ko[tid] = k.octave;
            const int row = (int)k.y;
            const float ylo = (float)row - a.rmax - 2.0f, yhi = (float)row + a.rmax + 2.0f;
            lo = rowtab[min(max((int)floorf(ylo), 0), a.nrows - 1)];
            const int hr = (int)floorf(yhi) + 1;
            hi = hr >= a.nrows ? nR : min(rowtab[max(hr, 0)], nR);
            lo = min(lo, hi);
            atomicMin(&s_lo, lo);
            atomicMax(&s_hi, hi);
        }
        s_kp[tid][0] = iL;
        s_kp[tid][1] = lo;
        s_kp[tid][2] = hi;
    }
    __syncthreads();
    const int ulo = s_lo, un = s_hi - s_lo;
    const bool staged = un <= ST_SCAP;   // workgroup-uniform
    if (staged) {
        const uint4 *dR4 = (const uint4 *)(a.R.desc + (long long)imgR * a.cap * 32);
        for (int j = tid; j < un; j += ST_NW * 64) {
            const uint4 r = srt[ulo + j];
            const int i = (int)(r.w & 0xFFFFu);
            s_rec[j] = r;
            s_d0[j] = dR4[2 * i];
            s_d1[j] = dR4[2 * i + 1];
        }
    }
    __syncthreads();
    const uint8_t *dRg = a.R.desc + (long long)imgR * a.cap * 32;
    for (int k = 0; k < ORBX_ST_KPW; k++) {
        const int slot = wv * ORBX_ST_KPW + k;
        const int iL = __builtin_amdgcn_readfirstlane(s_kp[slot][0]);
        if (iL < 0) break;   // the workgroup's last slots past nL
        const int lo = __builtin_amdgcn_readfirstlane(s_kp[slot][1]), hi = __builtin_amdgcn_readfirstlane(s_kp[slot][2]);
        orbx_kp kpL;   // x, y, octave: what the match and stereo_refine read
        kpL.x = s_kx[slot];
        kpL.y = s_ky[slot];
        kpL.octave = __builtin_amdgcn_readfirstlane(s_ko[slot]);
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const float minD = 0, maxD = a.maxD;
        const float minU = uL - maxD, maxU = uL - minD;
        const int row = (int)vL;
        const float yhi = (float)row + a.rmax + 2.0f;
        int bestDist = 100;  // ORBmatcher::TH_HIGH
        int bestIdxR = 0;
        float bestX = 0.0f;   // the best right keypoint's x (staged: from its LDS record)
        bool haveX = false;
        if (maxU >= 0) {
            const uint4 *dL4 = (const uint4 *)(a.L.desc + ((long long)imgL * a.cap + iL) * 32);   // (the global path)
            const uint4 q0 = s_q[slot][0], q1 = s_q[slot][1];
            unsigned best = 0xFFFFFFFFu;
            // the per-record test as one branch-free predicate (bitwise: no short-circuit branches)
            auto take = [&](const uint4 &e) {
                const float ky = __uint_as_float(e.x);
                const int oct = (int)(e.w >> 16);
                const float kx = __uint_as_float(e.y);
                const int minr = (int)(int16_t)(e.z & 0xFFFFu), maxr = (int)(int16_t)(e.z >> 16);
                return (ky <= yhi) & (row >= minr) & (row <= maxr) & ((unsigned)(oct - levelL + 1) <= 2u) & (kx >= minU) &
                       (kx <= maxU);
            };
            const uint4 NONE = make_uint4(0x7f800000u, 0u, 0u, 0u);
            int jb = 0;   // staged: the LDS slot of the lane's best record
            if (staged) {
                // LDS slots past the band are read anyway (clamped into the array) and masked
                const int end = hi - ulo;
                for (int base = lo - ulo; base < end; base += 128) {
                    const int c0 = base + lane, c1 = c0 + 64;
                    const int j0 = min(c0, ST_SCAP - 1), j1 = min(c1, ST_SCAP - 1);
                    const uint4 e0 = s_rec[j0], e1 = s_rec[j1];
                    const bool t0 = (c0 < end) & take(e0), t1 = (c1 < end) & take(e1);
                    if (t0) {
                        const unsigned k0 = ((unsigned)hamming_v(q0, q1, s_d0[j0], s_d1[j0]) << 16) | (e0.w & 0xFFFFu);
                        if (k0 < best) { best = k0; jb = j0; }
                    }
                    if (t1) {
                        const unsigned k1 = ((unsigned)hamming_v(q0, q1, s_d0[j1], s_d1[j1]) << 16) | (e1.w & 0xFFFFu);
                        if (k1 < best) { best = k1; jb = j1; }
                    }
                }
            } else {
                for (int base = lo; base < hi; base += 128) {
                    const int c0 = base + lane, c1 = c0 + 64;
                    const uint4 e0 = c0 < hi ? srt[c0] : NONE, e1 = c1 < hi ? srt[c1] : NONE;
                    const bool t0 = take(e0), t1 = take(e1);
                    const int i0 = (int)(e0.w & 0xFFFFu), i1 = (int)(e1.w & 0xFFFFu);
                    if (t0) best = min(best, ((unsigned)hamming32((const uint8_t *)dL4, dRg + (long long)i0 * 32) << 16) | (unsigned)i0);
                    if (t1) best = min(best, ((unsigned)hamming32((const uint8_t *)dL4, dRg + (long long)i1 * 32) << 16) | (unsigned)i1);
                }
            }
            const unsigned mine = best;   // the lane's own minimum (keys are unique: one record each)
            best = min(best, (unsigned)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)best, 0x111, 0xF, 0xF, false));
            best = min(best, (unsigned)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)best, 0x112, 0xF, 0xF, false));
            best = min(best, (unsigned)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)best, 0x114, 0xF, 0xF, false));
            best = min(best, (unsigned)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)best, 0x118, 0xF, 0xF, false));
            best = min(min((unsigned)__builtin_amdgcn_readlane((int)best, 15), (unsigned)__builtin_amdgcn_readlane((int)best, 31)),
                       min((unsigned)__builtin_amdgcn_readlane((int)best, 47), (unsigned)__builtin_amdgcn_readlane((int)best, 63)));
            if (best != 0xFFFFFFFFu && (int)(best >> 16) < bestDist) {
                bestDist = (int)(best >> 16);
                bestIdxR = (int)(best & 0xFFFF);
                if (staged) {   // the record holding it: its x instead of a global load of kR[bestIdxR]
                    const unsigned long long own = __ballot(mine == best);
                    const int jw = __builtin_amdgcn_readlane(jb, (int)__builtin_ctzll(own));
                    bestX = __uint_as_float(s_rec[jw].y);
                    haveX = true;
                }
            }
        }
        const bool matched = maxU >= 0 && bestDist < (100 + 50) / 2;   // thOrbDist (Frame.cc:842)
        int pitchL, pitchR;
        const uint8_t *imL = side_level(g, a.L, imgL, levelL, &pitchL), *imR = side_level(g, a.R, imgR, levelL, &pitchR);
        stereo_refine(kpL, matched, matched ? (haveX ? bestX : kR[bestIdxR].x) : 0.0f, imL, pitchL, imR, pitchR, g.lw[levelL],
                      g.scale[levelL], g.inv_scale[levelL], a.mbf, a.maxD, lane, (long long)p * a.cap + iL, u_right, depth,
                      sad);
    }
}

// ---- S3: median of SAD distances and outlier cut (Frame.cc:1112-1127)
// The reference sorts (SAD, iL) pairs and takes element nd/2; only that order statistic is
// needed: a two-pass radix select on the SAD value (< 121 * 510 < 2^16) with LDS histograms of
// its high and low byte. Replaces a 4096-key bitonic sort (74 -> a few us for one pair).
__global__ __launch_bounds__(ST_THREADS) void stereo_median_cut(StereoArgs a, float *u_right, float *depth,
                                                               const int *sad) {
    __shared__ int hist[256];
    __shared__ int nd, sel, rem;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int imgL = a.L.img_base + a.L.img_step * p;
    const int nL = min(a.L.cnt[imgL], a.cap);
    const int *s = sad + (long long)p * a.cap;
    if (tid < 256) hist[tid] = 0;
    if (tid == 0) nd = 0;
    __syncthreads();
    int mine = 0;
    for (int i = tid; i < nL; i += ST_THREADS) {
        const int v = s[i];
        if (v >= 0) { atomicAdd(&hist[min(v >> 8, 255)], 1); mine++; }
    }
    if (mine) atomicAdd(&nd, mine);
    __syncthreads();
    const int n = nd;
    if (n == 0) return;   // no match: nothing to cut (the reference would index an empty vector)
    const int k = n / 2;  // vDistIdx[vDistIdx.size() / 2] of the sorted SADs
    if (tid == 0) {
        int c = 0, b = 0;
        while (c + hist[b] <= k) c += hist[b++];
        sel = b;
        rem = k - c;
    }
    __syncthreads();
    const int hi = sel, r_lo = rem;
    __syncthreads();
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < nL; i += ST_THREADS) {
        const int v = s[i];
        if (v >= 0 && min(v >> 8, 255) == hi) atomicAdd(&hist[v & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int c = 0, b = 0;
        while (c + hist[b] <= r_lo) c += hist[b++];
        sel = (hi << 8) | b;
    }
    __syncthreads();
    const float median = (float)sel;
    const float thDist = 1.5f * 1.4f * median;
    float *u = u_right + (long long)p * a.cap;
    float *d = depth + (long long)p * a.cap;
    for (int i = tid; i < nL; i += ST_THREADS) {
        const int v = s[i];
        if (v >= 0 && !((float)v < thDist)) { u[i] = -1; d[i] = -1; }
    }
}

static int run_stereo(const ExtractGeom &g, StereoArgs &a, int n_pairs, orbx_engine *store,
                      hipStream_t s) {
    int sc = 1;
    while (sc < a.cap) sc <<= 1;
    a.sort_cap = sc;
    float smax = 0;
    for (int l = 0; l < g.nlevels; l++) smax = std::max(smax, g.scale[l]);
    a.rmax = 2.0f * smax;
    // the same IEEE single divisions the reference makes per frame / per extractor
    a.maxD = a.mbf / a.mb;
    const size_t slots = (size_t)n_pairs * a.cap;
    a.nrows = g.H + 2;
    HIPCHK(order_after_done(store, s));
    if (store->d_st_rows.ensure(4 * (size_t)n_pairs * a.nrows)) return ORBX_EDEVICE;
    a.rowtab = store->d_st_rows.as<int>();
    if (store->d_st_sorted.ensure(16 * (size_t)n_pairs * sc) || store->d_st_u.ensure(4 * slots) ||
        store->d_st_depth.ensure(4 * slots) || store->d_st_dist.ensure(4 * slots))
        return ORBX_EDEVICE;
    float *u = store->d_st_u.as<float>(), *d = store->d_st_depth.as<float>();
    int *sad = store->d_st_dist.as<int>();
    const size_t sort_lds = 4 * (2 * (size_t)a.nrows + 2 * (size_t)a.cap);
    if (sort_lds > 64 * 1024) return ORBX_EINVAL;
    int ph = prof_begin(store, s);
    if (store->d_st_res.ensure(4 * (size_t)n_pairs * sc)) return ORBX_EDEVICE;
    int *lidx = store->d_st_res.as<int>();
    stereo_sort_right<<<2 * n_pairs, ST_THREADS, sort_lds, s>>>(g, a, store->d_st_sorted.as<uint4>(), n_pairs, lidx);
    prof_end(store, s, ph, "stereo_sort_right");
    ph = prof_begin(store, s);
    for (int rep = 0; rep < ((exp_twice() & 8) ? 2 : 1); rep++)
        stereo_match_staged<<<dim3((a.cap + ST_NK - 1) / ST_NK, n_pairs), ST_NW * 64, 0, s>>>(
            g, a, store->d_st_sorted.as<uint4>(), lidx, u, d, sad);
    prof_end(store, s, ph, "stereo_match_staged");
    ph = prof_begin(store, s);
    stereo_median_cut<<<n_pairs, ST_THREADS, 0, s>>>(a, u, d, sad);
    prof_end(store, s, ph, "stereo_median_cut");
    HIPCHK(hipGetLastError());
    HIPCHK(mark_done(store, s));
    store->st_pairs = n_pairs;
    return ORBX_OK;
}

static StereoSide side_of(orbx_engine *e, int base, int step) {
    StereoSide s;
    s.kps = e->d_kps.as<orbx_kp>();
    s.desc = e->d_desc.as<uint8_t>();
    s.cnt = e->d_cnt.as<int>();
    s.in = e->last_in;
    s.pyr = e->d_pyr.as<uint8_t>();
    s.in_stride = e->last_stride;
    s.in_pitch = e->last_pitch;
    s.img_base = base;
    s.img_step = step;
    return s;
}

// ---- Hamming best / second best (the scan core every ORBmatcher search shares)
// One wavefront per query. The reference loops over its candidates in order with
//   if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx = idx; }
//   else if (dist < bestDist2) bestDist2 = dist;
// (e.g. ORBmatcher.cc:639-668), i.e. best = the FIRST minimum in candidate order and second =
// the minimum over the remaining candidates. Each lane keeps (dist << 20 | position) over its
// strided subset, then a butterfly merge keeps the lexicographic minimum as best and folds the
// other key into the second distance. CAND: candidates cand_idx[off[i] .. off[i+1]) (list
// order = position order); otherwise the whole database in index order.
template <bool CAND>
__global__ __launch_bounds__(256) void hamming_best2_kernel(const uint8_t *q, int nq, const uint8_t *db, int ndb,
                                                            const int *cand_off, const int *cand_idx, int *best_idx,
                                                            int *best_d, int *second_d) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave_id();
    if (i >= nq) return;
    const uint8_t *qi = q + (long long)i * 32;
    int c0 = 0, n = ndb;
    if (CAND) { c0 = cand_off[i]; n = cand_off[i + 1] - c0; }
    unsigned b1 = 0xFFFFFFFFu;   // (dist << 20) | position
    int d2 = INT_MAX;
    for (int j = lane; j < n; j += 64) {
        const int idx = CAND ? cand_idx[c0 + j] : j;
        const int d = (unsigned)idx < (unsigned)ndb ? hamming32(qi, db + (long long)idx * 32) : 256 + 1;
        if (d > 256) continue;   // out-of-range candidate index: skipped (the host checks them)
        const unsigned key = ((unsigned)d << 20) | (unsigned)j;
        if (key < b1) {
            if (b1 != 0xFFFFFFFFu) d2 = min(d2, (int)(b1 >> 20));
            b1 = key;
        } else {
            d2 = min(d2, d);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned ob1 = (unsigned)__shfl_xor((int)b1, off, 64);
        const int od2 = __shfl_xor(d2, off, 64);
        const unsigned lo = min(b1, ob1), hi = max(b1, ob1);
        int s2 = min(d2, od2);
        if (hi != 0xFFFFFFFFu) s2 = min(s2, (int)(hi >> 20));
        b1 = lo;
        d2 = s2;
    }
    if (lane == 0) {
        const int pos = (int)(b1 & 0xFFFFF);
        best_idx[i] = b1 == 0xFFFFFFFFu ? -1 : (CAND ? cand_idx[c0 + pos] : pos);
        best_d[i] = b1 == 0xFFFFFFFFu ? INT_MAX : (int)(b1 >> 20);
        second_d[i] = d2;
    }
}

}  // namespace orbamd

extern "C" {

int orbm_stereo_match(orbx_engine *left, orbx_engine *right, float mbf, float mb, float *u_right,
                      float *depth, int n) {
    if (!left || !right || n < 0) return ORBX_EINVAL;
    if (left->last_n < 1 || right->last_n < 1) return ORBX_ESTATE;
    if (left->W != right->W || left->H != right->H || left->p.nlevels != right->p.nlevels) return ORBX_EINVAL;
    HIPCHK(hipSetDevice(left->device));
    // the right extractor ran on its own stream / thread (Frame.cc:144-153): order after it
    // and after the left one's last launch, on the left stream only
    HIPCHK(hipStreamWaitEvent(left->stream, right->done, 0));
    HIPCHK(hipStreamWaitEvent(left->stream, left->done, 0));
    StereoArgs a{};
    a.L = side_of(left, 0, 1);
    a.R = side_of(right, 0, 1);
    a.cap = left->g.out_base[left->g.nlevels];
    if (right->g.out_base[right->g.nlevels] != a.cap) return ORBX_EINVAL;
    a.mbf = mbf;
    a.mb = mb;
    int rc = run_stereo(left->g, a, 1, left, left->stream);
    if (rc) return rc;
    // count, mvuRight, mvDepth in one round trip through the left engine's pinned staging
    const size_t cap = (size_t)a.cap;
    if (left->h_stage.ensure(64 + 8 * cap)) return ORBX_EDEVICE;
    HostCopy hc(left->stream, nullptr);   // same stream as the launches
    hc.d2h(left->h_stage.p, left->d_cnt.as<int>(), sizeof(int));
    hc.d2h(left->h_stage.as<void>(64), left->d_st_u.p, 4 * cap);
    hc.d2h(left->h_stage.as<void>(64 + 4 * cap), left->d_st_depth.p, 4 * cap);
    if (hc.finish()) return ORBX_EDEVICE;
    if (n != *left->h_stage.as<int>()) return ORBX_EINVAL;
    if (n > 0) {
        if (!u_right || !depth) return ORBX_EINVAL;
        std::memcpy(u_right, left->h_stage.as<void>(64), 4 * (size_t)n);
        std::memcpy(depth, left->h_stage.as<void>(64 + 4 * cap), 4 * (size_t)n);
    }
    return ORBX_OK;
}

int orbm_stereo_match_batch_device(orbx_engine *e, int n_pairs, float mbf, float mb, void *stream) {
    if (!e || n_pairs <= 0) return ORBX_EINVAL;
    if (e->last_n < 2 * n_pairs) return ORBX_ESTATE;
    StereoArgs a{};
    a.L = side_of(e, 0, 2);
    a.R = side_of(e, 1, 2);
    a.cap = e->g.out_base[e->g.nlevels];
    a.mbf = mbf;
    a.mb = mb;
    return run_stereo(e->g, a, n_pairs, e, stream ? (hipStream_t)stream : e->stream);
}

int orbm_stereo_results(orbx_engine *e, const float **d_u_right, const float **d_depth) {
    if (!e || !e->d_st_u.p) return ORBX_ESTATE;
    if (d_u_right) *d_u_right = e->d_st_u.as<float>();
    if (d_depth) *d_depth = e->d_st_depth.as<float>();
    return ORBX_OK;
}

int orbm_stereo_fetch(orbx_engine *e, int pair, float *u_right, float *depth, int cap) {
    if (!e) return ORBX_EINVAL;
    if (!e->d_st_u.p || e->st_pairs == 0) return ORBX_ESTATE;
    if (pair < 0 || pair >= e->st_pairs) return ORBX_EINVAL;
    const int kc = e->g.out_base[e->g.nlevels];
    if (cap < kc) return ORBX_ECAP;
    HIPCHK(hipSetDevice(e->device));
    HostCopy hc(e->stream, e->done);
    hc.d2h(u_right, e->d_st_u.as<float>() + (size_t)pair * kc, 4 * (size_t)kc);
    hc.d2h(depth, e->d_st_depth.as<float>() + (size_t)pair * kc, 4 * (size_t)kc);
    return hc.finish();
}

int orbm_create(float nnratio, int check_ori, orbm_matcher **out) {
    if (!out) return ORBX_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ORBX_EDEVICE;
    orbm_matcher *m = new orbm_matcher();
    m->nnratio = nnratio;
    m->check_ori = check_ori != 0;
    if (hipGetDevice(&m->device) != hipSuccess || hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
        !(m->done = make_done_event())) {
        if (m->stream) (void)hipStreamDestroy(m->stream);
        delete m;
        return ORBX_EDEVICE;
    }
    *out = m;
    return ORBX_OK;
}

void orbm_destroy(orbm_matcher *m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->done) { (void)hipEventSynchronize(m->done); (void)hipEventDestroy(m->done); }
    DevBuf *bufs[] = {&m->q, &m->db, &m->off, &m->idx, &m->out, &m->kun, &m->desc, &m->cnt, &m->keys,
                      &m->nkeys, &m->cstart, &m->prev, &m->m12, &m->nmatch, &m->list, &m->lcnt};
    for (DevBuf *b : bufs) b->release();
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int orbm_hamming_best2_cand_device(orbm_matcher *m, const uint8_t *d_q, int nq, const uint8_t *d_db, int ndb,
                                   const int32_t *d_cand_off, const int32_t *d_cand_idx, int32_t *d_best_idx,
                                   int32_t *d_best_d, int32_t *d_second_d, void *stream) {
    if (!m || nq < 0 || ndb < 0 || ndb >= (1 << 20)) return ORBX_EINVAL;
    if (nq == 0) return ORBX_OK;
    if (!d_q || (ndb > 0 && !d_db) || !d_best_idx || !d_best_d || !d_second_d) return ORBX_EINVAL;
    HIPCHK(hipSetDevice(m->device));
    const hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    HIPCHK(order_after_done(m, s));
    if (d_cand_off) {
        if (!d_cand_idx) return ORBX_EINVAL;
        hamming_best2_kernel<true><<<(nq + 3) / 4, 256, 0, s>>>(d_q, nq, d_db, ndb, d_cand_off, d_cand_idx, d_best_idx,
                                                                 d_best_d, d_second_d);
    } else {
        hamming_best2_kernel<false><<<(nq + 3) / 4, 256, 0, s>>>(d_q, nq, d_db, ndb, nullptr, nullptr, d_best_idx,
                                                                  d_best_d, d_second_d);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(mark_done(m, s));
    return ORBX_OK;
}

int orbm_hamming_best2_cand(orbm_matcher *m, const uint8_t *q, int nq, const uint8_t *db, int ndb,
                            const int32_t *cand_off, const int32_t *cand_idx, int32_t *best_idx, int32_t *best_d,
                            int32_t *second_d) {
    if (!m || nq < 0 || ndb < 0 || ndb >= (1 << 20)) return ORBX_EINVAL;
    if (nq == 0) return ORBX_OK;
    if (!q || !best_idx || !best_d || !second_d || (ndb > 0 && !db)) return ORBX_EINVAL;
    size_t nc = 0;
    if (cand_off) {   // CSR candidate lists: monotone offsets, indices inside db
        if (!cand_idx && cand_off[nq] > cand_off[0]) return ORBX_EINVAL;
        if (cand_off[0] != 0) return ORBX_EINVAL;
        for (int i = 0; i < nq; i++)
            if (cand_off[i + 1] < cand_off[i] || cand_off[i + 1] - cand_off[i] >= (1 << 20)) return ORBX_EINVAL;
        nc = (size_t)cand_off[nq];
        for (size_t c = 0; c < nc; c++)
            if (cand_idx[c] < 0 || cand_idx[c] >= ndb) return ORBX_EINVAL;
    }
    HIPCHK(hipSetDevice(m->device));
    HIPCHK(hipStreamWaitEvent(m->stream, m->done, 0));
    if (m->q.ensure(32 * (size_t)nq) || m->db.ensure(32 * (size_t)std::max(ndb, 1)) || m->out.ensure(12 * (size_t)nq) ||
        m->off.ensure(4 * ((size_t)nq + 1)) || m->idx.ensure(4 * std::max<size_t>(nc, 1)))
        return ORBX_EDEVICE;
    HostCopy up(m->stream, nullptr);
    up.h2d(m->q.p, q, 32 * (size_t)nq);
    up.h2d(m->db.p, db, 32 * (size_t)ndb);
    if (cand_off) {
        up.h2d(m->off.p, cand_off, 4 * ((size_t)nq + 1));
        up.h2d(m->idx.p, cand_idx, 4 * nc);
    }
    if (up.err != hipSuccess) return ORBX_EDEVICE;
    int *o = m->out.as<int>();
    const int rc = orbm_hamming_best2_cand_device(m, m->q.as<uint8_t>(), nq, m->db.as<uint8_t>(), ndb,
                                                  cand_off ? m->off.as<int>() : nullptr, cand_off ? m->idx.as<int>() : nullptr,
                                                  o, o + nq, o + 2 * nq, m->stream);
    if (rc) return rc;
    HostCopy dn(m->stream, nullptr);
    dn.d2h(best_idx, o, 4 * (size_t)nq);
    dn.d2h(best_d, o + nq, 4 * (size_t)nq);
    dn.d2h(second_d, o + 2 * nq, 4 * (size_t)nq);
    return dn.finish();
}

// The brute-force form without a matcher handle: one matcher per calling thread (its own stream
// and buffers), so concurrent callers never share state or wait for each other.
int orbm_hamming_best2(const uint8_t *q, int nq, const uint8_t *db, int ndb, int *best_idx, int *best_d,
                       int *second_d) {
    struct Tls {
        orbm_matcher *m = nullptr;
        ~Tls() { orbm_destroy(m); }
    };
    static thread_local Tls tls;
    if (nq < 0 || ndb < 0 || ndb >= (1 << 20)) return ORBX_EINVAL;
    if (nq == 0) return ORBX_OK;
    if (!tls.m) {
        const int rc = orbm_create(0.6f, 1, &tls.m);
        if (rc) return rc;
    }
    return orbm_hamming_best2_cand(tls.m, q, nq, db, ndb, nullptr, nullptr, best_idx, best_d, second_d);
}

}  // extern "C"
