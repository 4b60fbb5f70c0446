// MI355X-native ORBextractor: pyramid, per-cell FAST, quadtree distribution, IC_Angle,
// Gaussian blur and steered BRIEF as hand-written HIP kernels for gfx950, batched over
// many images per launch. Behaviour follows ORBextractor::operator() of ORB-SLAM2-noted
// (ORBextractor.cc:1543-1658) bit-for-bit; the OpenCV primitives follow SURVEY.md
// Appendix A. See DESIGN.md for layout and rooflines.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <type_traits>

#include "orb_device.h"
#include "orb_engine.h"
#include "orb_pattern_31.inc"

using namespace orbamd;

namespace orbamd {

static __constant__ __attribute__((aligned(16))) int8_t c_pattern[1024];  // bit_pattern_31_ (ORBextractor.cc:209-467) as data
static __constant__ int c_umax[16];
// describe2_kernel's per-lane constants (built on the host, orbx_create), one 48-byte load per lane:
//  * wt[k]: IC_Angle byte weights of the lane's row v = lane / 8 - 15 + 8 k, dword w = lane % 8 (the
//    row segment u = 4w-16 .. 4w-13): x = (u + 16) where |u| <= umax[|v|] else 0, y = 1 / 0 mask;
//  * pmask: the steered-BRIEF patch loads (lanes 0..59: row lane / 10 + 6 k, dword lane % 10 of the
//    40-byte aligned row window): bit 7 p + k = the dword can hold a pixel some rotation of the
//    pattern samples when the window starts p = 0..3 bytes before the patch (from bit_pattern_31_'s
//    radius); the others are not loaded.
// One table, so pmask arrives with the weights the first IC_Angle loads already wait for (a separate
// constant load was sunk to its first use and waited vmcnt(0) behind every load in flight there)
struct DescLane {
    uint2 wt[4];
    uint32_t pmask, pad[3];
};
static __constant__ __attribute__((aligned(16))) DescLane c_dlane[64];

#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "orbslam2_amd: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return ORBX_EDEVICE;                                                    \
        }                                                                           \
    } while (0)

void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}
int DevBuf::ensure(size_t n) {
    if (n <= bytes && p) return 0;
    release();
    if (n == 0) n = 16;
    if (hipMalloc(&p, n) != hipSuccess) { p = nullptr; return ORBX_EDEVICE; }
    bytes = n;
    return 0;
}

// ------------------------------------------------------------------------------------
// Level image addressing. Level 0 is the caller's input buffer (no copy); levels >= 1 live
// in the engine's pyramid block. Unpadded: the 19-px border of ComputePyramid
// (ORBextractor.cc:1704-1727) is never read downstream.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ const uint8_t *level_ptr(const ExtractGeom &g, const uint8_t *in,
                                                    const uint8_t *pyr, int b, int l, int *pitch) {
    if (l == 0) { *pitch = g.in_pitch; return in + (long long)b * g.in_stride; }
    *pitch = g.bp[l];
    return pyr + (long long)b * g.pyr_stride + g.pyr_off[l];
}

// ------------------------------------------------------------------------------------
// K1: cv::resize(INTER_LINEAR) of level l-1 into level l (ComputePyramid :1686-1691,
// SURVEY.md A.2). Column/row coefficient tables are precomputed on the host with the
// reference's float/double arithmetic; the kernel does the exact integer math in OpenCV's
// two passes (HResizeLinear: Q11 column sums per source row; VResizeLinear: row blend).
// One workgroup per RZ_TW x RZ_TH output tile:
//  1. horizontal pass over the tile's source rows [ry(y0).r0, ry(y1-1).r1] (each source row
//     once, ~1.2 per output row): a thread owns 4 output columns, reads the <= 12 source
//     bytes they span with 3 aligned dwords, picks each (p[sx], p[sx1]) pair with one
//     v_perm and forms a0 p[sx] + a1 p[sx1] with one v_dot2_u32_u16 -> int sums in LDS;
//  2. vertical pass: two ds_read_b128 per 4 output pixels, (S0 b0 + S1 b1 + 2^21) >> 22
//     (FixedPtCast) or the SSE2 VResizeLinearVec_32s8u lane arithmetic for the columns
//     OpenCV 3.2 vectorises (resize_mode 1), one dword store per 4 pixels.
// Column table entry: x = sx | a0 << 16, y = a1 | (sx1 - sx) << 16.
// ------------------------------------------------------------------------------------
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// dword of image bytes [x, x+4) of row `rowp` (x .. x+3 inside the row) from aligned loads
__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *pa = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t lo = pa[0];
    const uint32_t hi = sh ? pa[1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// bytes `sel` (0..3) of four dwords gathered into one dword (a0 -> byte 0 .. a3 -> byte 3)
template <int SEL>
__device__ __forceinline__ uint32_t gather_byte(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
    const uint32_t lo = __builtin_amdgcn_perm(a1, a0, 0x0c0c0000u | (uint32_t)(SEL + 4) << 8 | (uint32_t)SEL);
    const uint32_t hi = __builtin_amdgcn_perm(a3, a2, (uint32_t)(SEL + 4) << 24 | (uint32_t)SEL << 16 | 0x0c0cu);
    return lo | hi;
}

__device__ __forceinline__ uint32_t resize_px_simd(int S0, int S1, int4 ry) {  // SSE2 lane arithmetic
    int x0 = S0 >> 4, y0 = S1 >> 4;
    x0 = min(max(x0, -32768), 32767);
    y0 = min(max(y0, -32768), 32767);
    int t = ((x0 * (int)(int16_t)ry.z) >> 16) + ((y0 * (int)(int16_t)ry.w) >> 16);
    t = min(max(t, -32768), 32767);
    t = min(max(t + 2, -32768), 32767) >> 2;
    return (uint32_t)min(max(t, 0), 255);
}

#define RZ_TW 128   // output columns per tile (32 column groups of 4)
#define RZ_TH 32    // output rows per tile (16 / 64: 3.4 / 3.0 % slower)
// XCD-aware block runs of 64 workgroups in resize_level_kernel: its reads 98 -> 53 MB per launch
// (~1 GB less per C2 step), C2 +0.25 % same box (profiles/r05_traffic_xcd.log). The same runs for
// fast_blur_kernel cut its reads 1104 -> 405 MB per launch but made it 0.79 -> 0.94 ms alone and C2
// 11 % slower: not used there.
#define ORBX_RZ_XCD 64
#define RZ_HJ 6     // source rows per thread per load batch

template <bool SIMD>
__global__ __launch_bounds__(256) void resize_level_kernel(ExtractGeom g, int l, int tiles_x, const int2 *cxt,
                                                           const int4 *ryt, const uint8_t *in, uint8_t *pyr) {
    extern __shared__ uint4 rz_h[];   // [source row][32 column groups] horizontal sums
    const int dw = g.lw[l], dh = g.lh[l];
    // XCD-aware order: each XCD takes runs of ORBX_RZ_XCD consecutive (image, tile) blocks, so tiles
    // that share source rows and columns read them through one L2
    int bxr, b;
    xcd_remap2_chunk<ORBX_RZ_XCD>(bxr, b);
    const int ty = bxr / tiles_x, tx = bxr - ty * tiles_x;
    const int x0 = tx * RZ_TW, y0 = ty * RZ_TH, y1 = min(y0 + RZ_TH, dh);
    const int sr0 = ryt[y0].x, nsr = ryt[y1 - 1].y - sr0 + 1;
    int sp;
    const uint8_t *src = level_ptr(g, in, pyr, b, l - 1, &sp);
    const int cg = threadIdx.x & 31, dx0 = x0 + 4 * cg;
    // the thread's output rows' table entries (r0, r1, b0, b1), loaded before the horizontal
    // pass so their latency hides behind it
    int4 ryv[RZ_TH / 8];
#pragma unroll
    for (int i = 0; i < RZ_TH / 8; i++) {
        const int dy = y0 + (threadIdx.x >> 5) + 8 * i;
        ryv[i] = ryt[min(dy, y1 - 1)];
    }
    // workgroup-uniform buffer descriptors over the source level and the output level: row
    // offsets as 32-bit VGPR offsets (no per-row 64-bit address arithmetic, no flat loads)
    // (the source descriptor starts at the dword holding the level's first byte: the input image of a
    // batch may start at any byte). Each descriptor's record count is its level's exact extent --
    // the source from that dword to the dword holding the last pixel of the last row, the output to
    // its last row's end -- so the hardware range check returns 0 for (and drops stores to) any byte
    // past the level; none is addressed (the guarded loads below), so this is defence in depth for
    // level 1, whose source is the caller's image (include/orbslam2_amd.h: no readable tail).
    const uint32_t s0 = (uint32_t)((uintptr_t)src & 3);
    // bytes of the source level from the descriptor base to the end of its last row: a 12-byte
    // window of the last row's last column group can reach past it, and for level 0 of a
    // batch's last image that is past the end of the caller's buffer (a fault when the buffer
    // ends on a page: 512 VGA frames are exactly 75 x 2 MiB). Those windows load dword by dword,
    // none starting past the end (an aligned dword never crosses a page).
    const uint32_t lim = s0 + (uint32_t)((g.lh[l - 1] - 1) * sp + g.lw[l - 1]);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(src - s0), 0, (int)((lim + 3u) & ~3u), 0x00020000);
    // 1. horizontal pass
    {
        int2 c[4];
#pragma unroll
        for (int k = 0; k < 4; k++) c[k] = cxt[min(dx0 + k, dw - 1)];
        const int sxa = c[0].x & 0xFFFF;
        uint32_t coef[4];
        int o[4], d[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            o[k] = (c[k].x & 0xFFFF) - sxa;   // <= 3 * scale + 1 <= 7
            d[k] = c[k].y >> 16;              // sx1 - sx (0 at the right border)
            coef[k] = (uint32_t)(c[k].x >> 16) | (uint32_t)(c[k].y & 0xFFFF) << 16;
        }
        // the lane's 4 outputs read source bytes sxa + o .. sxa + o + d; when they all fall in
        // an 8-byte window (scale <= ~1.75, every lane at 1.2), two v_alignbyte per source row
        // build the window and each output is one v_perm with a lane-constant selector + one
        // v_dot2 (else the per-row selector path below)
        uint32_t sel[4];
        int span = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            sel[k] = 0x0c000c00u | (uint32_t)(o[k] + d[k]) << 16 | (uint32_t)o[k];
            span = max(span, o[k] + d[k]);
        }
        const bool win8 = span <= 7;
        // all loads of a thread's source rows are issued before any use (6 rows x 3 dwords
        // in flight; the level-1 pass streams the input image from HBM)
        for (int jb = threadIdx.x >> 5; jb < nsr; jb += 8 * RZ_HJ) {
            uint32_t D[RZ_HJ][3];
            int mis[RZ_HJ];
#pragma unroll
            for (int u = 0; u < RZ_HJ; u++) {
                const int j = jb + 8 * u;
                if (j < nsr) {
                    const uint32_t a = (uint32_t)(sr0 + j) * (uint32_t)sp + (uint32_t)sxa + s0, al = a & ~3u;
                    mis[u] = (int)(a & 3u);
                    if (al + 12u <= lim) {
                        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rsrc, (int)al, 0, 0);
                        D[u][0] = v[0]; D[u][1] = v[1]; D[u][2] = v[2];
                    } else {
                        D[u][0] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)al, 0, 0);
                        D[u][1] = al + 4u < lim ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)al + 4, 0, 0) : 0u;
                        D[u][2] = al + 8u < lim ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)al + 8, 0, 0) : 0u;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < RZ_HJ; u++) {
                const int j = jb + 8 * u;
                if (j >= nsr) break;
                uint32_t hv[4];
                if (win8) {
                    const uint32_t W0 = __builtin_amdgcn_alignbyte(D[u][1], D[u][0], (uint32_t)mis[u]);
                    const uint32_t W1 = __builtin_amdgcn_alignbyte(D[u][2], D[u][1], (uint32_t)mis[u]);
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        hv[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(W1, W0, sel[k])),
                                                       __builtin_bit_cast(u16x2, coef[k]), 0u, false);
                } else
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int q = o[k] + mis[u];   // byte offset of p[sx] in D0..D2 (<= 10)
                    const bool up = q > 6;
                    const int qq = up ? q - 4 : q;
                    const uint32_t pr = __builtin_amdgcn_perm(up ? D[u][2] : D[u][1], up ? D[u][1] : D[u][0],
                                                              0x0c000c00u | (uint32_t)(qq + d[k]) << 16 | (uint32_t)qq);
                    hv[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, pr), __builtin_bit_cast(u16x2, coef[k]), 0u, false);
                }
                rz_h[j * 32 + cg] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
            }
        }
    }
    __syncthreads();
    // 2. vertical pass
    uint8_t *dst = pyr + (long long)b * g.pyr_stride + g.pyr_off[l];
    const __amdgpu_buffer_rsrc_t rdst =
        __builtin_amdgcn_make_buffer_rsrc((void *)dst, 0, (dh - 1) * g.bp[l] + dw, 0x00020000);
    const int n = min(4, dw - dx0);
    if (n <= 0) return;
    const uint32_t bpl = (uint32_t)g.bp[l];
#pragma unroll
    for (int i = 0; i < RZ_TH / 8; i++) {
        const int dy = y0 + (threadIdx.x >> 5) + 8 * i;
        if (dy >= y1) break;
        const int4 ry = ryv[i];   // r0, r1, b0, b1
        const uint4 A = rz_h[(ry.x - sr0) * 32 + cg], B = rz_h[(ry.y - sr0) * 32 + cg];
        const uint32_t S0[4] = {A.x, A.y, A.z, A.w}, S1[4] = {B.x, B.y, B.z, B.w};
        uint32_t out = 0;
        if (!SIMD) {
            // FixedPtCast (b0 S0 + b1 S1 + 2^21) >> 22 as byte 3 of 4 (b0 S0 + b1 S1) + 2^23: with
            // S <= 255 * 2^11 (a0 + a1 = 2^11) and b0 + b1 = 2^11, 4 (b0 S0 + b1 S1) + 2^23 <=
            // 255 * 2^24 + 2^23 < 2^32 -- less than one bit of headroom, so engine_reserve refuses any
            // coefficient table whose pairs do not sum to exactly 2^11. Two full-rate
            // v_mad_u32_u24 per pixel and one byte gather per 4 pixels (the result is <= 255: no clamp)
            const uint32_t b0 = (uint32_t)ry.z << 2, b1 = (uint32_t)ry.w << 2;
            uint32_t t[4];
#pragma unroll
            for (int k = 0; k < 4; k++) t[k] = __umul24(S0[k], b0) + (__umul24(S1[k], b1) + (1u << 23));
            out = gather_byte<3>(t[0], t[1], t[2], t[3]);
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t v = (__umul24(S0[k], (uint32_t)ry.z) + __umul24(S1[k], (uint32_t)ry.w) + (1u << 21)) >> 22;
                if (dx0 + k < g.rz_simd_end[l]) v = resize_px_simd((int)S0[k], (int)S1[k], ry);
                out |= v << (8 * k);
            }
        }
        const uint32_t o = (uint32_t)dy * bpl + (uint32_t)dx0;
        if (n == 4) {
            __builtin_amdgcn_raw_buffer_store_b32(out, rdst, (int)o, 0, 0);
        } else {
            for (int k = 0; k < n; k++) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(out >> (8 * k)), rdst, (int)(o + k), 0, 0);
        }
    }
}

// ------------------------------------------------------------------------------------
// K2: FAST + per-cell non-maximum suppression + GaussianBlur over 128x16 tiles of every
// level, one 256-thread workgroup per tile (ComputeKeyPointsOctTree's cell loop,
// ORBextractor.cc:1084-1153, and the blur of :1617-1625).
//
// cornerScore<16> (OpenCV fast_score.cpp) returns max(th, M) - 1 where
//   M = max over the 16 circular 9-arcs of max(min_arc(v - ring), min_arc(ring - v)),
// and the FAST-9 test at threshold th is exactly M > th (the pre-tests of
// FAST_t are necessary conditions of the 9-arc test). M is pixel-intrinsic, and the cells
// of the grid partition the detection region: cell (i, j) detects in rows
// [19 + i*hCell, min(19 + (i+1)*hCell, maxBorderY - 3)) and the matching columns, its ROI
// being the detection rectangle plus cv::FAST's 3-pixel ring margin. cv::FAST's 3x3 NMS on
// the ROI scores neighbours outside the detection rectangle 0, so a pixel's NMS only reads
// the M of its 8 neighbours that share its cell. With s_th(q) = M_q > th ? M_q - 1 : 0 the
// survivors at a threshold th >= tlo = min(iniThFAST, minThFAST) are exactly the
// survivors at tlo with M > th (every neighbour keeps its order with M_p - 1), so one NMS
// at tlo serves both passes of the per-cell retry: the workgroup emits every survivor at
// tlo into its cell's slot list (score M - 1), and the quadtree kernel keeps a cell's
// entries with score >= iniThFAST when there is one, else those >= minThFAST (:1119-1135).
// The order inside a cell's list is free (global atomics): the only order the quadtree
// depends on -- the first key of maximal response in a node (:1028-1034) -- is restated
// there as the reference list position (cell row-major, then row-major in the cell).
//
// The LDS halo tile (24x136 bytes, reflect-101 at the level edges) feeds:
//  1. staging: one unaligned dwordx2 load per 8-byte pair (per-byte reflection only for the
//     pairs crossing a level edge, behind a wave-uniform branch);
//  2. FAST pre-filter over the tile plus its one-pixel ring (the NMS neighbours): every
//     9-arc holds two adjacent compass pixels (ring 0/4/8/12), so a pixel is a darker
//     (brighter) candidate only if an adjacent compass pair passes the halved-difference test
//     (SWAR on v_lerp_u8, four pixels per dword). Candidates (~20 % of the detection area,
//     ~5 % score above tlo) are pooled per workgroup (DPP scan of the lanes' counts), flagged
//     FB_INTILE when they are tile pixels;
//  3. exact M per candidate: one 9-arc score for the polarity the compass test allows
//     (v_xad signs the differences, v_min3 / v_max3 reduce the arcs; the candidates of both
//     polarities get their brighter score in a queued pass) into an LDS score tile (0
//     elsewhere: every M <= tlo behaves as 0). Tile pixels with M > tlo go to the wavefront's
//     hot list;
//  4. GaussianBlur 9x9 sigma 2 (bit-exact fixed-point path, SURVEY.md A.3 -- exact integer
//     row sums, Q16 column sums, (acc + 2^15) >> 16) as banded int8 products on the matrix
//     cores (fast_blur_mfma), written with dword stores at the row pitch g.bp[l];
//  5. NMS of the hot pixels against their in-cell neighbours and the atomic emission of
//     the survivors' keys (pack_key: x, y relative to minBorder, score M - 1).
// No strength map leaves the workgroup.
// ------------------------------------------------------------------------------------
#ifndef ORBX_BOUNDS_CHECK
#define ORBX_BOUNDS_CHECK 0
#endif
#define ORBX_BLUR_ALIGN 128   // blurred-level row alignment in bytes (16, the pyramid's: 481 -> 468 MB written, C2 -0.7 %)
#define FB_TW 128
#define FB_TH 16
#define FB_SB (FB_TW + 8)   // staged bytes per tile row (cols x0-4 .. x0+131)
#define FB_SD (FB_SB / 4)   // staged dwords per tile row
#define FB_LW (FB_TW + 8)   // LDS tile row stride in bytes (8-aligned rows for the blur's ds_read_b64)
#define FB_LD (FB_LW / 4)   // LDS tile row stride in dwords
#define FB_MR (FB_TH + 2)   // score rows y0-1 .. y0+16 (tile + NMS ring)
#define FB_NG (FB_MR * FB_LD)   // score tile dwords (a multiple of 4, <= 1024: cleared as uint4 by 256 threads)
#define FB_CCAP (2 * FB_MR * (FB_TW + 2))   // candidate entries: both polarities of every score pixel
                                          // (brighter from the front, darker from the back)
#define FB_INTILE 0x8000   // candidate flag: a tile pixel (not the NMS ring)
#define FB_POS 0x0FFF      // candidate: score-tile byte offset

__device__ __forceinline__ int refl101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

// bytes j, j+1 of the little-endian 16-byte segment w[0..3], zero-extended into int16 lanes
__device__ __forceinline__ s16x2 byte_pair(const uint32_t *w, int j) {
    const int k = j & 3, d = j >> 2;
    const uint32_t r = k < 3 ? __builtin_amdgcn_perm(0u, w[d], 0x0c000c00u | ((uint32_t)(k + 1) << 16) | (uint32_t)k)
                             : __builtin_amdgcn_perm(w[d + 1], w[d], 0x0c040c03u);
    return __builtin_bit_cast(s16x2, r);
}

// inclusive wavefront scan of int as six fused DPP adds (row_shr 1/2/4/8 with zero-filled
// out-of-row sources, row_bcast 15 / 31 on rows 1, 3 / 2, 3; unwritten rows keep v). Written
// out because the compiler keeps update_dpp + add as a v_mov_b32_dpp, a v_add and a zeroed
// old operand per step; the s_nop 1 covers the VALU-write -> DPP-read hazard.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    asm("s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(v));
    return v;
}

__device__ __forceinline__ uint32_t lane_rank(unsigned long long bal) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

// Two candidates per lane in packed f16 (candidate a: low half, b: high half). A pixel byte is
// kept as the f16 bit pattern of the byte, i.e. the denormal x * 2^-24: sums and differences of
// such values are exact fixed-point arithmetic (fp16 denormals are preserved, the kernel's
// float_denorm_mode_16_64), the packed min3 / max3 keep their order, and a score M in [0, 255]
// comes back as the integer bits of its half. VOP3P min3 / max3 have no compiler builtin here.
__device__ __forceinline__ uint32_t pk_min3h(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t pk_max3h(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t pk_fmah(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_pk_fma_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t pk_subh(uint32_t a, uint32_t b) {   // a - b per half
    uint32_t r;
    asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// the 16 Bresenham ring bytes and the centre byte of two score-tile pixels (pa, pb = the pixel's
// LDS tile byte - 3, the score row being LDS tile row + 3) packed into f16 halves: two ds_read_u8
// and one v_perm per ring pixel (ds_read_u8_d16 / _d16_hi cannot pack them here: on this gfx950
// the d16 loads zero the other half, tools/microbench/f16_denorm_probe.hip)
__device__ __forceinline__ void ring2(const uint8_t *pa, const uint8_t *pb, uint32_t (&R)[16], uint32_t &V) {
    constexpr int OFF[16] = {(3 + 3) * FB_LW + 0 + 3,  (3 + 3) * FB_LW + 1 + 3,  (3 + 2) * FB_LW + 2 + 3,
                             (3 + 1) * FB_LW + 3 + 3,  (3 + 0) * FB_LW + 3 + 3,  (3 - 1) * FB_LW + 3 + 3,
                             (3 - 2) * FB_LW + 2 + 3,  (3 - 3) * FB_LW + 1 + 3,  (3 - 3) * FB_LW + 0 + 3,
                             (3 - 3) * FB_LW - 1 + 3,  (3 - 2) * FB_LW - 2 + 3,  (3 - 1) * FB_LW - 3 + 3,
                             (3 + 0) * FB_LW - 3 + 3,  (3 + 1) * FB_LW - 3 + 3,  (3 + 2) * FB_LW - 2 + 3,
                             (3 + 3) * FB_LW - 1 + 3};
#pragma unroll
    for (int k = 0; k < 16; k++) R[k] = (uint32_t)pa[OFF[k]] | (uint32_t)pb[OFF[k]] << 16;
    V = (uint32_t)pa[3 * FB_LW + 3] | (uint32_t)pb[3 * FB_LW + 3] << 16;
}
// M of both halves, all of one polarity: brighter max(0, max_arc min_k ring_k - v) (min3 over
// the arcs, max3 over the 16 starts), darker max(0, v - min_arc max_k ring_k) (the mirror) --
// exact on the denormal-encoded bytes, no per-pixel difference pass
template <bool BRIGHT>
__device__ __forceinline__ uint32_t fast_arc_score2(const uint32_t (&R)[16], uint32_t V) {
    auto op3 = [](uint32_t a, uint32_t b, uint32_t c) { return BRIGHT ? pk_min3h(a, b, c) : pk_max3h(a, b, c); };
    auto red3 = [](uint32_t a, uint32_t b, uint32_t c) { return BRIGHT ? pk_max3h(a, b, c) : pk_min3h(a, b, c); };
    uint32_t n3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) n3[k] = op3(R[k], R[(k + 1) & 15], R[(k + 2) & 15]);
    uint32_t n9[16];
#pragma unroll
    for (int k = 0; k < 16; k++) n9[k] = op3(n3[k], n3[(k + 3) & 15], n3[(k + 6) & 15]);
    uint32_t A = red3(n9[0], n9[1], n9[2]);
#pragma unroll
    for (int k = 3; k < 15; k += 2) A = red3(A, n9[k], n9[k + 1]);
    A = red3(A, n9[15], n9[15]);
    const uint32_t d = BRIGHT ? pk_subh(A, V) : pk_subh(V, A);
    return pk_max3h(d, 0u, 0u);   // -0 / negative halves -> +0
}

// GaussianBlur 9x9 sigma 2 of one 128 x 16 tile as two banded integer products on
// v_mfma_i32_16x16x32_i8 (lane maps: tools/microbench/mfma_i8_layout.hip). OpenCV's bit-exact
// fixed-point path: exact row sums R = sum_k w_k p, then (sum_i w_i R + 2^15) >> 16
// with w = [7,17,32,46,52,46,32,17,7] (sum 256).
//  row pass, per 16-column block and 16-row block: R (rows x cols) = T (rows x staged cols) . W,
//    A = staged pixels - 128 (byte XOR 0x80: the i8 MFMA is signed; 8 bytes per lane = the 32
//    staged columns a 16-column block reads), B = band W[c][x] = w[c - x]; the accumulator is
//    R - 2^15, whose low 16 bits are R ^ 0x8000: byte 1 is hi(R) - 128 and byte 0 is lo(R),
//    R = 256 hi + lo;
//  column pass: O^T (cols x out rows) = R^T . V on the hi and lo bytes (two MFMAs), the row-pass
//    accumulators used in place as A (lane l holds rows 4 (l >> 4) + r and 16 + 4 (l >> 4) + r of
//    column l & 15: the K order is permuted and V's rows follow it), B = band
//    V[rho(k)][y] = w[rho(k) - y]; the hi product starts from 128 * 257 + 128 (the byte offsets,
//    times 256, and the rounding 2^15 / 256), so out = (256 accH + accL) >> 16 is byte 2 of
//    256 accH + accL.
// 8 MFMAs and ~80 VALU instructions per wavefront replace ~160 VALU instructions of v_dot4 /
// v_dot2 row and column passes.
struct FbBlurTab {
    unsigned long long wb[64];   // row-pass B fragment of lane l: W[k = 8 (l >> 4) + j][x = l & 15]
    unsigned long long vb[64];   // column-pass B fragment: V[rho(k)][y = l & 15]
};
constexpr FbBlurTab make_fb_blur_tab() {
    constexpr int K9[9] = {7, 17, 32, 46, 52, 46, 32, 17, 7};
    FbBlurTab t{};
    for (int l = 0; l < 64; l++) {
        const int n = l & 15, gq = l >> 4;
        for (int j = 0; j < 8; j++) {
            const int tw = 8 * gq + j - n;
            const int rho = j < 4 ? 4 * gq + j : 16 + 4 * gq + (j - 4);
            const int tv = rho - n;
            const unsigned long long bw = (tw >= 0 && tw <= 8) ? (unsigned long long)K9[tw] : 0ull;
            const unsigned long long bv = (tv >= 0 && tv <= 8) ? (unsigned long long)K9[tv] : 0ull;
            t.wb[l] |= bw << (8 * j);
            t.vb[l] |= bv << (8 * j);
        }
    }
    return t;
}
static __constant__ FbBlurTab c_fbblur = make_fb_blur_tab();

typedef int i32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ long i8x8(uint32_t lo, uint32_t hi) { return (long)((unsigned long long)hi << 32 | lo); }

// BM32 (blur_mode 1): OpenCV 3.2's column pass (SymmColumnVec_32s8u, README.md:9) accumulates in
// float and rounds half to EVEN (_mm_cvtps_epi32) over the columns it vectorises -- the prefix
// [0, w & ~3) of each row (16, then 4 at a time) -- while its scalar tail and OpenCV >= 3.4 round
// half up. 256 accH + accL is exactly acc + 2^15, so an exact tie (acc mod 2^17 = 2^15) reads
// as low 17 bits == 0x10000, and half-even takes one off the (odd) output byte there.
template <bool BM32>
__device__ __forceinline__ void fast_blur_mfma(const uint32_t *tin, uint8_t *dst, int bp, int x0, int y0, int w,
                                               int h, int xb0, int xb1, int lane) {
    const int n = lane & 15, gq = lane >> 4;
    const long WB = (long)c_fbblur.wb[lane], VB = (long)c_fbblur.vb[lane];
    const uint8_t *t8 = (const uint8_t *)tin;
    // row-pass A: staged row 16 yb + n (rows past the 24 staged ones repeat row 23: their V
    // weights are 0), columns 16 xb + 8 gq + 0..7 (the last block's upper columns fall past
    // the staged row: W is 0 there)
    const int r0 = n, r1 = min(16 + n, FB_TH + 7);
    const uint32_t XM = 0x80808080u;
    const int KH = 128 * 257 + 128;
    const i32x4 z = {0, 0, 0, 0}, kh = {KH, KH, KH, KH};
    // blocks past the level's right edge hold no output column (the last tile of a row: 10 % of the
    // tile area over C2's levels, 16 % over C3's) -- not computed
    const int xbe = min(xb1, (w - x0 + 15) >> 4);
#pragma unroll
    for (int xb = xb0; xb < xbe; xb++) {   // wave-uniform range of 16-column blocks
        const int c = 16 * xb + 8 * gq;
        const uint2 a0 = *(const uint2 *)(t8 + r0 * FB_LW + c);
        const uint2 a1 = *(const uint2 *)(t8 + r1 * FB_LW + c);
        const i32x4 R0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(i8x8(a0.x ^ XM, a0.y ^ XM), WB, z, 0, 0, 0);
        const i32x4 R1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(i8x8(a1.x ^ XM, a1.y ^ XM), WB, z, 0, 0, 0);
        // column-pass A fragments: K elements 0..3 = rows 4 gq + r (R0), 4..7 = rows 16 + 4 gq + r (R1)
        const long AH = i8x8(gather_byte<1>((uint32_t)R0.x, (uint32_t)R0.y, (uint32_t)R0.z, (uint32_t)R0.w),
                             gather_byte<1>((uint32_t)R1.x, (uint32_t)R1.y, (uint32_t)R1.z, (uint32_t)R1.w));
        const long AL = i8x8(gather_byte<0>((uint32_t)R0.x, (uint32_t)R0.y, (uint32_t)R0.z, (uint32_t)R0.w) ^ XM,
                             gather_byte<0>((uint32_t)R1.x, (uint32_t)R1.y, (uint32_t)R1.z, (uint32_t)R1.w) ^ XM);
        const i32x4 OH = __builtin_amdgcn_mfma_i32_16x16x32_i8(AH, VB, kh, 0, 0, 0);
        const i32x4 OL = __builtin_amdgcn_mfma_i32_16x16x32_i8(AL, VB, z, 0, 0, 0);
        // lane: output row y0 + n, columns x0 + 16 xb + 4 gq + r
        uint32_t v0 = ((uint32_t)OH.x << 8) + (uint32_t)OL.x, v1 = ((uint32_t)OH.y << 8) + (uint32_t)OL.y;
        uint32_t v2 = ((uint32_t)OH.z << 8) + (uint32_t)OL.z, v3 = ((uint32_t)OH.w << 8) + (uint32_t)OL.w;
        const int y = y0 + n, x = x0 + 16 * xb + 4 * gq;
        if (BM32) {
            const int se = w & ~3;   // OpenCV 3.2's vectorised prefix of the row
            v0 -= ((v0 & 0x1FFFFu) == 0x10000u && x + 0 < se) ? 0x10000u : 0u;
            v1 -= ((v1 & 0x1FFFFu) == 0x10000u && x + 1 < se) ? 0x10000u : 0u;
            v2 -= ((v2 & 0x1FFFFu) == 0x10000u && x + 2 < se) ? 0x10000u : 0u;
            v3 -= ((v3 & 0x1FFFFu) == 0x10000u && x + 3 < se) ? 0x10000u : 0u;
        }
        const uint32_t val = gather_byte<2>(v0, v1, v2, v3);
        if (y < h && x < w) {
            uint8_t *o = dst + (long long)y * bp + x;
            if (x + 3 < w) {
                *(uint32_t *)o = val;
            } else {
                for (int k = 0; k < w - x; k++) o[k] = (uint8_t)(val >> (8 * k));
            }
        }
    }
}

template <bool BM32>
__global__ __launch_bounds__(256) void fast_blur_kernel(ExtractGeom g, const uint8_t *in, const uint8_t *pyr,
                                                        uint8_t *blur, int *cell_cnt, uint32_t *cell_keys) {
    __shared__ __align__(16) uint32_t tin[(FB_TH + 8) * FB_LD];
    __shared__ __align__(16) uint32_t mt[FB_NG];   // exact M bytes, (mrow, x - x0 + 4)
    __shared__ uint16_t clist[FB_CCAP];   // pooled candidates (score-tile byte offsets | FB_INTILE)
    __shared__ uint16_t hlist[FB_TW * FB_TH];   // hot tile pixels (score-tile byte offsets; each at most once)
    __shared__ int ncand_sh, hcnt_sh;   // ncand_sh: brighter count | darker count << 16
    const int b = blockIdx.y;
    int t = blockIdx.x, l = 0;
    while (l + 1 < g.nlevels && t >= g.blur_tile_base[l + 1]) l++;
    t -= g.blur_tile_base[l];
    // t / blur_tiles_x by the rounded-up reciprocal (exact while t * blur_tiles_x < 2^31): scalar
    // multiplies instead of the compiler's VALU reciprocal for a scalar division
    const int ty = (int)__umulhi(2u * (unsigned)t, g.blur_tx_rcp[l]), tx = t - ty * g.blur_tiles_x[l];
    const int w = g.lw[l], h = g.lh[l];
    const int x0 = tx * FB_TW, y0 = ty * FB_TH;
    int pitch;
    const uint8_t *src = level_ptr(g, in, pyr, b, l, &pitch);
    // 1. stage rows y0-4 .. y0+19, cols x0-4 .. x0+131 as 8-byte pairs: thread -> pair
    // jj = tid % 17 of rows tid / 17 and tid / 17 + 15 (255 threads), one unaligned dwordx2 load
    // per pair; reflect-101 of rows (the 4-row halo never reaches past a level of >= 40 rows)
    // and, per byte, of the few pairs that cross the left / right edge.
    static_assert(FB_SD / 2 == 17 && FB_TH + 8 <= 30, "staging map: 17 pairs x 15 rows per pass");
    if (threadIdx.x < 255) {
        const int rr0 = (threadIdx.x * 241) >> 12, jj = threadIdx.x - 17 * rr0;   // tid / 17 for tid < 255
        const int xs = x0 - 4 + 8 * jj;
        // a pair wholly past column w + 3 feeds no output: the blur of column x < w reads up to x + 4,
        // the FAST ring and the pre-filter stop inside the detection region (x < w - 19). Not staged
        // (its LDS bytes only meet the masked outputs of a partial blur block), so the right edge's
        // reflected per-byte path runs for the one or two pairs that straddle w instead of every
        // pair of the tile's overhang
        const bool skip = xs > w + 3;
        const bool fast = skip || (xs >= 0 && xs + 7 < w);
        auto row_of = [&](int rr) {
            int yy = y0 - 4 + rr;
            yy = yy < 0 ? -yy : yy;
            yy = yy >= h ? 2 * h - 2 - yy : yy;
            return src + (long long)yy * pitch;
        };
        if (__all(fast)) {   // wave-uniform: interior pairs only (keeps the edge code out of this path)
            // both rows' loads in flight before either LDS write (one global round trip)
            const bool two = rr0 + 15 < FB_TH + 8;
            uint2 v0, v1 = make_uint2(0u, 0u);
            const uint8_t *p0, *p1;
            if (y0 >= 4 && y0 + FB_TH + 4 <= h) {   // workgroup-uniform: all 24 staged rows inside the level
                p0 = src + (long long)(y0 - 4) * pitch + (rr0 * pitch + xs);
                p1 = p0 + 15 * (long long)pitch;
            } else {
                p0 = row_of(rr0) + xs;
                p1 = row_of(min(rr0 + 15, FB_TH + 7)) + xs;
            }
            if (!skip) {
                __builtin_memcpy(&v0, p0, 8);
                if (two) __builtin_memcpy(&v1, p1, 8);
                *(uint2 *)&tin[rr0 * FB_LD + 2 * jj] = v0;
                if (two) *(uint2 *)&tin[(rr0 + 15) * FB_LD + 2 * jj] = v1;
            }
        } else if (!skip) {
            for (int rr = rr0; rr < FB_TH + 8; rr += 15) {
                const uint8_t *rowp = row_of(rr);
                uint2 v;
                if (fast) {
                    __builtin_memcpy(&v, rowp + xs, 8);
                } else {
                    v.x = v.y = 0;
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        int xx = xs + e;
                        xx = xx < 0 ? -xx : xx;
                        xx = xx >= w ? 2 * w - 2 - xx : xx;
                        const uint32_t by = rowp[xx];
                        if (e < 4) v.x |= by << (8 * e); else v.y |= by << (8 * (e - 4));
                    }
                }
                *(uint2 *)&tin[rr * FB_LD + 2 * jj] = v;
            }
        }
    }
    static_assert(FB_NG % 4 == 0 && FB_NG / 4 <= 256, "score tile cleared as one uint4 per thread");
    if (threadIdx.x < FB_NG / 4) ((uint4 *)mt)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x == 0) { ncand_sh = 0; hcnt_sh = 0; }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = wave_id();
    const int th_a = min(max(g.ini_th, 0), 255), th_b = min(max(g.min_th, 0), 255);
    const int tlo = min(th_a, th_b);
    // 2. FAST pre-filter over the score domain rows y0-1 .. y0+16, cols x0-1 .. x0+128 (the
    // tile and its NMS ring), clipped to the detection region [19, w-19) x [19, h-19) (cell
    // ROIs start at minBorder 16 and end at maxBorder = size - 16, cv::FAST detects in
    // [3, roi - 3)). Tile rows: 16 threads x 8 pixels per row; ring rows y0-1 and y0+16:
    // 17 groups of 8 each on wavefront 2; ring columns x0-1 and x0+128 (32 pixels) go to the
    // exact score unfiltered on wavefront 3 (the two wavefronts with one blur-row task).
    {
        const int dx0 = max(19, x0 - 1), dx1 = min(w - 19, x0 + FB_TW + 1);
        const int dy0 = max(19, y0 - 1), dy1 = min(h - 19, y0 + FB_TH + 1);
        // Compass bound on four pixels per dword (SWAR on v_lerp_u8, which adds two bytes and a
        // rounding bit and halves, per byte): lerp(u, ~K, 1) has its top bit set iff u >= K.
        // Darker pass at compass pixel r: c - r >= T (T = tlo + 1); brighter: r - c >= T. A
        // pixel is a candidate iff (N or S) and (E or W) pass for one polarity (every 9-arc
        // holds two adjacent compass pixels). The bound is only ever looser than the exact
        // test, never tighter.
        // One halved difference per compass pixel serves both polarities:
        // u = lerp(r, ~c, 1) = 128 + floor((r - c) / 2); brighter (r - c >= T) implies u >= KB =
        // 128 + floor(T / 2), darker (c - r >= T) implies u <= 128 - ceil(T / 2), i.e. NOT
        // u >= KD = 129 - ceil(T / 2) -- so the darker pass of a direction pair is the complement
        // of "both fail", and one NOT serves the four directions.
        const uint32_t ONE = 0x01010101u, HI = 0x80808080u;
        const int T = tlo + 1;
        const uint32_t NKB = ~((uint32_t)min(128 + (T >> 1), 255) * ONE);
        const uint32_t NKD = ~((uint32_t)(129 - ((T + 1) >> 1)) * ONE);
        auto swar4 = [&](uint32_t C, uint32_t Cm, uint32_t Cp, uint32_t N, uint32_t S) {
            const uint32_t W = __builtin_amdgcn_alignbyte(C, Cm, 1);   // cols -3 .. 0
            const uint32_t E = __builtin_amdgcn_alignbyte(Cp, C, 3);   // cols +3 .. +6
            const uint32_t NC = ~C;
            const uint32_t uN = __builtin_amdgcn_lerp(N, NC, ONE), uS = __builtin_amdgcn_lerp(S, NC, ONE);
            const uint32_t uE = __builtin_amdgcn_lerp(E, NC, ONE), uW = __builtin_amdgcn_lerp(W, NC, ONE);
            auto bk = [&](uint32_t u) { return __builtin_amdgcn_lerp(u, NKB, ONE); };   // top bit: u >= KB
            auto df = [&](uint32_t u) { return __builtin_amdgcn_lerp(u, NKD, ONE); };   // top bit: u >= KD
            const uint32_t bright = (bk(uN) | bk(uS)) & (bk(uE) | bk(uW));
            const uint32_t dark_fail = (df(uN) & df(uS)) | (df(uE) & df(uW));
            return make_uint2(bright & HI, ~dark_fail & HI);   // (brighter, darker) candidate bits
        };
        // candidates among the 8 pixels xb .. xb+7 of score row mrow (xb = x0 + 4 d): LDS dwords
        // d .. d+3 of the centre row (cols xb-4 .. xb+11), d+1 and d+2 of the rows 3 above / below
        auto prefilter8 = [&](int mrow, int d, bool active, uint32_t tflag, bool chk) {
            const int y = y0 - 1 + mrow, xb = x0 + 4 * d;
            uint2 cA = make_uint2(0u, 0u), cB = cA;   // top bit of byte i: pixel xb+i (cA), xb+4+i (cB); .x brighter, .y darker
            if (active && y >= dy0 && y < dy1 && xb + 7 >= dx0 && xb < dx1) {
                const uint32_t *row = tin + (mrow + 3) * FB_LD;
                // tile rows read dwords 0 .. 33 only; the ring rows' groups reach one dword past
                // either end (chk: those read as 0)
                auto ld = [&](const uint32_t *rw, int i) { return !chk || (unsigned)i < (unsigned)FB_SD ? rw[i] : 0u; };
                const uint32_t C0 = ld(row, d), C1 = ld(row, d + 1), C2 = ld(row, d + 2), C3 = ld(row, d + 3);
                const uint32_t *rn = row - 3 * FB_LD, *rs = row + 3 * FB_LD;
                cA = swar4(C1, C0, C2, ld(rn, d + 1), ld(rs, d + 1));
                cB = swar4(C2, C1, C3, ld(rn, d + 2), ld(rs, d + 2));
                if (xb < dx0 || xb + 8 > dx1) {   // only the lanes at the detection region's edge
                    const int lo = max(dx0 - xb, 0), hi = min(dx1 - xb, 8);   // valid pixels [lo, hi)
                    const unsigned long long vm = hi > lo ? (~0ull << (8 * lo)) & (~0ull >> (64 - 8 * hi)) : 0ull;
                    cA.x &= (uint32_t)vm; cA.y &= (uint32_t)vm;
                    cB.x &= (uint32_t)(vm >> 32); cB.y &= (uint32_t)(vm >> 32);
                }
            }
            // compaction into the pooled list: the lane's 8 candidate bits (v_dot4 gathers the
            // byte top bits), an inclusive DPP scan of their counts over the wavefront, one LDS
            // atomic per wavefront for the slots, then each lane writes its own candidates
            const int pos0 = mrow * FB_LW + 4 * d + 4;   // score-tile byte of pixel xb
            // one entry per (pixel, polarity) that passes: a pixel of both polarities gets two
            // (at most one of its two scores is nonzero, see step 3)
            const uint32_t mb = __builtin_amdgcn_udot4(cB.x >> 7, 0x80402010u,
                                                       __builtin_amdgcn_udot4(cA.x >> 7, 0x08040201u, 0u, false), false);
            const uint32_t md = __builtin_amdgcn_udot4(cB.y >> 7, 0x80402010u,
                                                       __builtin_amdgcn_udot4(cA.y >> 7, 0x08040201u, 0u, false), false);
            const int cnt = __builtin_popcount(mb) | __builtin_popcount(md) << 16;   // both counts, one scan
            const int inc = wave_incl_scan_dpp(cnt);
            const int tot8 = __builtin_amdgcn_readlane(inc, 63);
            if (tot8 == 0) return;   // wave-uniform
            int base = 0;
            if (lane == 0) base = atomicAdd(&ncand_sh, tot8);
            base = __builtin_amdgcn_readfirstlane(base) + inc - cnt;
            int bb = base & 0xFFFF, bd = FB_CCAP - 1 - (base >> 16);
            for (uint32_t mm = mb; mm; mm &= mm - 1) clist[bb++] = (uint16_t)((pos0 + __builtin_ctz(mm)) | tflag);
            for (uint32_t mm = md; mm; mm &= mm - 1) clist[bd--] = (uint16_t)((pos0 + __builtin_ctz(mm)) | tflag);
        };
        const int r = threadIdx.x >> 4, cb = (threadIdx.x & 15) * 8;   // pixels (y0 + r, x0 + cb + i)
#ifndef FB_SKIP_PRE   // instruction-count experiments (make variant VDEFS=-DFB_SKIP_...)
        if (y0 + 4 * wv + 3 >= dy0 && y0 + 4 * wv < dy1)   // wave-uniform: 4 tile rows per wavefront
            prefilter8(r + 1, cb >> 2, true, FB_INTILE, false);
        if (wv == 2) {   // ring rows: lanes 0..16 row y0-1, lanes 17..33 row y0+16
            const int hr = lane >= 17, j = lane - 17 * hr;
            if ((y0 - 1 >= dy0 && y0 - 1 < dy1) || (y0 + FB_TH >= dy0 && y0 + FB_TH < dy1))
                prefilter8(hr ? FB_TH + 1 : 0, 2 * j - 1, lane < 34, 0u, true);
        }
        if (wv == 3) {   // ring columns: lane -> (row y0 + (lane & 15), column x0-1 or x0+128)
            const int y = y0 + (lane & 15), x = lane < 16 ? x0 - 1 : x0 + FB_TW;
            const bool f = lane < 32 && y >= dy0 && y < dy1 && x >= dx0 && x < dx1;
            const unsigned long long bal = __ballot(f);
            if (bal) {   // both polarities: one brighter and one darker entry per pixel
                int base = 0;
                if (lane == 0) base = atomicAdd(&ncand_sh, __popcll(bal) * 0x10001);
                base = __builtin_amdgcn_readfirstlane(base);
                const uint16_t e = (uint16_t)(((lane & 15) + 1) * FB_LW + (x - x0 + 4));
                if (f) {
                    clist[(base & 0xFFFF) + lane_rank(bal)] = e;
                    clist[FB_CCAP - 1 - ((base >> 16) + lane_rank(bal))] = e;
                }
            }
        }
#endif
    }
    // 4. GaussianBlur on the matrix cores (fast_blur_mfma): 16-column blocks 0-2 on wavefront 0,
    // 3-5 on wavefront 1, 6-7 on wavefront 3, x the tile's 16 rows
#ifndef FB_SKIP_BLUR
    {
        // column blocks per wavefront balance the pre-filter's extra work: wavefront 2 scores
        // the ring rows (one more 8-pixel group per lane), wavefront 3 the ring columns
        const int xb0 = wv == 0 ? 0 : wv == 1 ? 3 : 6, xb1 = wv == 0 ? 3 : wv == 1 ? 6 : wv == 2 ? 6 : 8;
        fast_blur_mfma<BM32>(tin, blur + (long long)b * g.blur_stride + g.blur_off[l], g.bbp[l], x0, y0, w, h, xb0, xb1, lane);
    }
#endif
    __syncthreads();
    // 3. exact M of the pooled (pixel, polarity) entries, two per lane (halves a, b), one polarity
    // per 128-entry chunk (the brighter chunks, then the darker ones from the list's back):
    // wavefront wv takes chunks wv, wv + 4, ...; tile pixels with M > tlo go to the hot list. At
    // most one polarity of a pixel scores above 0 (a darker 9-arc with every difference > 0 meets
    // every brighter 9-arc in >= 2 pixels: 9 + 9 > 16), so the two entries of a pixel that passed
    // both compass tests never both write: a score is stored only when nonzero (the score tile is
    // zero elsewhere) and only the nonzero one can be hot.
#ifdef FB_SKIP_EXACT
    const int ncd = 0;
#else
    const int ncd = ncand_sh;
#endif
    {
        uint8_t *m8 = (uint8_t *)mt;
        const uint8_t *t8 = (const uint8_t *)tin;
        auto push_hot = [&](bool ha, int pa, bool hb, int pb) {   // both halves, one LDS atomic per chunk
            const unsigned long long ba = __ballot(ha), bb = __ballot(hb);
            if ((ba | bb) == 0) return;   // wave-uniform
            const int na = __popcll(ba);
            int h0 = 0;
            if (lane == 0) h0 = atomicAdd(&hcnt_sh, na + __popcll(bb));
            h0 = __builtin_amdgcn_readfirstlane(h0);
            // Invariant: a tile pixel is pushed at most once -- only a pixel's nonzero-scoring
            // polarity can be hot (step 3's comment; tlo >= 0), and a pixel has one entry per
            // polarity -- so hcnt_sh <= FB_TW * FB_TH (hlist's size). A change to the pre-filter or to
            // the threshold clamp must keep it: LDS writes out of range do not fault. ORBX_BOUNDS_CHECK
            // builds (make variant VDEFS=-DORBX_BOUNDS_CHECK=1) trap on a violation; the product
            // build does not pay the 5 VALU per chunk (1.4 % of the kernel, measured).
            const int ia = h0 + (int)lane_rank(ba), ib = h0 + na + (int)lane_rank(bb);
#if ORBX_BOUNDS_CHECK
            if ((ha && ia >= FB_TW * FB_TH) || (hb && ib >= FB_TW * FB_TH)) __builtin_trap();
#endif
            if (ha) hlist[ia] = (uint16_t)pa;
            if (hb) hlist[ib] = (uint16_t)pb;
        };
        // a dummy position for idle halves: a tile pixel whose ring stays inside the staged rows
        constexpr int kIdle = 4;
        const int nb = ncd & 0xFFFF, nd = ncd >> 16, chb = (nb + 127) >> 7, chd = (nd + 127) >> 7;
        auto chunk = [&](auto bright_tag, int q0, int n) {
            constexpr bool BR = decltype(bright_tag)::value;
            const int qa = q0 + lane, qb = q0 + 64 + lane;
            const bool xa = qa < n, xb = qb < n;
            const int ea = xa ? clist[BR ? qa : FB_CCAP - 1 - qa] : 0, eb = xb ? clist[BR ? qb : FB_CCAP - 1 - qb] : 0;
            const int pa = xa ? ea & FB_POS : kIdle, pb = xb ? eb & FB_POS : kIdle;
            uint32_t R[16], V;
            ring2(t8 + pa - 3, t8 + pb - 3, R, V);
            const uint32_t A = fast_arc_score2<BR>(R, V);
            const int Ma = (int)(A & 0xFFFFu), Mb = (int)(A >> 16);
            if (xa && Ma > 0) m8[pa] = (uint8_t)Ma;
            if (xb && Mb > 0) m8[pb] = (uint8_t)Mb;
            push_hot(xa && Ma > tlo && (ea & FB_INTILE), pa, xb && Mb > tlo && (eb & FB_INTILE), pb);
        };
        for (int c = wv; c < chb + chd; c += 4) {
            if (c < chb) chunk(std::true_type{}, 128 * c, nb);   // wave-uniform
            else chunk(std::false_type{}, 128 * (c - chb), nd);
        }
    }
    __syncthreads();
    // 5. 3x3 NMS of the hot pixels at tlo against their in-cell neighbours (others score 0),
    // survivors appended to their cell's slot list
    {
        const int htot = hcnt_sh;   // <= FB_TW * FB_TH (the invariant at push_hot)
        const uint8_t *m8 = (const uint8_t *)mt;
        const int hC = g.hcell[l], wC = g.wcell[l];
        const int ry_end = g.maxBY[l] - 3, rx_end = g.maxBX[l] - 3;
        for (int base = 64 * wv; base < htot; base += 256) {
            const int q = base + lane;
            if (q >= htot) continue;
            const int pos = hlist[q];
            const int mrow = pos / FB_LW, col = pos - mrow * FB_LW;
            const int y = y0 - 1 + mrow, x = x0 - 4 + col;
            // cell of (x, y): (v - 19) / cell side by a 20-bit reciprocal (exact for v < 2^20 / side)
            const int ci = (int)(((unsigned)(y - 19) * (unsigned)g.hcell_mag[l]) >> 20);
            const int cj = (int)(((unsigned)(x - 19) * (unsigned)g.wcell_mag[l]) >> 20);
            const int ry0 = 19 + ci * hC, ry1 = min(ry0 + hC, ry_end);
            const int rx0 = 19 + cj * wC, rx1 = min(rx0 + wC, rx_end);
            if (ci >= g.ncell_rows[l] || cj >= g.ncell_cols[l] || y >= ry1 || x >= rx1) continue;
            const bool up = y > ry0, dn = y + 1 < ry1, lf = x > rx0, rt = x + 1 < rx1;
            // cv::FAST's NMS at tlo keeps p iff s_p > s_q for every in-cell neighbour q, with
            // s = M > tlo ? M - 1 : 0. p is hot (M_p > tlo, so s_p = M_p - 1 >= tlo), and a
            // neighbour with M_q <= tlo has M_q - 1 < tlo <= s_p: the test is M_p > max(M_q, 1)
            // over the in-cell neighbours, on the raw M bytes (0 outside the candidates)
            const uint8_t *pm = m8 + pos;
            // the 8 neighbours read unconditionally (a hot pixel is a tile pixel: rows 1..16,
            // columns 4..131 of the 18 x 136-byte score tile, so every neighbour is inside it) and
            // masked to their cell: no divergent branch per neighbour
            int nb[8];
            const int noff[8] = {-1, 1, -FB_LW - 1, -FB_LW, -FB_LW + 1, FB_LW - 1, FB_LW, FB_LW + 1};
#pragma unroll
            for (int k = 0; k < 8; k++) nb[k] = pm[noff[k]];
            const int sp = (int)pm[0] - 1;
            const bool nin[8] = {lf, rt, up && lf, up, up && rt, dn && lf, dn, dn && rt};
#pragma unroll
            for (int k = 0; k < 8; k++) nb[k] = nin[k] ? nb[k] : 0;
            const int mn = max(max(max(nb[0], nb[1]), max(nb[2], nb[3])), max(max(nb[4], nb[5]), max(nb[6], nb[7])));
            const bool keep = (int)pm[0] > max(mn, 1);
            if (keep) {
                const long long cidx = (long long)b * g.ncell_total + g.cell_base[l] + ci * g.ncell_cols[l] + cj;
                const int slot = atomicAdd(cell_cnt + cidx, 1);
                if (slot < g.cell_cap) cell_keys[cidx * g.cell_cap + slot] = pack_key(x - 16, y - 16, sp);
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// K4: DistributeOctTree (ORBextractor.cc:696-1042), one 256-thread workgroup per
// (level, image). Exact reformulation of the list algorithm:
//  * the final std::list order equals DESCENDING node creation sequence (every node is
//    push_front'ed, :831-886/:946-986), with the push_back'ed roots last in ascending
//    order -> every node carries a sort key (creation id; roots -1-i);
//  * a phase-1 round splits every non-leaf node in list order (= reverse creation order
//    of the previous round's multi-key children); children get consecutive ids in
//    n1,n2,n3,n4 order;
//  * the final phase orders the last round's multi-key nodes by (size, id) descending
//    (the sort at :935 iterated back to front, pointer tie pinned to creation order) and
//    stops at the first node that brings the size to >= N (:991).
// Node keys live in a ping-pong key array (LDS when they fit); stable partitions keep each
// node's keys in candidate order, so "first max response" (:1028) is first in array order.
// ------------------------------------------------------------------------------------
struct QNode {
    int16_t x0, y0, x1, y1;
    int s;      // segment start in the current key buffer
    int n;      // key count
    int id;     // creation id
};

// per-node scratch of one split round
// quadrant counters: 4 x u32 fields in two u64 (q0 | q1 << 32, q2 | q3 << 32); plain u64
// adds never carry across fields for counts < 2^32
struct QCnt {
    unsigned long long a, b;
    __device__ QCnt &operator+=(const QCnt &o) { a += o.a; b += o.b; return *this; }
    __device__ QCnt operator-(const QCnt &o) const { return {a - o.a, b - o.b}; }
    __device__ QCnt operator+(const QCnt &o) const { return {a + o.a, b + o.b}; }
    __device__ int f(int k) const { return (int)(uint32_t)((k < 2 ? a : b) >> (32 * (k & 1))); }
};
__device__ __forceinline__ QCnt qone(int k) {
    const unsigned long long v = 1ull << (32 * (k & 1));
    return k < 2 ? QCnt{v, 0ull} : QCnt{0ull, v};
}

// per-node scratch of one split round
struct QTmp {
    QCnt pstart, pend;   // quadrant prefix at the node's segment start / end
    int16_t cm[4];       // child k: >= 0 next-round node, < 0 leaf -> outrec[-1 - cm]
    int keep;            // -1 divided; else next-array index of the node kept undivided
    int pad;
};

__device__ __forceinline__ void qnode_mid(const QNode &q, int *mx, int *my) {
    *mx = q.x0 + ((q.x1 - q.x0 + 1) >> 1);   // x0 + ceil((x1 - x0) / 2), DivideNode :612-613
    *my = q.y0 + ((q.y1 - q.y0 + 1) >> 1);
}

__device__ __forceinline__ int quadrant(uint32_t k, int midx, int midy) {
    return (key_x(k) >= midx ? 1 : 0) + (key_y(k) >= midy ? 2 : 0);
}

struct QShared {
    int live, next_id, n_out, n_next, n_act, cross, lim_mu;
    int root_cnt[64], root_start[64], root_fill[64], root_node[64], root_out[64];
    int wcnt[4][64];
    QCnt wsum[2][4];
};

// block-wide exclusive scan of one value per thread; two LDS slots alternate so
// back-to-back scans need one barrier each

// inclusive wavefront scan of u32 (wave_incl_scan_dpp: six fused DPP adds)
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) { return (uint32_t)wave_incl_scan_dpp((int)v); }

__device__ __forceinline__ QCnt block_scan(QShared &S, QCnt v, QCnt *total, int &par) {
    const int lane = threadIdx.x & 63, wv = wave_id();
    // the four u32 counters scan independently (their sums stay below 2^32: no carries
    // between the packed fields), on DPP instead of LDS permutes
    auto sc64 = [](unsigned long long x) {
        return (unsigned long long)wave_incl_scan_u32((uint32_t)x) |
               (unsigned long long)wave_incl_scan_u32((uint32_t)(x >> 32)) << 32;
    };
    const QCnt incl{sc64(v.a), sc64(v.b)};
    if (lane == 63) S.wsum[par][wv] = incl;
    __syncthreads();
    QCnt base{0ull, 0ull}, tot{0ull, 0ull};
#pragma unroll
    for (int w = 0; w < ORBX_QT_THREADS / 64; w++) {
        const QCnt s = S.wsum[par][w];
        if (w < wv) base += s;
        tot += s;
    }
    par ^= 1;
    *total = tot;
    return base + incl - v;
}

// scalar form (one u64 lane)
__device__ __forceinline__ unsigned long long block_scan64(QShared &S, unsigned long long v,
                                                           unsigned long long *total, int &par) {
    QCnt tot;
    const QCnt r = block_scan(S, QCnt{v, 0ull}, &tot, par);
    *total = tot.a;
    return r.a;
}

// bitonic sort of n (pow2) u64 values, descending. Thread t owns elements t + 256 e, so a
// stage with j < 64 pairs elements of the same wavefront: those stages are ordered with a
// wavefront LDS fence; workgroup barriers only around the stages with j >= 64 (10 of the 45
// stages at n = 512).
__device__ void block_sort_desc(unsigned long long *a, int n) {
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += ORBX_QT_THREADS) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = a[i], y = a[ixj];
                    const bool desc = (i & k) == 0;
                    if (desc ? (x < y) : (x > y)) { a[i] = y; a[ixj] = x; }
                }
            }
            // a stage with j >= 64 writes other wavefronts' elements: barrier after it, and
            // before the next one that reads across wavefronts (and at the end)
            const int jn = j > 1 ? j >> 1 : k;   // next stage's distance (k: next k's first)
            if (j >= 64 || jn >= 64 || (j == 1 && k == n)) __syncthreads();
            else wave_lds_sync();
        }
    }
}

// descending order of n distinct u64 values by rank counting: src[i] goes to
// dst[#{j : src[j] > src[i]}]. Every lane of a wavefront reads the same src[j], so with src
// in LDS each read is a broadcast and the whole sort is one dependent pass (the bitonic
// network's 45 barrier-separated stages at n = 512 are latency bound). Two elements per
// thread share each read, and sixteen reads (eight ds_read_b128) are in flight per step:
// src is 16-byte aligned and zero-padded to a multiple of 16 (zeros never outrank a value).
// Ends with a workgroup barrier.
__device__ void block_rank_sort_desc(const unsigned long long *src, unsigned long long *dst, int n) {
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 *s2 = (const u64x2 *)src;
    const int n16 = (n + 15) >> 4;
    for (int i = threadIdx.x; i < n; i += 2 * ORBX_QT_THREADS) {
        const int i2 = i + ORBX_QT_THREADS;
        const unsigned long long v = src[i], w = i2 < n ? src[i2] : ~0ull;
        int r = 0, r2 = 0;
        for (int j = 0; j < n16; j++) {
            u64x2 u[8];
#pragma unroll
            for (int k = 0; k < 8; k++) u[k] = s2[8 * j + k];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                r += (u[k].x > v) + (u[k].y > v);
                r2 += (u[k].x > w) + (u[k].y > w);
            }
        }
        dst[r] = v;
        if (i2 < n) dst[r2] = w;
    }
    __syncthreads();
}

// Quadtree working set of one (image, level)
struct QT {
    QNode *cur, *nxt;
    QTmp *tmp;
    unsigned long long *outrec, *sortbuf;
    uint32_t *K[2];
    int16_t *NO[2];   // node index of each key position (-1: not in a live multi-key node)
    int src;          // buffer holding the live nodes' keys
    int M, NP, NC;
    // buffer selection by select (no dynamically indexed private arrays -> no scratch)
    __device__ uint32_t *keys(int i) const { return i ? K[1] : K[0]; }
    __device__ int16_t *nodes_of(int i) const { return i ? NO[1] : NO[0]; }
};

// S1: quadrant prefix of every live key in buffer order; segment start / end prefixes per
// node. Thread tid owns the contiguous key run [tid*R, tid*R + R). Returns the run's base.
__device__ QCnt qt_prefix(QShared &S, QT &Q, int &par) {
    const int R = (Q.M + ORBX_QT_THREADS - 1) / ORBX_QT_THREADS;
    const int i0 = threadIdx.x * R, i1 = min(i0 + R, Q.M);
    const uint32_t *K = Q.keys(Q.src);
    const int16_t *NO = Q.nodes_of(Q.src);
    // a node's keys are contiguous: its midpoint is fetched once per run of keys (the node
    // arrays sit in global scratch, so every fetch is a dependent L2 round trip)
    QCnt run{0ull, 0ull};
    int last = -1, mx = 0, my = 0;
    for (int i = i0; i < i1; i++) {
        const int nd = NO[i];
        if (nd < 0) continue;
        if (nd != last) { qnode_mid(Q.cur[nd], &mx, &my); last = nd; }
        run += qone(quadrant(K[i], mx, my));
    }
    QCnt tot;
    const QCnt base = block_scan(S, run, &tot, par);
    QCnt p = base;
    last = -1;
    for (int i = i0; i < i1; i++) {
        const int nd = NO[i];
        if (nd < 0) continue;
        if (nd != last) { qnode_mid(Q.cur[nd], &mx, &my); last = nd; }
        if (i == 0 || NO[i - 1] != nd) Q.tmp[nd].pstart = p;
        p += qone(quadrant(K[i], mx, my));
        if (i == Q.M - 1 || NO[i + 1] != nd) Q.tmp[nd].pend = p;
    }
    __syncthreads();
    return base;
}

// S3: one split round over `na` live nodes in processing order (order: 0 ascending,
// 1 descending, 2 Q.sortbuf); nodes at positions >= limit are kept undivided (final phase).
// Children get consecutive ids in processing order and n1..n4 order; multi-key children
// (then kept nodes) form the next array in that order, single-key children become leaves.
__device__ void qt_assign(QShared &S, QT &Q, int na, int order, int limit, int &par) {
    const int Rn = (na + ORBX_QT_THREADS - 1) / ORBX_QT_THREADS;
    const int t0 = threadIdx.x * Rn, t1 = min(t0 + Rn, na);
    auto node_at = [&](int t) { return order == 2 ? (int)(Q.sortbuf[t] & 0xFFFF) : order == 1 ? na - 1 - t : t; };
    unsigned long long run = 0;
    for (int t = t0; t < t1 && t < limit; t++) {
        const QTmp &T = Q.tmp[node_at(t)];
        const QCnt c = T.pend - T.pstart;
        int ne = 0, mu = 0, si = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) { const int ck = c.f(k); ne += ck > 0; mu += ck > 1; si += ck == 1; }
        run += (unsigned long long)ne | (unsigned long long)mu << 16 | (unsigned long long)si << 32;
    }
    unsigned long long tot;
    const unsigned long long pre = block_scan64(S, run, &tot, par);
    const int tot_ne = (int)(tot & 0xFFFF), tot_mu = (int)((tot >> 16) & 0xFFFF), tot_si = (int)(tot >> 32);
    int id = S.next_id + (int)(pre & 0xFFFF);
    int m = S.n_next + (int)((pre >> 16) & 0xFFFF);
    int o = S.n_out + (int)(pre >> 32);
    for (int t = t0; t < t1; t++) {
        const int nd = node_at(t);
        QTmp &T = Q.tmp[nd];
        if (t >= limit) {
            const int km = S.n_next + tot_mu + (t - limit);
            T.keep = km < Q.NC ? km : -1;   // (never exceeds NC: the list stays below N + 4)
            if (km < Q.NC) Q.nxt[km] = Q.cur[nd];
            continue;
        }
        T.keep = -1;
        const QNode q = Q.cur[nd];
        const QCnt c = T.pend - T.pstart;
        int mx, my;
        qnode_mid(q, &mx, &my);
        int cs = q.s;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int ck = c.f(k);
            int16_t cmk = 0;
            if (ck > 0) {
                const int cid = id++;
                if (ck > 1) {
                    QNode ch;
                    ch.x0 = (k & 1) ? (int16_t)mx : q.x0;
                    ch.x1 = (k & 1) ? q.x1 : (int16_t)mx;
                    ch.y0 = (k & 2) ? (int16_t)my : q.y0;
                    ch.y1 = (k & 2) ? q.y1 : (int16_t)my;
                    ch.s = cs;
                    ch.n = ck;
                    ch.id = cid;
                    if (m < Q.NC) Q.nxt[m] = ch;
                    cmk = (int16_t)(m < Q.NC ? m : -32768);
                    m++;
                } else {
                    if (o < Q.NP) Q.outrec[o] = (unsigned long long)(uint32_t)(cid + 0x40000000) << 32;
                    cmk = (int16_t)(o < Q.NP ? -1 - o : -32768);
                    o++;
                }
            }
            T.cm[k] = cmk;
            cs += ck;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int ndiv = min(limit, na);
        S.next_id += tot_ne;
        S.n_out += tot_si;
        S.live += tot_ne - ndiv;
        S.n_act = min(S.n_next + tot_mu + (na - ndiv), Q.NC);
    }
}

// S4: move every live key to its child's segment in the other buffer (stable), record its
// next-round node; leaves receive their key.
__device__ void qt_move(QShared &S, QT &Q, QCnt base) {
    const int R = (Q.M + ORBX_QT_THREADS - 1) / ORBX_QT_THREADS;
    const int i0 = threadIdx.x * R, i1 = min(i0 + R, Q.M);
    const int s = Q.src, d = s ^ 1;
    const uint32_t *Ks = Q.keys(s);
    const int16_t *Ns = Q.nodes_of(s);
    uint32_t *Kd = Q.keys(d);
    int16_t *Nd = Q.nodes_of(d);
    QCnt p = base;
    int last = -1, mx = 0, my = 0, qs = 0;
    QTmp T{};
    for (int i = i0; i < i1; i++) {
        const int nd = Ns[i];
        if (nd < 0) { Nd[i] = -1; continue; }
        const uint32_t key = Ks[i];
        if (nd != last) {   // once per run of the node's keys (see qt_prefix)
            const QNode q = Q.cur[nd];
            qnode_mid(q, &mx, &my);
            qs = q.s;
            T = Q.tmp[nd];
            last = nd;
        }
        const int k = quadrant(key, mx, my);
        if (T.keep >= 0) {
            Kd[i] = key;
            Nd[i] = (int16_t)T.keep;
        } else {
            const QCnt c = T.pend - T.pstart;
            int pos = qs + (p - T.pstart).f(k);
            for (int j = 0; j < k; j++) pos += c.f(j);
            Kd[pos] = key;
            const int cmk = k < 2 ? (k ? T.cm[1] : T.cm[0]) : (k == 3 ? T.cm[3] : T.cm[2]);   // no private indexing
            if (cmk >= 0) {
                Nd[pos] = (int16_t)cmk;
            } else {
                Nd[pos] = -1;
                if (cmk != -32768) Q.outrec[-1 - cmk] |= key;
            }
        }
        p += qone(k);
    }
    __syncthreads();
    if (threadIdx.x == 0) S.n_next = 0;
    Q.src = d;
    QNode *t = Q.cur; Q.cur = Q.nxt; Q.nxt = t;
    __syncthreads();
}

// NL: the node arrays in LDS (ORBX_QT_NODES_LDS) or in global scratch, a template argument so every
// node access compiles to one address space (a pointer chosen at run time between LDS and global
// compiles to flat loads and stores, which wait on both counters)
template <bool NL>
__global__ __launch_bounds__(ORBX_QT_THREADS) void quadtree_kernel(
    ExtractGeom g, const int *cell_cnt, const uint32_t *cell_keys, uint32_t *qt_keys,
    unsigned char *qt_nodes, uint32_t *sel, int *sel_cnt) {
    extern __shared__ __align__(16) unsigned char qt_lds[];
    __shared__ QShared S;
    // grid (images, levels) in hardware order: every image's level 0 -- the longest workgroups --
    // is dispatched first, then level 1, ... (longest first shortens the kernel's tail); the
    // workgroups share no data, so no XCD-aware remap
    const int b = blockIdx.x, l = blockIdx.y;
    const int tid = threadIdx.x;
#ifdef ORBX_QT_PROFILE
    long long qt_t[8], qt_sub[3] = {0, 0, 0};
    int qt_rounds = 0;
    qt_t[0] = wall_clock64();
#define QT_MARK(k) do { if (tid == 0) qt_t[k] = wall_clock64(); } while (0)
#else
#define QT_MARK(k) do {} while (0)
#endif
    const int cb0 = g.cell_base[l], ncell = g.cell_base[l + 1] - cb0;
    const int N = g.N[l], nIni = g.nIni[l];
    const int NC = g.node_cap, NP = g.node_pow2;
    int par = 0;
    // ---- LDS / global carving
    unsigned char *lds = qt_lds;
    unsigned char *const nodes = NL ? lds : qt_nodes + ((long long)b * g.nlevels + l) * g.qt_node_stride * 4;
    if (NL) lds += 16 * NP + (sizeof(QTmp) + 2 * sizeof(QNode)) * NC;
    // ---- 1. gather the cells' keypoints in cell order -> M. A cell's slots hold its FAST
    //         survivors at min(iniThFAST, minThFAST) with score M - 1; FAST at iniThFAST keeps
    //         those with score >= iniThFAST, and the cell retries at minThFAST when none does
    //         (:1119-1135). The order inside a cell is restated in step 5.
    const int *cnt = cell_cnt + (long long)b * g.ncell_total + cb0;
    const int th_a = min(max(g.ini_th, 0), 255), th_b = min(max(g.min_th, 0), 255);
    // A thread owns cells c0 + tid; its cell's slot row (cell_cap is a multiple of 4) is read 16
    // keys per batch of four uint4 loads in flight: the count pass keeps, per owned cell, the
    // kept count and threshold in registers (up to QG_IT cells per thread) for the copy pass.
    constexpr int QG_IT = 4;
    auto cell_keys4 = [&](int c) {
        return (const uint4 *)(cell_keys + ((long long)b * g.ncell_total + cb0 + c) * g.cell_cap);
    };
    auto cell_take = [&](int c, int *th) {   // keypoints of cell c, threshold in *th
        const uint4 *src = cell_keys4(c);
        const int v = min(cnt[c], g.cell_cap);
        int na = 0, nb = 0;
        for (int i = 0; i < v; i += 16) {
            uint4 q[4];
#pragma unroll
            for (int u = 0; u < 4; u++) q[u] = i + 4 * u < v ? src[(i >> 2) + u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t kk[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const bool in = i + 4 * u + e < v;
                    const int sc = key_score(kk[e]);
                    na += in && sc >= th_a;
                    nb += in && sc >= th_b;
                }
            }
        }
        *th = na > 0 ? th_a : th_b;
        return na > 0 ? na : nb;
    };
    int kept_r[QG_IT], th_r[QG_IT];
    int M = 0;
    {
        int it = 0;
        for (int c0 = 0; c0 < ncell; c0 += ORBX_QT_THREADS, it++) {
            const int c = c0 + tid;
            int th = 0;
            const int v = c < ncell ? cell_take(c, &th) : 0;
#pragma unroll
            for (int k = 0; k < QG_IT; k++) if (k == it) { kept_r[k] = v; th_r[k] = th; }
            unsigned long long tot;
            block_scan64(S, (unsigned)v, &tot, par);
            M += (int)tot;
        }
    }
#ifdef ORBX_QT_PROFILE
    const long long t_gm = wall_clock64();
#endif
    // the rest in two copies, keys in LDS (KL) or in global scratch: each key access one address space
    // (the working set is a local of each copy)
    auto body = [&](auto kl_tag) {
    constexpr bool KL = decltype(kl_tag)::value;
    QT Q;
    Q.NC = NC; Q.NP = NP; Q.M = M;
    {
        unsigned char *p = nodes;
        Q.outrec = (unsigned long long *)p; p += 8 * NP;
        Q.sortbuf = (unsigned long long *)p; p += 8 * NP;
        Q.tmp = (QTmp *)p; p += sizeof(QTmp) * NC;
        Q.cur = (QNode *)p; p += sizeof(QNode) * NC;
        Q.nxt = (QNode *)p;
    }
    if (KL) {
        Q.K[0] = (uint32_t *)lds;
        Q.K[1] = Q.K[0] + g.qt_kl;
        Q.NO[0] = (int16_t *)(Q.K[1] + g.qt_kl);
        Q.NO[1] = Q.NO[0] + g.qt_kl;
    } else {
        uint32_t *gk = qt_keys + (long long)b * g.qt_off[g.nlevels] + g.qt_off[l];
        const long long cap = (g.qt_off[l + 1] - g.qt_off[l]) / 3;
        Q.K[0] = gk;
        Q.K[1] = gk + cap;
        Q.NO[0] = (int16_t *)(gk + 2 * cap);
        Q.NO[1] = Q.NO[0] + cap;
    }
    {
        int base = 0, it = 0;
        for (int c0 = 0; c0 < ncell; c0 += ORBX_QT_THREADS, it++) {
            const int c = c0 + tid;
            int th = 0, v = 0;
            if (it < QG_IT) {
#pragma unroll
                for (int k = 0; k < QG_IT; k++) if (k == it) { v = kept_r[k]; th = th_r[k]; }
            } else if (c < ncell) {
                v = cell_take(c, &th);
            }
            unsigned long long tot;
            const int pre = (int)block_scan64(S, (unsigned)v, &tot, par);
            if (v > 0) {
                const uint4 *src = cell_keys4(c);
                const int nv = min(cnt[c], g.cell_cap);
                uint32_t *dk = Q.K[0] + base + pre;
                int o = 0;
                for (int i = 0; i < nv; i += 16) {
                    uint4 q[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) q[u] = i + 4 * u < nv ? src[(i >> 2) + u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t kk[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
                        for (int e = 0; e < 4; e++)
                            if (i + 4 * u + e < nv && key_score(kk[e]) >= th) dk[o++] = kk[e];
                    }
                }
            }
            base += (int)tot;
        }
    }
    QT_MARK(1);
    // ---- 2. roots (:700-745): stable counting partition into buffer 1
    const float hX = g.hX[l];
    if (tid < 64) { S.root_cnt[tid] = 0; S.root_fill[tid] = 0; }
    __syncthreads();
    for (int i = tid; i < M; i += ORBX_QT_THREADS) {
        const int r = min((int)((float)key_x(Q.K[0][i]) / hX), nIni - 1);
        atomicAdd(&S.root_cnt[r], 1);
    }
    __syncthreads();
    if (tid == 0) {
        const int H = g.maxBY[l] - 16;
        int a = 0, na = 0, no = 0, live = 0;
        for (int r = 0; r < nIni; r++) {
            const int n = S.root_cnt[r];
            S.root_start[r] = a;
            S.root_node[r] = -1;
            S.root_out[r] = -1;
            a += n;
            if (n == 0) continue;
            live++;
            if (n == 1) {
                S.root_out[r] = no++;
            } else {
                QNode q;
                q.x0 = (int16_t)(int)(hX * (float)r);
                q.x1 = (int16_t)(int)(hX * (float)(r + 1));
                q.y0 = 0;
                q.y1 = (int16_t)H;
                q.s = S.root_start[r];
                q.n = n;
                q.id = -1 - r;
                S.root_node[r] = na;
                Q.cur[na++] = q;
            }
        }
        S.live = live; S.n_out = no; S.n_act = na; S.next_id = nIni; S.n_next = 0;
    }
    __syncthreads();
    const int lane = tid & 63, wv = tid >> 6;
    for (int cs = 0; cs < M; cs += ORBX_QT_THREADS) {
        const int i = cs + tid;
        int r = -1;
        uint32_t key = 0;
        if (i < M) { key = Q.K[0][i]; r = min((int)((float)key_x(key) / hX), nIni - 1); }
        int my_rank = 0;
        for (int rr = 0; rr < nIni; rr++) {
            const unsigned long long m = __ballot(r == rr);
            if (r == rr) my_rank = __popcll(m & ((1ull << lane) - 1ull));
            if (lane == 0) S.wcnt[wv][rr] = __popcll(m);
        }
        __syncthreads();
        if (r >= 0) {
            int pos = S.root_start[r] + S.root_fill[r] + my_rank;
            for (int w = 0; w < wv; w++) pos += S.wcnt[w][r];
            Q.K[1][pos] = key;
            Q.NO[1][pos] = (int16_t)S.root_node[r];
            if (S.root_out[r] >= 0) Q.outrec[S.root_out[r]] = ((unsigned long long)(uint32_t)(-1 - r + 0x40000000) << 32) | key;
        }
        __syncthreads();
        if (tid < nIni) {
            int add = 0;
            for (int w = 0; w < ORBX_QT_THREADS / 64; w++) add += S.wcnt[w][tid];
            S.root_fill[tid] += add;
        }
        __syncthreads();
    }
    Q.src = 1;
    QT_MARK(2);
    // ---- 3. phase-1 rounds (:772-913): every live node divided, roots ascending, then
    //         the previous round's multi-key children in reverse creation order
    int order = 0;
    bool finished = false, final_phase = false;
    while (!finished) {
        const int prev = S.live, na = S.n_act;
#ifdef ORBX_QT_PROFILE
        const long long ta = wall_clock64();
#endif
        const QCnt base = qt_prefix(S, Q, par);
#ifdef ORBX_QT_PROFILE
        const long long tb = wall_clock64();
#endif
        qt_assign(S, Q, na, order, na, par);
#ifdef ORBX_QT_PROFILE
        const long long tc = wall_clock64();
#endif
        qt_move(S, Q, base);
        order = 1;
#ifdef ORBX_QT_PROFILE
        qt_rounds++;
        const long long td = wall_clock64();
        qt_sub[0] += tb - ta; qt_sub[1] += tc - tb; qt_sub[2] += td - tc;
#endif
        const int live = S.live, nToExpand = S.n_act;
        if (live >= N || live == prev) finished = true;
        else if (live + nToExpand * 3 > N) { final_phase = true; finished = true; }
    }
    QT_MARK(3);
    // ---- 4. final phase (:914-997): nodes by (size, id) descending; divide until the
    //         list reaches N
    if (final_phase) {
        bool done = false;
        while (!done) {
            const int prev = S.live, na = S.n_act;
            const QCnt base = qt_prefix(S, Q, par);
            // distinct keys (n, id, position): rank-sorted from an LDS stage -- the other key
            // buffer, free until qt_move, or the whole key area when the keys live in global
            // scratch -- into sortbuf; the bitonic network over sortbuf when neither fits
            const int na16 = (na + 15) & ~15;
            const bool keys_lds = KL;
            const bool rank = na16 <= (keys_lds ? g.qt_kl / 2 : 12 * g.qt_kl / 8);
            // (each branch with its own pointer: one address space per access)
            unsigned long long *const rstage = keys_lds ? (unsigned long long *)Q.keys(Q.src ^ 1) : (unsigned long long *)lds;
            int np2 = 1;
            while (np2 < na) np2 <<= 1;
            auto fill = [&](unsigned long long *stage, int nfill) {
                for (int i = tid; i < nfill; i += ORBX_QT_THREADS) {
                    unsigned long long v = 0;
                    if (i < na) {
                        const QNode &q = Q.cur[i];
                        v = ((unsigned long long)(uint32_t)q.n << 40) | ((unsigned long long)(uint32_t)(q.id & 0xFFFFFF) << 16) | (unsigned)i;
                    }
                    stage[i] = v;
                }
            };
            if (rank) fill(rstage, na16);
            else fill(Q.sortbuf, np2);
            if (tid == 0) S.cross = na;
            __syncthreads();
            if (rank) block_rank_sort_desc(rstage, Q.sortbuf, na);
            else block_sort_desc(Q.sortbuf, np2);
            // first sorted position whose split brings the size to >= N
            {
                const int Rn = (na + ORBX_QT_THREADS - 1) / ORBX_QT_THREADS;
                const int t0 = tid * Rn, t1 = min(t0 + Rn, na);
                int run = 0;
                for (int t = t0; t < t1; t++) {
                    const QTmp &T = Q.tmp[Q.sortbuf[t] & 0xFFFF];
                    const QCnt c = T.pend - T.pstart;
                    run += (c.f(0) > 0) + (c.f(1) > 0) + (c.f(2) > 0) + (c.f(3) > 0) - 1;
                }
                unsigned long long tot;
                int acc = S.live + (int)block_scan64(S, (unsigned long long)(long long)run, &tot, par);
                for (int t = t0; t < t1; t++) {
                    const QTmp &T = Q.tmp[Q.sortbuf[t] & 0xFFFF];
                    const QCnt c = T.pend - T.pstart;
                    acc += (c.f(0) > 0) + (c.f(1) > 0) + (c.f(2) > 0) + (c.f(3) > 0) - 1;
                    if (acc >= N) { atomicMin(&S.cross, t); break; }
                }
            }
            __syncthreads();
            const int limit = min(S.cross + 1, na);
            qt_assign(S, Q, na, 2, limit, par);
            qt_move(S, Q, base);
#ifdef ORBX_QT_PROFILE
            qt_rounds += 100;
#endif
            if (S.live >= N || S.live == prev) done = true;
        }
    }
    QT_MARK(4);
    // ---- 5. every remaining multi-key node -> its first key of maximal response (:1028) in
    //         the reference list order: cells row-major (:1084-1093), then cv::FAST's row-major
    //         order inside the cell; rank = (cell, row, column in the cell), from the key
    {
        const int na = S.n_act;
        // each node's best key as a u64 maximum: in LDS (the idle key buffer) when it fits, else in
        // the node scratch; two copies so each access has one address space
        auto step5 = [&](unsigned long long *best) {
        const int R = (M + ORBX_QT_THREADS - 1) / ORBX_QT_THREADS;
        const int i0 = tid * R, i1 = min(i0 + R, M);
        const int hC = g.hcell[l], wC = g.wcell[l];
        for (int i = tid; i < na; i += ORBX_QT_THREADS) best[i] = 0ull;
        __syncthreads();
        for (int i = i0; i < i1; i++) {
            const int nd = Q.nodes_of(Q.src)[i];
            if (nd >= 0) {
                const uint32_t key = Q.keys(Q.src)[i];
                const int ry = key_y(key) - 3, rx = key_x(key) - 3;   // from the first detection row / column
                const int ci = (int)(((unsigned)ry * (unsigned)g.hcell_mag[l]) >> 20);
                const int cj = (int)(((unsigned)rx * (unsigned)g.wcell_mag[l]) >> 20);
                const uint32_t rank = ((uint32_t)(ci * g.ncell_cols[l] + cj) << 12) | ((uint32_t)(ry - ci * hC) << 6) |
                                      (uint32_t)(rx - cj * wC);
                atomicMax(&best[nd], ((unsigned long long)key_score(key) << 56) |
                                         ((unsigned long long)(0xFFFFFFFFu - rank) << 24) | (unsigned)i);
            }
        }
        __syncthreads();
        for (int t = tid; t < na; t += ORBX_QT_THREADS) {
            const int o = S.n_out + t;
            if (o < NP) {
                const uint32_t key = Q.keys(Q.src)[best[t] & 0xFFFFFF];
                Q.outrec[o] = ((unsigned long long)(uint32_t)(Q.cur[t].id + 0x40000000) << 32) | key;
            }
        }
        };
        if (KL && 2 * na <= g.qt_kl) step5((unsigned long long *)Q.keys(Q.src ^ 1));
        else step5(Q.sortbuf);
        __syncthreads();
        if (tid == 0) S.n_out += na;
        __syncthreads();
    }
    QT_MARK(5);
    const int nout = min(S.n_out, NP);
    if (12 * g.qt_kl >= 8 * ((nout + 15) & ~15)) {
        // the output records are distinct (one per key): stage them in the key area of LDS,
        // free after step 5, and rank-sort them back into outrec
        unsigned long long *stage = (unsigned long long *)lds;
        for (int i = tid; i < ((nout + 15) & ~15); i += ORBX_QT_THREADS) stage[i] = i < nout ? Q.outrec[i] : 0ull;
        __syncthreads();
        block_rank_sort_desc(stage, Q.outrec, nout);
    } else {
        for (int i = nout + tid; i < NP; i += ORBX_QT_THREADS) Q.outrec[i] = 0;
        __syncthreads();
        block_sort_desc(Q.outrec, NP);
    }
    QT_MARK(6);
    const int ncap = min(nout, g.out_cap[l]);
    uint32_t *dst = sel + (long long)b * g.out_base[g.nlevels] + g.out_base[l];
    for (int i = tid; i < ncap; i += ORBX_QT_THREADS) dst[i] = (uint32_t)(Q.outrec[i] & 0xFFFFFFFFull);
    if (tid == 0) sel_cnt[b * g.nlevels + l] = ncap;
#ifdef ORBX_QT_PROFILE
    if (tid == 0 && (b < 2 || (b & 31) == 0))
        printf("QTPROF b=%d l=%d M=%d NP=%d nout=%d rounds=%d start=%lld end=%lld gather=%lld roots=%lld ph1=%lld final=%lld best=%lld sort=%lld prefix=%lld assign=%lld move=%lld gatherM=%lld\n", b, l, M,
               NP, nout, qt_rounds, qt_t[0], wall_clock64(), qt_t[1] - qt_t[0], qt_t[2] - qt_t[1], qt_t[3] - qt_t[2], qt_t[4] - qt_t[3],
               qt_t[5] - qt_t[4], qt_t[6] - qt_t[5], qt_sub[0], qt_sub[1], qt_sub[2], t_gm - qt_t[0]);
#endif
    };
    if (M <= g.qt_kl) body(std::true_type{});
    else body(std::false_type{});
}

// ------------------------------------------------------------------------------------
// exact integer wavefront sum on DPP (quad perms, half-row / row mirrors, row broadcasts
// 15 / 31), result read from lane 63 -- no LDS traffic
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}

// K5: IC_Angle (:94-141) + computeOrbDescriptor (:153-204) + keypoint assembly (:1603-1657), NS = 8
// output slots per wavefront (3 per wavefront with a dependent global round trip per slot before:
// 444 -> 340 us per 128 pairs alone):
//  1. the NS slots are resolved lane-parallel (lane r = slot s0 + r: level, output row, key,
//     IC_Angle row base, blurred-patch base) in one round trip;
//  2. the IC_Angle rows of all NS slots and the steered-BRIEF patches of the first G slots are
//     issued together (second round trip); the moments (v_dot4 + DPP wave sums) land in lane r;
//  3. fastAtan2 + glibc sincosf run once for all NS slots (lanes 0..NS-1);
//  4. G slots at a time: the group's patch registers go to LDS, the next group's patch loads are
//     issued, and the 256 tests of each slot run from LDS; the ballot words collect in lanes
//     4r + w;
//  5. one store per lane: descriptor word w of slot r by lane 4r + w, keypoint r by lane r.
// v_writelane_b32: lane `r` of `old` := the wave-uniform `v`. The s_nop covers the hazard of a
// VALU write of the SGPR source (a v_cmp's VCC) right before: without it the writelane read the
// previous VCC on MI355X (tools/dbg/desc_diff.py: word 3 of every descriptor carried word 2's low half)
__device__ __forceinline__ int write_lane(int v, int r, int old) {
    asm volatile("s_nop 3\n\tv_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(v), "i"(r));
    return old;
}

// Loads: only the patch / IC_Angle dwords a keypoint can read (c_pmask, c_icw: 370 -> 308-310 patch
// and 248 -> 208 IC_Angle dwords per slot, C2 +0.65 %). Measured and not kept: 4, 6 or
// 12 slots per wavefront, groups of 4, prefetch distance 2-4 (1-4 % slower, more VGPRs); 16-byte
// loads (the texture pipeline stays as busy, no faster).
constexpr int kDescNS = 8;   // slots per wavefront (the moment butterfly holds 8)
__global__ __launch_bounds__(256) void describe2_kernel(ExtractGeom g, const uint8_t *in, const uint8_t *pyr,
                                                        const uint8_t *blur, const uint32_t *sel, const int *sel_cnt,
                                                        orbx_kp *kps, uint8_t *desc, int *cnt) {
    constexpr int NS = kDescNS, G = 2, NB = 2, PRE = 1;   // slots, group size, patch buffers, groups issued early
    static_assert(NS % G == 0 && NS <= 8, "slot groups; the moment butterfly holds 8 slots");
    constexpr int NG = NS / G;
    const int lane = threadIdx.x & 63, wv = wave_id();
    int bxr, b;
    xcd_remap2(bxr, b);
    constexpr int PW = 10;   // patch row stride in dwords (LDS)
    constexpr int PSZ = 372;
    __shared__ __align__(16) uint32_t patch[4][G][PSZ];
    const int L = g.nlevels, cap = g.out_base[L];   // L <= ORBX_MAXL = 16: one DPP row
    const int s0 = (bxr * 4 + wv) * NS;
    // IC_Angle byte weights of the lane's four rows (the same for every slot): issued first, with
    // the slot loads, instead of after each slot's rows
    const int w8 = lane & 7, vr = lane >> 3;
    const DescLane dl = c_dlane[lane];
    uint2 wt[4];
#pragma unroll
    for (int k = 0; k < 4; k++) wt[k] = dl.wt[k];
    const uint32_t pmask = dl.pmask;
    // 1. lane k < L: selected keypoints of level k; lane r < NS: slot s0 + r
    const int scl = lane < L ? sel_cnt[(long long)b * L + lane] : 0;
    const int slot = s0 + lane;
    const bool inr = lane < NS && slot < cap;
    const uint32_t key = inr ? sel[(long long)b * cap + slot] : 0u;
    int inc = scl;   // inclusive level prefix on row 0
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x111, 0xF, 0xF, false);   // row_shr:1
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x112, 0xF, 0xF, false);   // row_shr:2
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x114, 0xF, 0xF, false);   // row_shr:4
    inc += __builtin_amdgcn_update_dpp(0, inc, 0x118, 0xF, 0xF, false);   // row_shr:8
    if (s0 == 0) {
        const int tot = __builtin_amdgcn_readlane(inc, L - 1);
        if (lane == 0) cnt[b] = tot;
    }
    // level of the slot = the last k with out_base[k] <= slot (out_base is increasing)
    int l = 0, lbase = 0;
#pragma unroll
    for (int k = 1; k < ORBX_MAXL; k++)
        if (k < L && slot >= g.out_base[k]) { l = k; lbase = g.out_base[k]; }
    const int idx = slot - lbase;
    const int nl = __shfl(scl, l), incl = __shfl(inc, l);
    const bool valid = inr && idx < nl;
    const unsigned long long vmask = __ballot(valid);
    if (vmask == 0) return;
    const int off = incl - nl + idx;
    const int kx = key_x(key) + 16, ky = key_y(key) + 16;   // + minBorderX/Y (:1177-1186)
    const uint8_t *img = l == 0 ? in + (long long)b * g.in_stride : pyr + (long long)b * g.pyr_stride + g.pyr_off[l];
    const int pitch = l == 0 ? g.in_pitch : g.bp[l];
    const unsigned long long icb = (unsigned long long)(img + (long long)(ky - 15) * pitch + kx - 16);
    // Every descriptor below carries the exact byte count from its base to the end of its level's
    // last row, so the hardware range check zeroes anything past the level -- for level 0 that is the
    // caller's image, which has no readable tail (include/orbslam2_amd.h). No load reaches there: a
    // keypoint lies in the detection region [19, w - 19) x [19, h - 19) (fast_blur_kernel), the
    // IC_Angle rows read columns kx - 16 .. kx + 15 <= w - 5 of rows ky - 15 .. ky + 15 <= h - 5 and
    // the blurred patch columns <= kx + 21 <= w + 1 of rows <= ky + 18 <= h - 2 (a row that is not the
    // level's last, so a byte past its width is the next row's). Loads that add a row step in
    // soffset are covered by that argument, not by the range check.
    const int icn = (int)((long long)(l == 0 ? g.in_pitch : g.bp[l]) * (g.lh[l] - (ky - 15) - 1) + g.lw[l] - (kx - 16));
    const int bw = g.bbp[l];
    const long long c0 = (long long)b * g.blur_stride + g.blur_off[l] + (long long)(ky - 18) * bw + (kx - 18);
    const int psh = (int)(c0 & 3);
    const long long a0 = c0 - psh;
    const int bln = (int)(((long long)bw * (g.lh[l] - (ky - 18) - 1) + g.lw[l] - (kx - 18) + psh + 3) & ~3LL);
    const long long amax = (long long)g.nimg * g.blur_stride - 4;
    const unsigned long long smask = __ballot(valid && a0 >= 0 && a0 + 36LL * bw + 4 * PW <= amax + 4);
    auto rl64 = [](unsigned long long v, int r) {
        return (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, r) |
               (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), r) << 32;
    };
    // 2. IC_Angle rows of every slot: lane -> dword w = lane % 8 of rows v0, v0 + 8, v0 + 16,
    // v0 + 24 (v0 = lane / 8 - 15), unaligned dword loads
    // (buffer loads: the slot's row base in the descriptor, rows 8k apart in soffset, the lane's
    // row / dword in voffset -- no 64-bit address arithmetic per load)
    uint32_t P[NS][4];
#pragma unroll
    for (int r = 0; r < NS; r++) {
#pragma unroll
        for (int k = 0; k < 4; k++) P[r][k] = 0u;
        if (!((vmask >> r) & 1)) continue;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)rl64(icb, r), 0, __builtin_amdgcn_readlane(icn, r), 0x00020000);
        const int pr = __builtin_amdgcn_readlane(pitch, r);
        // 24-bit multiply-add: a plain int multiply-add became v_mad_u64_u32 with an undefined high
        // addend register that aliased a load destination of the previous slot, so every slot waited
        // vmcnt(0) for the previous one's rows
        const int vo = (int)__umul24((unsigned)vr, (unsigned)pr) + 4 * w8;
#pragma unroll
        for (int k = 0; k < 4; k++)   // a dword with no pixel inside the umax circle has weight 0
            if ((k < 3 || vr <= 6) && wt[k].y != 0u) P[r][k] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 8 * k * pr, 0);
    }
    // steered-BRIEF patch of slot r (rows y-18 .. y+18, bytes x-18 .. x+21 as 10 aligned dwords
    // per row; lanes 0..59 -> (row lane / 10, dword lane % 10), six rows per pass) into registers
    const int rr0 = (lane * 205) >> 11, q10 = lane - 10 * rr0;
    constexpr int TK = 7;   // patch registers per slot and lane
    uint32_t T[NB][G][TK];   // NB groups' patches in flight (prefetch distance NB)
    auto issue_patch = [&](int gi, uint32_t (&dst)[G][TK]) {
#pragma unroll
        for (int j = 0; j < G; j++) {
            const int r = gi * G + j;
#pragma unroll
            for (int k = 0; k < TK; k++) dst[j][k] = 0u;
            if (!((smask >> r) & 1)) continue;
            const int bwr = __builtin_amdgcn_readlane(bw, r);
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void *)(blur + (long long)rl64((unsigned long long)a0, r)), 0,
                                                  __builtin_amdgcn_readlane(bln, r), 0x00020000);
            const int vo = (int)__umul24((unsigned)rr0, (unsigned)bwr) + 4 * q10;
            const uint32_t pm = pmask >> (7 * __builtin_amdgcn_readlane(psh, r));
            if (lane < 60) {
#pragma unroll
                for (int k = 0; k < 7; k++)
                    if ((k < 6 || rr0 == 0) && ((pm >> k) & 1u)) dst[j][k] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 6 * k * bwr, 0);
            }
        }
    };
    // PRE groups issued with the IC rows, the rest of the NB once P is consumed
#pragma unroll
    for (int q = 0; q < PRE && q < NG; q++) issue_patch(q, T[q]);
    // moments: the lane's partial sums of every slot (x[r] = m10, x[8 + r] = m01; exact integers),
    // then one butterfly reduction of the 16 values over the wavefront. Each DPP pairing inside a
    // row halves the values a lane holds; partners always hold the same value indices: the row
    // mirror (lanes i, 15 - i, split by bit 3) while every lane still holds all 16, then the
    // half-row mirror (i, 7 - i: same bit 3, split by bit 2), lane ^ 2 and lane ^ 1, so lane j of
    // every row ends with value j & 15 summed over its row; two cross-row xor shuffles finish the
    // sums. Lane r < 8 then holds m10 of slot r, lane 8 + r its m01.
    int x[16];
#pragma unroll
    for (int r = 0; r < 8; r++) {
        int m01 = 0, m10 = 0;
        if (r < NS && ((vmask >> r) & 1)) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int v = vr - 15 + 8 * k;
                if (k < 3 || vr <= 6) {
                    const int su = (int)__builtin_amdgcn_udot4(P[r < NS ? r : 0][k], wt[k].x, 0u, false);
                    const int sm = (int)__builtin_amdgcn_udot4(P[r < NS ? r : 0][k], wt[k].y, 0u, false);
                    m10 += su - 16 * sm;
                    m01 += v * sm;
                }
            }
        }
        x[r] = m10;
        x[8 + r] = m01;
    }
    int msum;
    {
        int y[8], z[4], u[2];
        const bool b0 = lane & 1, b1 = (lane >> 1) & 1, b2 = (lane >> 2) & 1, b3 = (lane >> 3) & 1;
#pragma unroll
        for (int m = 0; m < 8; m++)   // row mirror: keep x[8 b3 + m]
            y[m] = (b3 ? x[8 + m] : x[m]) + __builtin_amdgcn_update_dpp(0, b3 ? x[m] : x[8 + m], 0x140, 0xF, 0xF, false);
#pragma unroll
        for (int m = 0; m < 4; m++)   // half-row mirror: keep y[4 b2 + m]
            z[m] = (b2 ? y[4 + m] : y[m]) + __builtin_amdgcn_update_dpp(0, b2 ? y[m] : y[4 + m], 0x141, 0xF, 0xF, false);
#pragma unroll
        for (int m = 0; m < 2; m++)   // lane ^ 2: keep z[2 b1 + m]
            u[m] = (b1 ? z[2 + m] : z[m]) + __builtin_amdgcn_update_dpp(0, b1 ? z[m] : z[2 + m], 0x4E, 0xF, 0xF, false);
        msum = (b0 ? u[1] : u[0]) + __builtin_amdgcn_update_dpp(0, b0 ? u[0] : u[1], 0xB1, 0xF, 0xF, false);
        msum += __shfl_xor(msum, 16);
        msum += __shfl_xor(msum, 32);
    }
    const int m10v = msum;
    const int m01v = __builtin_amdgcn_update_dpp(0, msum, 0x108, 0xF, 0xF, false);   // row_shl:8: lane r <- lane r + 8
#pragma unroll
    for (int q = PRE; q < NB && q < NG; q++) issue_patch(q, T[q]);
    // 3. angle = fastAtan2(m01, m10) and (float) cos / sin of every slot, lane r
    const float ang = fast_atan2_deg((float)m01v, (float)m10v);
    float sa, ca;
    glibc_sincosf(ang * (float)(3.1415926535897932384626433832795 / 180.f), &sa, &ca);
    // pattern coordinates of the lane's 4 test pairs as floats (int8 -> f32, exact), the two
    // points of a pair packed for v_pk_mul_f32 / v_pk_add_f32
    f32x2 PX[4], PY[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t pw = ((const uint32_t *)c_pattern)[w * 64 + lane];   // x0 y0 x1 y1 as int8
        PX[w] = f32x2{(float)(int8_t)(pw & 0xFF), (float)(int8_t)((pw >> 16) & 0xFF)};
        PY[w] = f32x2{(float)(int8_t)((pw >> 8) & 0xFF), (float)(int8_t)(pw >> 24)};
    }
    // 4. groups of G slots
    uint32_t dlo = 0u, dhi = 0u;   // descriptor word (lane 4r + w = word w of slot r)
#pragma unroll
    for (int gi = 0; gi < NG; gi++) {
#pragma unroll
        for (int j = 0; j < G; j++) {
            const int r = gi * G + j;
            if (!((vmask >> r) & 1)) continue;
            uint32_t *pt = patch[wv][j];
            if ((smask >> r) & 1) {
                if (lane < 60) {
#pragma unroll
                    for (int k = 0; k < 7; k++)
                        if (k < 6 || rr0 == 0) pt[10 * (rr0 + 6 * k) + q10] = T[gi % NB][j][k];
                }
            } else {   // near the end of the blurred buffer: clamped loads, staged directly
                const long long ar = (long long)rl64((unsigned long long)a0, r);
                const int bwr = __builtin_amdgcn_readlane(bw, r);
#pragma unroll
                for (int k = 0; k < 7; k++) {
                    const int id = lane + 64 * k;
                    if (id < 37 * PW) {
                        const int rr = id / PW, q = id - rr * PW;
                        long long ad = ar + (long long)rr * bwr + 4 * q;
                        ad = ad < 0 ? 0 : (ad > amax ? amax & ~3LL : ad);
                        pt[id] = *(const uint32_t *)(blur + ad);
                    }
                }
            }
        }
        wave_lds_sync();
        if (gi + NB < NG) issue_patch(gi + NB, T[gi % NB]);   // the buffer just staged
#pragma unroll
        for (int j = 0; j < G; j++) {
            const int r = gi * G + j;
            if (!((vmask >> r) & 1)) continue;
            const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ca), r));
            const float bs = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sa), r));
            // GET_VALUE(idx) = center[cvRound(x*b + y*a)*step + cvRound(x*a - y*b)] (:158-160), the
            // products and sums rounded one by one as on x86 (no contraction). cvRound (round half to
            // even) as v + 1.5*2^23: for |v| < 2^22 the float sum holds round(v) in its low mantissa
            // bits, bits = 0x4B400000 + round(v); the rotated offsets are within +-18, so the byte
            // index (dy + 18) * 4 PW + dx + 18 + psh = bits_y * 4 PW + bits_x - C (24-bit multiply of
            // bits_y's low 24 bits 0x400000 + dy, unsigned wrap-around)
            const uint8_t *pc = (const uint8_t *)patch[wv][j];
            const uint32_t ib = (uint32_t)(18 * 4 * PW + 18 + __builtin_amdgcn_readlane(psh, r)) - (0x400000u * 4u * PW + 0x4B400000u);
            const f32x2 av = {a, a}, bv = {bs, bs}, MAG = {12582912.0f, 12582912.0f};
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const f32x2 qy = (PX[w] * bv + PY[w] * av) + MAG;
                const f32x2 qx = (PX[w] * av - PY[w] * bv) + MAG;
                const uint32_t i0 = __umul24(__float_as_uint(qy.x), 4u * PW) + __float_as_uint(qx.x) + ib;
                const uint32_t i1 = __umul24(__float_as_uint(qy.y), 4u * PW) + __float_as_uint(qx.y) + ib;
                const unsigned long long word = __ballot(pc[i0] < pc[i1]);
                dlo = (uint32_t)write_lane((int)(uint32_t)word, 4 * r + w, (int)dlo);
                dhi = (uint32_t)write_lane((int)(uint32_t)(word >> 32), 4 * r + w, (int)dhi);
            }
        }
        if (gi + 1 < NG) wave_lds_sync();   // this group's reads before the next group's writes
    }
    // 5. outputs
    const int rd = lane >> 2;
    const int offd = __shfl(off, rd);
    if (lane < 4 * NS && ((vmask >> rd) & 1))
        *(uint2 *)(desc + ((long long)b * cap + offd) * 32 + 8 * (lane & 3)) = make_uint2(dlo, dhi);
    if (valid) {
        orbx_kp kp;
        kp.x = (float)kx;
        kp.y = (float)ky;
        if (l != 0) { const float s = g.scale[l]; kp.x *= s; kp.y *= s; }   // :1642-1651
        kp.size = (float)g.scaled_patch[l];
        kp.angle = ang;
        kp.response = (float)key_score(key);
        kp.octave = l;
        kp.class_id = -1;
        kps[(long long)b * cap + off] = kp;
    }
}

// ------------------------------------------------------------------------------------
// Host: tables and geometry
// ------------------------------------------------------------------------------------
static inline int host_round(float v) { return (int)std::lrintf(v); }

static void compute_tables(orbx_engine *e) {
    const orbx_params &p = e->p;
    const double sf = (double)p.scale_factor;  // ORBextractor.h:203 double member
    e->scale[0] = 1.0f;
    e->sigma2[0] = 1.0f;
    for (int i = 1; i < p.nlevels; i++) {
        e->scale[i] = (float)((double)e->scale[i - 1] * sf);
        e->sigma2[i] = e->scale[i] * e->scale[i];
    }
    for (int i = 0; i < p.nlevels; i++) {
        e->inv_scale[i] = 1.0f / e->scale[i];
        e->inv_sigma2[i] = 1.0f / e->sigma2[i];
    }
    const float factor = (float)(1.0f / sf);
    float nDesired = p.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; l++) {
        e->nfeat[l] = host_round(nDesired);
        sum += e->nfeat[l];
        nDesired *= factor;
    }
    e->nfeat[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
    const char *hex = ORB_PATTERN_31_HEX;
    for (int i = 0; i < 1024; i++) {
        auto nib = [](char ch) { return ch <= '9' ? ch - '0' : (ch | 0x20) - 'a' + 10; };
        e->pattern[i] = (int8_t)(uint8_t)(nib(hex[2 * i]) * 16 + nib(hex[2 * i + 1]));
    }
    int v, v0, vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
    const double hp2 = 15 * 15;
    for (v = 0; v <= vmax; ++v) e->umax[v] = (int)std::lrint(std::sqrt(hp2 - v * v));
    for (v = 15, v0 = 0; v >= vmin; --v) {
        while (e->umax[v0] == e->umax[v0 + 1]) ++v0;
        e->umax[v] = v0;
        ++v0;
    }
}

int prof_begin(orbx_engine *e, hipStream_t s) {
    if (!e->prof) return -1;
    if (e->ev_used + 2 > e->ev_pool.size()) {
        for (int k = 0; k < 64; k++) {
            hipEvent_t ev;
            if (hipEventCreate(&ev) != hipSuccess) return -1;
            e->ev_pool.push_back(ev);
        }
    }
    const int h = (int)e->ev_used;
    e->ev_used += 2;
    (void)hipEventRecord(e->ev_pool[h], s);
    return h;
}

void prof_end(orbx_engine *e, hipStream_t s, int h, const char *name, int launches) {
    if (!e->prof || h < 0) return;
    (void)hipEventRecord(e->ev_pool[h + 1], s);
    e->prof_recs.push_back({name, e->ev_pool[h], e->ev_pool[h + 1], launches});
}

static int simd_end_for(int width) {
    int x = 0;
    for (; x <= width - 16; x += 16) {}
    for (; x < width - 4; x += 4) {}
    return x;
}

int engine_reserve(orbx_engine *e, int W, int H, int max_images) {
    if (W <= 0 || H <= 0 || max_images <= 0) return ORBX_EINVAL;
    if (W > 4000 || H > 4000) return ORBX_EINVAL;  // packed keys use 12-bit coordinates
    HIPCHK(hipSetDevice(e->device));
    const bool same = (W == e->W && H == e->H);
    if (same && max_images <= e->max_images) return ORBX_OK;
    // A new size is built into locals and committed only after every check and upload has
    // passed, so a rejected size leaves the engine's current geometry intact.
    ExtractGeom gnew{};
    int rz_rows[ORBX_MAXL] = {};
    ExtractGeom &g = same ? e->g : gnew;
    if (!same) {
        const int L = e->p.nlevels;
        g.nlevels = L; g.W = W; g.H = H;
        long long pyr = 0, blur = 0;
        for (int l = 0; l < L; l++) {
            g.lw[l] = host_round((float)W * e->inv_scale[l]);
            g.lh[l] = host_round((float)H * e->inv_scale[l]);
            if (g.lw[l] < 40 || g.lh[l] < 40) return ORBX_EINVAL;
            g.pyr_off[l] = l == 0 ? 0 : pyr;
            g.bp[l] = (g.lw[l] + 15) & ~15;
            if (l > 0) pyr += ((long long)g.bp[l] * g.lh[l] + 63) & ~63LL;
            // blurred levels: rows on ORBX_BLUR_ALIGN (128) bytes, so fast_blur_kernel's 128-column tile
            // rows are whole 128-B lines, each written by one workgroup (no partial-line write-backs)
            g.bbp[l] = (g.lw[l] + ORBX_BLUR_ALIGN - 1) & ~(ORBX_BLUR_ALIGN - 1);
            g.blur_off[l] = blur;
            blur += ((long long)g.bbp[l] * g.lh[l] + 127) & ~127LL;
            g.scale[l] = e->scale[l];
            g.inv_scale[l] = e->inv_scale[l];
            g.scaled_patch[l] = (int)(31 * e->scale[l]);
        }
        g.pyr_stride = std::max(pyr, 64LL);
        g.blur_stride = blur;
        // FAST cell grid (:1046-1153): the cells of a level are the rows i < ncell_rows, columns
        // j < ncell_cols that pass this fork's skip tests, numbered row-major from cell_base
        int cell_cap = 0, maxM_total = 0, ncells = 0;
        long long qt = 0;
        int node_cap = 0;
        for (int l = 0; l < L; l++) {
            const int minB = 16, maxBX = g.lw[l] - 19 + 3, maxBY = g.lh[l] - 19 + 3;
            g.maxBX[l] = maxBX; g.maxBY[l] = maxBY;
            const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
            const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
            if (nCols <= 0 || nRows <= 0) return ORBX_EINVAL;
            const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
            if (wCell + 6 > ORBX_TMAX || hCell + 6 > ORBX_TMAX) return ORBX_EINVAL;
            cell_cap = std::max(cell_cap, ((((wCell + 1) / 2) * ((hCell + 1) / 2) + 3) & ~3));   // uint4 slot rows
            g.cell_base[l] = ncells;
            int rows = 0, cols = 0;
            for (int i = 0; i < nRows; i++)
                if ((float)(minB + i * hCell) < maxBY - 3) rows = i + 1;   // :1099 skips iniY >= maxBorderY - 3
            for (int j = 0; j < nCols; j++)
                if ((float)(minB + j * wCell) < maxBX - 6) cols = j + 1;   // this fork's bound (:1112)
            g.hcell[l] = hCell; g.wcell[l] = wCell;
            g.ncell_rows[l] = rows; g.ncell_cols[l] = cols;
            // ceil(2^20 / side): floor(v * mag / 2^20) == v / side for v * (mag * side - 2^20) < 2^20,
            // i.e. every coordinate below 4096 with side <= 60
            g.hcell_mag[l] = ((1 << 20) + hCell - 1) / hCell;
            g.wcell_mag[l] = ((1 << 20) + wCell - 1) / wCell;
            ncells += rows * cols;
            // quadtree parameters (:700-705)
            g.N[l] = e->nfeat[l];
            const int nIni = (int)std::round((float)(maxBX - minB) / (maxBY - minB));
            if (nIni <= 0 || nIni > 64) return ORBX_EINVAL;
            g.nIni[l] = nIni;
            g.hX[l] = (float)(maxBX - minB) / nIni;
            g.out_cap[l] = std::max(g.N[l] + 3, 4 * nIni);
            node_cap = std::max(node_cap, g.out_cap[l] + 4);
        }
        g.cell_base[L] = ncells;
        g.ncell_total = g.cell_base[L];
        g.cell_cap = cell_cap;
        g.out_base[0] = 0;
        for (int l = 0; l < L; l++) g.out_base[l + 1] = g.out_base[l] + g.out_cap[l];
        for (int l = 0; l < L; l++) {
            g.qt_off[l] = qt;
            const long long mcap = (long long)(g.cell_base[l + 1] - g.cell_base[l]) * cell_cap;
            qt += 3 * mcap;   // K0, K1, node index (2 x int16) -- global fallback
            maxM_total = std::max<long long>(maxM_total, mcap);
        }
        g.qt_off[L] = qt;
        g.node_cap = (node_cap + 63) & ~63;
        int np2 = 1;
        while (np2 < g.node_cap) np2 <<= 1;
        g.node_pow2 = np2;
        if (g.node_cap > 32767 || maxM_total >= (1 << 24)) return ORBX_EINVAL;  // int16 node ids, 24-bit positions
        const size_t node_bytes = (2 * sizeof(QNode) + sizeof(QTmp)) * g.node_cap + 16 * (size_t)np2;
        // Node arrays live in global scratch (L2-resident, per-workgroup slice) and the keys
        // (2 x u32) + node index (2 x int16) per candidate take at most 28 KB of LDS with the
        // static QShared, so five workgroups share a CU; levels with more candidates run on the
        // global scratch. Measured at 256 KITTI pairs (tools/env_sweep.sh): nodes in LDS + 80 KB
        // (2 per CU) 0.64 ms, nodes in LDS + keys 256 (3 per CU) 0.60 ms, nodes global + 28 KB
        // (5 per CU) 0.52 ms, 32 KB (4 per CU) 0.57 ms, 16 KB 0.59 ms. ORBX_QT_NODES_LDS=1 /
        // ORBX_QT_LDS_KB=<k> are tuning knobs.
        g.qt_nodes_in_lds = 0;
        g.qt_nodes_in_lds = orbx_layout_knob("ORBX_QT_NODES_LDS", 0) != 0 && node_bytes <= 48 * 1024;
        g.qt_node_stride = (long long)((node_bytes + 15) / 16) * 4;
        long long qt_lds = 28 * 1024;
        qt_lds = std::max(16, std::min(160, orbx_layout_knob("ORBX_QT_LDS_KB", 28))) * 1024LL;
        const long long kl_bytes = qt_lds - (long long)sizeof(QShared) - 256 -
                                   (g.qt_nodes_in_lds ? (long long)node_bytes : 0);
        g.qt_kl = (int)std::max<long long>(256, (kl_bytes / 12) & ~63LL);
        g.ini_th = e->p.ini_th_fast;
        g.min_th = e->p.min_th_fast;
        g.resize_mode = e->p.resize_mode;
        g.blur_mode = e->p.blur_mode;
        // resize coefficient tables
        std::vector<int2> rzc;
        std::vector<int4> rzr;
        for (int l = 1; l < L; l++) {
            const int sw = g.lw[l - 1], sh = g.lh[l - 1], dw = g.lw[l], dh = g.lh[l];
            const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
            if (scale_x > 2.0) return ORBX_EINVAL;   // 4 outputs span <= 8 source bytes
            auto satS = [](float v) { int r = host_round(v); return std::min(std::max(r, -32768), 32767); };
            g.rz_col_off[l] = (int)rzc.size();
            for (int dx = 0; dx < dw; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = (int)std::floor(fx);
                fx -= sx;
                if (sx < 0) { fx = 0; sx = 0; }
                if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
                const int a0 = satS((1.f - fx) * 2048), a1 = satS(fx * 2048);
                // the kernel's vertical pass has no clamp (resize_level_kernel): it needs
                // a0 + a1 == b0 + b1 == 2^11 -- every level of every width <= 4000 at scale factors
                // 1.1-2.0 has it (float32 emulation); enforced here, not assumed
                if (a0 < 0 || a1 < 0 || a0 + a1 != 2048) return ORBX_EINVAL;
                const int sx1 = std::min(sx + 1, sw - 1);
                rzc.push_back(make_int2(sx | (a0 << 16), a1 | ((sx1 - sx) << 16)));
            }
            g.rz_row_off[l] = (int)rzr.size();
            for (int dy = 0; dy < dh; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = (int)std::floor(fy);
                fy -= sy;
                auto clip = [sh](int y) { return y >= 0 ? (y < sh ? y : sh - 1) : 0; };
                const int b0 = satS((1.f - fy) * 2048), b1 = satS(fy * 2048);
                if (b0 < 0 || b1 < 0 || b0 + b1 != 2048) return ORBX_EINVAL;   // as a0 + a1 above
                rzr.push_back(make_int4(clip(sy), clip(sy + 1), b0, b1));
            }
            g.rz_simd_end[l] = e->p.resize_mode ? simd_end_for(dw) : 0;
            // source rows one output tile spans (LDS of the horizontal pass)
            int rows = 0;
            for (int y0 = 0; y0 < dh; y0 += RZ_TH) {
                const int y1 = std::min(y0 + RZ_TH, dh) - 1;
                rows = std::max(rows, rzr[g.rz_row_off[l] + y1].y - rzr[g.rz_row_off[l] + y0].x + 1);
            }
            if (rows * 32 * (int)sizeof(uint4) > 64 * 1024) return ORBX_EINVAL;
            rz_rows[l] = rows;
        }
        if (rzc.empty()) rzc.push_back(make_int2(0, 0));
        if (rzr.empty()) rzr.push_back(make_int4(0, 0, 0, 0));
        // blur tiles
        g.blur_tile_base[0] = 0;
        for (int l = 0; l < L; l++) {
            g.blur_tiles_x[l] = (g.lw[l] + FB_TW - 1) / FB_TW;
            g.blur_tx_rcp[l] = (unsigned)(((1ull << 31) + g.blur_tiles_x[l] - 1) / g.blur_tiles_x[l]);
            g.blur_tiles_y[l] = (g.lh[l] + FB_TH - 1) / FB_TH;
            g.blur_tile_base[l + 1] = g.blur_tile_base[l] + g.blur_tiles_x[l] * g.blur_tiles_y[l];
        }
        // From here on the engine's tables change: drop the old size first, so a failure
        // below leaves an engine that rebuilds on the next call instead of one that runs the
        // new tables against the old geometry.
        HIPCHK(hipStreamSynchronize(e->stream));
        if (e->done) HIPCHK(hipEventSynchronize(e->done));   // last launches may still read the tables
        e->W = e->H = 0;
        e->max_images = 0;
        e->last_n = 0;
        e->st_pairs = 0;
        e->pending_in = nullptr;
        if (e->d_rz.ensure(sizeof(int2) * rzc.size()) || e->d_rzr.ensure(sizeof(int4) * rzr.size())) return ORBX_EDEVICE;
        HIPCHK(hipMemcpy(e->d_rz.p, rzc.data(), sizeof(int2) * rzc.size(), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->d_rzr.p, rzr.data(), sizeof(int4) * rzr.size(), hipMemcpyHostToDevice));
        e->g = gnew;
        for (int l = 0; l < ORBX_MAXL; l++) e->rz_rows[l] = rz_rows[l];
        e->W = W; e->H = H;
    }
    ExtractGeom &gc = e->g;
    const long long B = max_images;
    // the pyramid carries a 64-byte readable tail (fast_blur_kernel's staging loads)
    if (e->d_pyr.ensure(B * gc.pyr_stride + 64) || e->d_blur.ensure(B * gc.blur_stride) ||
        e->d_cell_cnt.ensure(sizeof(int) * B * gc.ncell_total) ||
        e->d_cell_keys.ensure(sizeof(uint32_t) * B * gc.ncell_total * gc.cell_cap) ||
        e->d_qt.ensure(sizeof(uint32_t) * B * gc.qt_off[gc.nlevels]) ||
        e->d_qt_nodes.ensure(gc.qt_nodes_in_lds ? 16 : (size_t)4 * B * gc.nlevels * gc.qt_node_stride) ||
        e->d_sel.ensure(sizeof(uint32_t) * B * gc.out_base[gc.nlevels]) ||
        e->d_sel_cnt.ensure(sizeof(int) * B * gc.nlevels) ||
        e->d_kps.ensure(sizeof(orbx_kp) * B * gc.out_base[gc.nlevels]) ||
        e->d_desc.ensure((size_t)32 * B * gc.out_base[gc.nlevels]) || e->d_cnt.ensure(sizeof(int) * B))
        return ORBX_EDEVICE;
    e->max_images = max_images;
    return ORBX_OK;
}

int engine_extract_device(orbx_engine *e, const uint8_t *d_imgs, int n, int pitch,
                          long long stride, hipStream_t s, int phase) {
    ExtractGeom g = e->g;
    g.nimg = n;
    g.in_pitch = pitch;
    g.in_stride = stride;
    const int L = g.nlevels;
    uint8_t *pyr = e->d_pyr.as<uint8_t>();
    const int cap = g.out_base[L];
    HIPCHK(order_after_done(e, s));
    if (phase & 1) {
    int ph = prof_begin(e, s);
    for (int rep = 0; rep < ((exp_twice() & 1) ? 2 : 1); rep++)
    for (int l = 1; l < L; l++) {
        const int tiles_x = (g.lw[l] + RZ_TW - 1) / RZ_TW, tiles_y = (g.lh[l] + RZ_TH - 1) / RZ_TH;
        const size_t lds = sizeof(uint4) * 32 * (size_t)e->rz_rows[l];
        const dim3 grid((unsigned)(tiles_x * tiles_y), n);
        const int2 *cx = e->d_rz.as<int2>() + g.rz_col_off[l];
        const int4 *ry = e->d_rzr.as<int4>() + g.rz_row_off[l];
        if (g.resize_mode)
            resize_level_kernel<true><<<grid, 256, lds, s>>>(g, l, tiles_x, cx, ry, d_imgs, pyr);
        else
            resize_level_kernel<false><<<grid, 256, lds, s>>>(g, l, tiles_x, cx, ry, d_imgs, pyr);
    }
    prof_end(e, s, ph, "resize_level_kernel", (L - 1) * ((exp_twice() & 1) ? 2 : 1));   // one launch per level
    HIPCHK(hipMemsetAsync(e->d_cell_cnt.p, 0, sizeof(int) * (size_t)n * g.ncell_total, s));   // cell slot counters
    if (e->fb_gate) HIPCHK(hipStreamWaitEvent(s, e->fb_gate, 0));
    ph = prof_begin(e, s);
    if (g.blur_mode)
        fast_blur_kernel<true><<<dim3(g.blur_tile_base[L], n), 256, 0, s>>>(g, d_imgs, pyr, e->d_blur.as<uint8_t>(),
                                                                         e->d_cell_cnt.as<int>(), e->d_cell_keys.as<uint32_t>());
    else
        fast_blur_kernel<false><<<dim3(g.blur_tile_base[L], n), 256, 0, s>>>(g, d_imgs, pyr, e->d_blur.as<uint8_t>(),
                                                                          e->d_cell_cnt.as<int>(), e->d_cell_keys.as<uint32_t>());
    prof_end(e, s, ph, "fast_blur_kernel");
    }
    if (phase & 2) {
    int ph = prof_begin(e, s);
    size_t lds = 12 * (size_t)g.qt_kl;
    if (g.qt_nodes_in_lds) lds += (2 * sizeof(QNode) + sizeof(QTmp)) * g.node_cap + 16 * (size_t)g.node_pow2;
    for (int rep = 0; rep < ((exp_twice() & 2) ? 2 : 1); rep++)
    (g.qt_nodes_in_lds ? quadtree_kernel<true> : quadtree_kernel<false>)<<<dim3(n, L), ORBX_QT_THREADS, lds, s>>>(
        g, e->d_cell_cnt.as<int>(), e->d_cell_keys.as<uint32_t>(), e->d_qt.as<uint32_t>(),
        e->d_qt_nodes.as<unsigned char>(), e->d_sel.as<uint32_t>(), e->d_sel_cnt.as<int>());
    prof_end(e, s, ph, "quadtree_kernel");
    ph = prof_begin(e, s);
    const uint8_t *d_blur = e->d_blur.as<uint8_t>();
    for (int rep = 0; rep < ((exp_twice() & 4) ? 2 : 1); rep++)
        describe2_kernel<<<dim3((cap + 4 * kDescNS - 1) / (4 * kDescNS), n), 256, 0, s>>>(
            g, d_imgs, pyr, d_blur, e->d_sel.as<uint32_t>(), e->d_sel_cnt.as<int>(), e->d_kps.as<orbx_kp>(),
            e->d_desc.as<uint8_t>(), e->d_cnt.as<int>());
    prof_end(e, s, ph, "describe2_kernel");
    }
    HIPCHK(hipGetLastError());
    HIPCHK(mark_done(e, s));
    e->last_in = d_imgs;
    e->last_pitch = pitch;
    e->last_stride = stride;
    e->last_n = n;
    if (phase & 2) e->gen++;
    return ORBX_OK;
}

}  // namespace orbamd

// ------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------
extern "C" {

const char *orbslam2_amd_version(void) { return "orbslam2_amd 0.1 (gfx950)"; }

int orbslam2_amd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int orbx_create(const orbx_params *p, orbx_engine **out) {
    if (!p || !out) return ORBX_EINVAL;
    *out = nullptr;
    if (p->struct_size != sizeof(orbx_params)) return ORBX_EINVAL;   // a caller built against another layout
    if (p->nlevels < 1 || p->nlevels > ORBX_MAXL || p->nfeatures < 0 || !(p->scale_factor > 1.0f))
        return ORBX_EINVAL;
    if ((unsigned)p->resize_mode > 1u || (unsigned)p->blur_mode > 1u) return ORBX_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return ORBX_EDEVICE;
    orbx_engine *e = new orbx_engine();
    e->p = *p;
    if (hipGetDevice(&e->device) != hipSuccess) { delete e; return ORBX_EDEVICE; }
    compute_tables(e);
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { delete e; return ORBX_EDEVICE; }
    e->done = orbamd::make_done_event();
    if (!e->done) { (void)hipStreamDestroy(e->stream); delete e; return ORBX_EDEVICE; }
    uint2 icw[16 * 8];
    for (int av = 0; av < 16; av++) {
        for (int w = 0; w < 8; w++) {
            uint32_t wu = 0, wm = 0;
            for (int b = 0; b < 4; b++) {
                const int u = 4 * w + b - 16;
                if (std::abs(u) <= e->umax[av]) { wu |= (uint32_t)(u + 16) << (8 * b); wm |= 1u << (8 * b); }
            }
            icw[av * 8 + w] = make_uint2(wu, wm);
        }
    }
    // describe2's patch-load mask (c_pmask): row dy = r - 18 of the 37-row patch holds sampled pixels
    // only at |dx| <= floor(sqrt(R^2 - (|dy| - 1/2)^2) + 1/2), R = the pattern's largest radius
    // (cvRound moves a rotated point by <= 1/2 per axis; 1e-3 covers the float rotation's error)
    uint32_t pmask[64] = {};
    {
        double R2 = 0;
        for (int k = 0; k < 512; k++)
            R2 = std::max(R2, (double)e->pattern[2 * k] * e->pattern[2 * k] + (double)e->pattern[2 * k + 1] * e->pattern[2 * k + 1]);
        R2 = (std::sqrt(R2) + 1e-3) * (std::sqrt(R2) + 1e-3);
        for (int l = 0; l < 60; l++) {
            const int rr0 = l / 10, q = l % 10;
            for (int k = 0; k < 7; k++) {
                const int r = rr0 + 6 * k;
                if (r > 36) continue;
                const double ay = std::max(0.0, std::abs(r - 18) - 0.5);
                const int w = ay * ay >= R2 ? -1 : std::min(18, (int)std::floor(std::sqrt(R2 - ay * ay) + 0.5));
                for (int p = 0; p < 4; p++)   // bytes 18 - w + p .. 18 + w + p of the window
                    if (w >= 0 && q >= (18 - w + p) / 4 && q <= (18 + w + p) / 4) pmask[l] |= 1u << (7 * p + k);
            }
        }
    }
    DescLane dlane[64] = {};
    for (int l = 0; l < 64; l++) {
        const int w8 = l & 7, vr = l >> 3;
        for (int k = 0; k < 4; k++) {
            const int v = vr - 15 + 8 * k;
            if (k < 3 || vr <= 6) dlane[l].wt[k] = icw[std::abs(v) * 8 + w8];
        }
        dlane[l].pmask = pmask[l];
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), e->pattern, 1024) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_umax), e->umax, sizeof(e->umax)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_dlane), dlane, sizeof(dlane)) != hipSuccess) {
        (void)hipEventDestroy(e->done);
        (void)hipStreamDestroy(e->stream);
        delete e;
        return ORBX_EDEVICE;
    }
    *out = e;
    return ORBX_OK;
}

void orbx_destroy(orbx_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->done) (void)hipEventSynchronize(e->done);
    orbamd::frame_state_free(e);
    orbamd::DevBuf *bufs[] = {&e->d_rz, &e->d_rzr, &e->d_pattern, &e->d_in, &e->d_pyr, &e->d_blur,
                              &e->d_cell_cnt, &e->d_cell_keys, &e->d_qt, &e->d_qt_nodes, &e->d_sel,
                              &e->d_sel_cnt, &e->d_kps, &e->d_desc, &e->d_cnt, &e->d_st_sorted,
                              &e->d_st_res, &e->d_st_u, &e->d_st_depth, &e->d_st_dist, &e->d_st_rows};
    for (auto *b : bufs) b->release();
    e->h_stage.release();
    for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
    if (e->done) (void)hipEventDestroy(e->done);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

int orbx_levels(const orbx_engine *e, int *nlevels, float *scale, float *inv_scale, float *sigma2,
                float *inv_sigma2, int *features_per_level) {
    if (!e) return ORBX_EINVAL;
    const int L = e->p.nlevels;
    if (nlevels) *nlevels = L;
    for (int l = 0; l < L; l++) {
        if (scale) scale[l] = e->scale[l];
        if (inv_scale) inv_scale[l] = e->inv_scale[l];
        if (sigma2) sigma2[l] = e->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = e->inv_sigma2[l];
        if (features_per_level) features_per_level[l] = e->nfeat[l];
    }
    return ORBX_OK;
}

void *orbx_stream(orbx_engine *e) { return e ? (void *)e->stream : nullptr; }

int orbslam2_amd_set_device(int device) {
    return hipSetDevice(device) == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

int orbslam2_amd_device_sync(void) {
    return hipDeviceSynchronize() == hipSuccess ? ORBX_OK : ORBX_EDEVICE;
}

int orbx_profile(orbx_engine *e, int enable) {
    if (!e) return ORBX_EINVAL;
    for (auto &r : e->prof_recs) (void)hipEventSynchronize(r.b);   // events are reused after the reset
    e->prof = enable != 0;
    e->prof_recs.clear();
    e->ev_used = 0;
    return ORBX_OK;
}

int orbx_profile_read(orbx_engine *e, int idx, char *name, int name_cap, double *total_ms,
                      int *launches) {
    if (!e || idx < 0) return ORBX_EINVAL;
    for (auto &r : e->prof_recs) HIPCHK(hipEventSynchronize(r.b));
    std::vector<std::string> names;
    for (auto &r : e->prof_recs)
        if (std::find(names.begin(), names.end(), std::string(r.name)) == names.end()) names.push_back(r.name);
    if (idx >= (int)names.size()) return ORBX_ESTATE;
    double tot = 0;
    int cnt = 0;
    for (auto &r : e->prof_recs) {
        if (names[idx] != r.name) continue;
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, r.a, r.b));
        tot += ms;
        cnt += r.launches;
    }
    if (name && name_cap > 0) {
        std::snprintf(name, (size_t)name_cap, "%s", names[idx].c_str());
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = cnt;
    return ORBX_OK;
}

int orbx_reserve(orbx_engine *e, int w, int h, int max_images) {
    if (!e) return ORBX_EINVAL;
    return orbamd::engine_reserve(e, w, h, max_images);
}

int orbx_extract_batch_device(orbx_engine *e, const uint8_t *d_imgs, int n_images, int w, int h,
                              int pitch, size_t image_stride, void *stream) {
    return orbx_extract_batch_device_phase(e, d_imgs, n_images, w, h, pitch, image_stride, stream, 3);
}

int orbx_extract_batch_device_phase(orbx_engine *e, const uint8_t *d_imgs, int n_images, int w, int h,
                                    int pitch, size_t image_stride, void *stream, int phase) {
    if (!e || !d_imgs || n_images <= 0 || w <= 0 || h <= 0 || pitch < w || phase < 1 || phase > 3) return ORBX_EINVAL;
    if (n_images > 1 && image_stride < (size_t)pitch * (size_t)(h - 1) + (size_t)w) return ORBX_EINVAL;  // images overlap
    if (phase == 2 && (e->pending_in != d_imgs || e->pending_n != n_images || e->pending_w != w ||
                       e->pending_h != h || e->pending_pitch != pitch || e->pending_stride != (long long)image_stride))
        return ORBX_ESTATE;   // phase 2 must continue exactly the phase-1 batch
    int rc = orbamd::engine_reserve(e, w, h, std::max(n_images, e->max_images));
    if (rc) return rc;
    rc = orbamd::engine_extract_device(e, d_imgs, n_images, pitch, (long long)image_stride,
                                       stream ? (hipStream_t)stream : e->stream, phase);
    const bool p1 = phase == 1 && rc == ORBX_OK;
    e->pending_in = p1 ? d_imgs : nullptr;
    e->pending_n = p1 ? n_images : 0;
    e->pending_w = p1 ? w : 0;
    e->pending_h = p1 ? h : 0;
    e->pending_pitch = p1 ? pitch : 0;
    e->pending_stride = p1 ? (long long)image_stride : 0;
    return rc;
}

int orbx_capacity(const orbx_engine *e, int *cap) {
    if (!e || !cap) return ORBX_EINVAL;
    if (e->W == 0) return ORBX_ESTATE;   // no size reserved yet
    *cap = e->g.out_base[e->g.nlevels];
    return ORBX_OK;
}

int orbx_batch_results(orbx_engine *e, const int **d_counts, const orbx_kp **d_kps,
                       const uint8_t **d_desc, int *cap) {
    if (!e || e->last_n == 0) return ORBX_ESTATE;
    if (d_counts) *d_counts = e->d_cnt.as<int>();
    if (d_kps) *d_kps = e->d_kps.as<orbx_kp>();
    if (d_desc) *d_desc = e->d_desc.as<uint8_t>();
    if (cap) *cap = e->g.out_base[e->g.nlevels];
    return ORBX_OK;
}

// One image's results through the engine's pinned staging buffer: count, keypoints and
// descriptors (all `cap` rows) in one round trip on the engine's own stream, then the first
// `count` rows copied into the caller's arrays.
static int fetch_staged(orbx_engine *e, int image, orbx_kp *kps, uint8_t *desc, int cap, int *n, hipEvent_t producer) {
    const size_t kc = (size_t)e->g.out_base[e->g.nlevels];
    const size_t o_kps = 64, o_desc = o_kps + sizeof(orbx_kp) * kc;
    if (e->h_stage.ensure(o_desc + 32 * kc)) return ORBX_EDEVICE;
    orbamd::HostCopy hc(e->stream, producer);
    hc.d2h(e->h_stage.p, e->d_cnt.as<int>() + image, sizeof(int));
    hc.d2h(e->h_stage.as<void>(o_kps), e->d_kps.as<orbx_kp>() + image * kc, sizeof(orbx_kp) * kc);
    hc.d2h(e->h_stage.as<void>(o_desc), e->d_desc.as<uint8_t>() + image * kc * 32, 32 * kc);
    if (hc.finish()) return ORBX_EDEVICE;
    const int cnt = *e->h_stage.as<int>();
    *n = cnt;
    if (cnt > cap) return ORBX_ECAP;
    if (cnt > 0) {
        if (kps) std::memcpy(kps, e->h_stage.as<void>(o_kps), sizeof(orbx_kp) * cnt);
        if (desc) std::memcpy(desc, e->h_stage.as<void>(o_desc), 32 * (size_t)cnt);
    }
    return ORBX_OK;
}

int orbx_batch_fetch(orbx_engine *e, int image, orbx_kp *kps, uint8_t *desc, int cap, int *n) {
    if (!e || !n) return ORBX_EINVAL;
    if (e->last_n == 0 || image < 0 || image >= e->last_n) return ORBX_ESTATE;
    HIPCHK(hipSetDevice(e->device));
    return fetch_staged(e, image, kps, desc, cap, n, e->done);
}

int orbx_extract(orbx_engine *e, const uint8_t *img, int w, int h, int stride, orbx_kp *kps,
                 uint8_t *desc, int cap, int *n) {
    if (!e || !n) return ORBX_EINVAL;
    *n = 0;
    if (!img || w == 0 || h == 0) return ORBX_OK;  // ORBextractor.cc:1547 returns untouched
    if (w < 0 || h < 0 || stride < w) return ORBX_EINVAL;
    HIPCHK(hipSetDevice(e->device));
    int rc = orbamd::engine_reserve(e, w, h, std::max(1, e->max_images));
    if (rc) return rc;
    // exactly the image: no kernel reads past its last pixel (include/orbslam2_amd.h, input range)
    const size_t img_bytes = (size_t)w * h;
    if (e->d_in.ensure(img_bytes)) return ORBX_EDEVICE;
    // the host image is packed into the pinned staging buffer (the previous call's transfers on
    // this stream have completed: every call ends with a stream synchronisation) and goes up in
    // one DMA
    if (e->h_stage.ensure(std::max<size_t>(img_bytes, 64))) return ORBX_EDEVICE;
    HIPCHK(hipStreamWaitEvent(e->stream, e->done, 0));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (stride == w) {
        std::memcpy(e->h_stage.p, img, img_bytes);
    } else {
        for (int r = 0; r < h; r++) std::memcpy(e->h_stage.as<uint8_t>((size_t)r * w), img + (size_t)r * stride, (size_t)w);
    }
    HIPCHK(hipMemcpyAsync(e->d_in.p, e->h_stage.p, img_bytes, hipMemcpyHostToDevice, e->stream));
    rc = orbamd::engine_extract_device(e, e->d_in.as<uint8_t>(), 1, w, (long long)w * h, e->stream, 3);
    if (rc) return rc;
    return fetch_staged(e, 0, kps, desc, cap, n, nullptr);   // same stream: no event wait
}

int orbx_pyramid_level(orbx_engine *e, int image, int level, uint8_t *dst, int *w, int *h) {
    if (!e || level < 0 || level >= e->p.nlevels) return ORBX_EINVAL;
    if (e->last_n == 0 || image < 0 || image >= e->last_n) return ORBX_ESTATE;
    const int lw = e->g.lw[level], lh = e->g.lh[level];
    if (w) *w = lw;
    if (h) *h = lh;
    if (!dst) return ORBX_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamWaitEvent(e->stream, e->done, 0));
    if (level == 0) {
        HIPCHK(hipMemcpy2DAsync(dst, lw, e->last_in + image * e->last_stride, e->last_pitch, lw, lh, hipMemcpyDeviceToHost,
                                e->stream));
    } else {
        HIPCHK(hipMemcpy2DAsync(dst, lw, e->d_pyr.as<uint8_t>() + image * e->g.pyr_stride + e->g.pyr_off[level],
                                e->g.bp[level], lw, lh, hipMemcpyDeviceToHost, e->stream));
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return ORBX_OK;
}

int orbx_blurred_level(orbx_engine *e, int image, int level, uint8_t *dst, int *w, int *h) {
    if (!e || level < 0 || level >= e->p.nlevels) return ORBX_EINVAL;
    if (e->last_n == 0 || image < 0 || image >= e->last_n) return ORBX_ESTATE;
    const int lw = e->g.lw[level], lh = e->g.lh[level];
    if (w) *w = lw;
    if (h) *h = lh;
    if (!dst) return ORBX_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamWaitEvent(e->stream, e->done, 0));
    HIPCHK(hipMemcpy2DAsync(dst, lw, e->d_blur.as<uint8_t>() + image * e->g.blur_stride + e->g.blur_off[level],
                            e->g.bbp[level], lw, lh, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return ORBX_OK;
}

}  // extern "C"
