// Device-side numerics shared by the orbslam2_amd HIP kernels (gfx950).
//
// Every helper reproduces a host-side primitive of the reference bit-for-bit:
//   * cv_round_f        cvRound(float)  = SSE2 cvtss2si, round-half-even
//   * fast_atan2_deg    cv::fastAtan2   (SURVEY.md A.4), float, no contraction
//   * glibc_cosf/sinf   glibc >= 2.28 cosf/sinf as called by computeOrbDescriptor
//                       (ORBextractor.cc:157-158); double evaluation identical to
//                       sysdeps/ieee754/flt-32/{s_cosf,s_sinf}.c
// The whole library is compiled with -ffp-contract=off so a*b+c stays two roundings,
// like the reference's x86-64 SSE2 build (CMakeLists.txt:19-23, no -march=native).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbamd {

__device__ __forceinline__ int cv_round_f(float v) { return (int)__builtin_rintf(v); }

// ORBmatcher::DescriptorDistance (ORBmatcher.cc:2123-2143): popcount of the XOR of two 32-byte
// descriptors (rows 16-byte aligned), as two 16-byte loads per side
__device__ __forceinline__ int hamming32(const uint8_t *a, const uint8_t *b) {
    const uint4 *pa = (const uint4 *)a, *pb = (const uint4 *)b;
    const uint4 x0 = pa[0], x1 = pa[1], y0 = pb[0], y1 = pb[1];
    return __popc(x0.x ^ y0.x) + __popc(x0.y ^ y0.y) + __popc(x0.z ^ y0.z) + __popc(x0.w ^ y0.w) +
           __popc(x1.x ^ y1.x) + __popc(x1.y ^ y1.y) + __popc(x1.z ^ y1.z) + __popc(x1.w ^ y1.w);
}

// XCD-aware workgroup remap (cdna_hip_programming.md §5.5 T1, bijective form). Workgroups are
// dealt round-robin over the 8 XCDs (each with a private L2); remapping the linear id so every
// XCD works one contiguous range of the grid keeps an image's pyramid / blurred pixels in one
// L2 instead of eight. A pure speed choice: any placement gives the same results.
__device__ __forceinline__ unsigned xcd_linear() {
    const unsigned nwg = gridDim.x * gridDim.y * gridDim.z;
    const unsigned orig = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    const unsigned q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
// Chunked form: the linear ids are cut into runs of 8 M workgroups; inside a run XCD k (which the
// hardware gives ids k, k + 8, ...) takes M consecutive logical ids. Neighbouring workgroups share an
// L2 while the chip as a whole still sweeps the grid in order (addresses stay close together).
template <int M> __device__ __forceinline__ void xcd_remap2_chunk(int &bx, int &by) {
    const unsigned nwg = gridDim.x * gridDim.y;
    const unsigned orig = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned c = orig / (8u * M), r = orig - c * (8u * M);
    unsigned w = c * (8u * M) + (r % 8u) * M + r / 8u;
    if (c * (8u * M) + 8u * M > nwg) w = orig;   // the last partial run keeps the hardware order
    bx = (int)(w % gridDim.x);
    by = (int)(w / gridDim.x);
}
__device__ __forceinline__ void xcd_remap2(int &bx, int &by) {
    const unsigned w = xcd_linear();
    bx = (int)(w % gridDim.x);
    by = (int)(w / gridDim.x);
}
__device__ __forceinline__ void xcd_remap3(int &bx, int &by, int &bz) {
    const unsigned w = xcd_linear();
    bx = (int)(w % gridDim.x);
    by = (int)((w / gridDim.x) % gridDim.y);
    bz = (int)(w / (gridDim.x * gridDim.y));
}

__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
    const float kR2D = (float)(180.0 / 3.1415926535897932384626433832795);
    const float p1 = 0.9997878412794807f * kR2D;
    const float p3 = -0.3258083974640975f * kR2D;
    const float p5 = 0.1555786518463281f * kR2D;
    const float p7 = -0.04432655554792128f * kR2D;
    const float eps = (float)2.2204460492503131e-16;
    float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// glibc's sincosf table (__sincosf_table, sincosf.h) as immediates: entry 1 is entry 0 with the cosine
// coefficients c0..c4 negated, and since negation is exact and round-to-nearest is sign-symmetric,
// the cosine polynomial on entry 1 is exactly the negated one on entry 0. No table in memory: a vector
// load of the table (its index is per lane) made every caller wait vmcnt(0) for all its loads in flight.
struct SinCosK {
    static constexpr double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
    static constexpr double c0 = 0x1p0, c1 = -0x1ffffffd0c621cp-54, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                            c4 = 0x1.99343027bf8c3p-16;
    static constexpr double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
};

__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

// glibc's sinf_poly: n even -> the sine polynomial, odd -> the cosine polynomial (of table entry 0;
// entry 1's is its negation, applied by the caller)
__device__ __forceinline__ float sc_poly(double x, double x2, int n) {
    using K = SinCosK;
    if ((n & 1) == 0) {
        double x3 = x * x2, s1 = K::s2 + x2 * K::s3, x7 = x3 * x2, s = x + x3 * K::s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2, c2 = K::c3 + x2 * K::c4, c1 = K::c0 + x2 * K::c1, x6 = x4 * x2;
    double c = c1 + x4 * K::c2;
    return (float)(c + x6 * c2);
}

// cos and sin of a float angle in [0, 2*pi] exactly as glibc's cosf / sinf.
__device__ __forceinline__ void glibc_sincosf(float y, float *s_out, float *c_out) {
    double x = y;
    const float pio4 = 0x1.921FB6p-1f;
    if (abstop12(y) < abstop12(pio4)) {
        if (abstop12(y) < abstop12(0x1p-12f)) { *c_out = 1.0f; *s_out = y; return; }
        *c_out = sc_poly(x, x * x, 1);
        *s_out = sc_poly(x, x * x, 0);
        return;
    }
    double r = x * SinCosK::hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * SinCosK::hpi;
    const double s = ((n ^ (n >> 1)) & 1) ? -1.0 : 1.0;   // glibc's sign[n & 3] = {1, -1, -1, 1}
    const bool neg = (n & 2) != 0;                        // table entry 1: its cosine polynomial negated
    const float cv = sc_poly(x * s, x * x, n ^ 1), sv = sc_poly(x * s, x * x, n);
    *c_out = (neg && ((n ^ 1) & 1)) ? -cv : cv;
    *s_out = (neg && (n & 1)) ? -sv : sv;
}

// Packed candidate key: score (8b) | x (12b) << 8 | y (12b) << 20, x/y relative to
// (minBorderX, minBorderY) as in ComputeKeyPointsOctTree (ORBextractor.cc:1141-1146).
__device__ __forceinline__ uint32_t pack_key(int x, int y, int score) {
    return (uint32_t)score | ((uint32_t)x << 8) | ((uint32_t)y << 20);
}
__device__ __forceinline__ int key_score(uint32_t k) { return (int)(k & 0xFF); }
__device__ __forceinline__ int key_x(uint32_t k) { return (int)((k >> 8) & 0xFFF); }
__device__ __forceinline__ int key_y(uint32_t k) { return (int)(k >> 20); }

__device__ __forceinline__ int wave_lane() { return (int)__lane_id(); }

// wavefront index inside the workgroup as a wave-uniform (SGPR) value: lets the compiler keep
// everything derived from it (slot / cell / keypoint ids, their loads and branches) scalar
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }


// order LDS traffic between lanes of one wavefront (LDS executes a wave's ops in order)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace orbamd
