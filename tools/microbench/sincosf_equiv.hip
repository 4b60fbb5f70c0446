// Exhaustive check of orb_device.h's glibc_sincosf (immediates, round 6) against the previous
// table-in-memory form (kept below verbatim): every float in [0, 2*pi] (+ the describe angles' full
// range 0 .. 360 degrees times pi/180), bit-identical sin and cos required.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../orb-slam2-noted_amd/csrc sincosf_equiv.hip -o /tmp/sincosf_equiv
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "orb_device.h"

namespace old {
struct SinCosTab {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
static __constant__ SinCosTab kTab[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1ffffffd0c621cp-54,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1ffffffd0c621cp-54,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
__device__ float poly(double x, double x2, const SinCosTab &p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2, s1 = p.s2 + x2 * p.s3, x7 = x3 * x2, s = x + x3 * p.s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2, c2 = p.c3 + x2 * p.c4, c1 = p.c0 + x2 * p.c1, x6 = x4 * x2;
    double c = c1 + x4 * p.c2;
    return (float)(c + x6 * c2);
}
__device__ void sincosf(float y, float *s_out, float *c_out) {
    double x = y;
    const float pio4 = 0x1.921FB6p-1f;
    if (orbamd::abstop12(y) < orbamd::abstop12(pio4)) {
        if (orbamd::abstop12(y) < orbamd::abstop12(0x1p-12f)) { *c_out = 1.0f; *s_out = y; return; }
        *c_out = poly(x, x * x, kTab[0], 1);
        *s_out = poly(x, x * x, kTab[0], 0);
        return;
    }
    double r = x * kTab[0].hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * kTab[0].hpi;
    double s = kTab[0].sign[n & 3];
    const SinCosTab &p = kTab[(n & 2) ? 1 : 0];
    *c_out = poly(x * s, x * x, p, n ^ 1);
    *s_out = poly(x * s, x * x, p, n);
}
}  // namespace old

__global__ void check(uint32_t lo, uint32_t n, unsigned long long *bad, uint32_t *first) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float y = __uint_as_float(lo + i);
    float s0, c0, s1, c1;
    old::sincosf(y, &s0, &c0);
    orbamd::glibc_sincosf(y, &s1, &c1);
    if (__float_as_uint(s0) != __float_as_uint(s1) || __float_as_uint(c0) != __float_as_uint(c1)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, lo + i);
    }
}

int main() {
    float tp = 6.2831855f;
    uint32_t tpb;
    memcpy(&tpb, &tp, 4);
    const uint32_t lo = 0u, hi = tpb + 1u;   // +0 .. just past 2*pi
    unsigned long long *bad;
    uint32_t *first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(first, 0xFF, 4);
    const uint32_t n = hi - lo;
    check<<<(n + 255) / 256, 256>>>(lo, n, bad, first);
    unsigned long long hb = 0;
    uint32_t hf = 0;
    if (hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    printf("{\"floats\": %u, \"mismatches\": %llu, \"first_bits\": %u}\n", n, hb, hf);
    return hb == 0 ? 0 : 1;
}
