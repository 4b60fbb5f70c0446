// Probe: packed f16 arithmetic on denormal-encoded bytes (byte b as the f16 bit pattern b, i.e.
// b * 2^-24) and the ds_read_u8_d16 / _d16_hi packing, as fast_blur's two-candidate exact score
// uses them. Prints each op's result bits next to the exact expectation.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t *out) {
    __shared__ uint8_t lds[64];
    const int t = threadIdx.x;
    if (t < 64) lds[t] = (uint8_t)(3 * t + 1);
    __syncthreads();
    if (t != 0) return;
    const uint32_t a = (200u << 16) | 17u, b = (35u << 16) | 90u, c = (120u << 16) | 60u;
    const uint32_t Sd = 0xBC003C00u;   // hi: -1, lo: +1
    uint32_t r;
    asm volatile("v_pk_fma_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(Sd), "v"(c)); out[0] = r;      // lo 17+60=77, hi -200+120=-80
    asm volatile("v_pk_min_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); out[1] = r;                     // lo 17, hi 35
    asm volatile("v_pk_max_f16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); out[2] = r;                     // lo 90, hi 200
    asm volatile("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); out[3] = r;    // lo 17, hi 35
    asm volatile("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); out[4] = r;    // lo 90, hi 200
    asm volatile("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b)); out[5] = r;  // lo -73, hi 165
    const uint32_t base = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) uint8_t *)lds);
    uint32_t v;
    asm volatile("ds_read_u8_d16 %0, %1 offset:5\n\tds_read_u8_d16_hi %0, %2 offset:7\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(v) : "v"(base), "v"(base + 1) : "memory");
    out[6] = v;   // lo lds[5] = 16, hi lds[8] = 25
    asm volatile("v_pk_fma_f16 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(0x3C00BC00u), "v"(0x80000000u | 10u)); out[7] = r;  // lo -16+10=-6, hi 25-0=25
}

int main() {
    uint32_t *d, h[8];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    probe<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *name[8] = {"fma", "min", "max", "minimum3", "maximum3", "sub", "d16pack", "fma2"};
    for (int i = 0; i < 8; i++) {
        const int lo = (int16_t)(h[i] & 0xFFFF), hi = (int16_t)(h[i] >> 16);
        auto val = [](int bits) { return (bits & 0x8000) ? -(bits & 0x7FFF) : bits; };   // sign-magnitude denormal
        printf("%-9s bits %08x  lo %d  hi %d\n", name[i], h[i], val(lo & 0xFFFF), val(hi & 0xFFFF));
    }
    return 0;
}
