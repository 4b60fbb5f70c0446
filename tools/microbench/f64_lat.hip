// FP64 VALU / DPP64 latency and issue cost on one wavefront (gfx950): cycles per instruction of
// dependent chains and independent streams, timed with s_memtime (clock64). Informs the LocalBA
// diagonal-tile Cholesky (lba.hip chol16_pipe / chol16_factor).
#include <hip/hip_runtime.h>
#include <cstdio>
#define REP 256
__global__ void k(double *out, long long *cyc, double seed) {
    double a = seed + threadIdx.x * 1e-3, b = 1.0000001, c = 0.5, acc[8];
    for (int i = 0; i < 8; i++) acc[i] = a + i;
    long long t0, t1;
    // 0: dependent v_fma_f64 chain
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    t1 = clock64(); if (threadIdx.x == 0) cyc[0] = t1 - t0;
    // 1: independent v_fma_f64 (8 accumulators round robin)
    t0 = clock64();
    for (int i = 0; i < REP / 8; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[j]) : "v"(b), "v"(c));
    }
    t1 = clock64(); if (threadIdx.x == 0) cyc[1] = t1 - t0;
    // 2: dependent v_fmac_f64_dpp on the accumulator (DPP source fixed)
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(b), "v"(c));
    t1 = clock64(); if (threadIdx.x == 0) cyc[2] = t1 - t0;
    // 3: independent v_fmac_f64_dpp (8 accumulators)
    t0 = clock64();
    for (int i = 0; i < REP / 8; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++)
            asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(acc[j]) : "v"(b), "v"(c));
    }
    t1 = clock64(); if (threadIdx.x == 0) cyc[3] = t1 - t0;
    // 4: dependent v_mov_b64_dpp chain through the DPP source (+ the 2 wait states)
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(a));
    t1 = clock64(); if (threadIdx.x == 0) cyc[4] = t1 - t0;
    // 5: s_nop 1 alone
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("s_nop 1");
    t1 = clock64(); if (threadIdx.x == 0) cyc[5] = t1 - t0;
    // 6: dependent v_rsq_f64 chain (+ 1 wait state)
    double r = a * a + 1.0;
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("v_rsq_f64 %0, %0\n\ts_nop 0" : "+v"(r));
    t1 = clock64(); if (threadIdx.x == 0) cyc[6] = t1 - t0;
    // 7: independent v_rsq_f64 (8)
    t0 = clock64();
    for (int i = 0; i < REP / 8; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) asm volatile("v_rsq_f64 %0, %0" : "+v"(acc[j]));
    }
    t1 = clock64(); if (threadIdx.x == 0) cyc[7] = t1 - t0;
    // 8: dependent v_mul_f64 chain
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));
    t1 = clock64(); if (threadIdx.x == 0) cyc[8] = t1 - t0;
    // 9: dependent chain fmac_dpp where the NEXT op's DPP source is the previous result (critical form)
    double s = b;
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++)
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\tv_mov_b64 %1, %0" : "+v"(a), "+v"(s) : "v"(c));
    t1 = clock64(); if (threadIdx.x == 0) cyc[9] = t1 - t0;
    // 10: v_mov_b64 alone dependent
    t0 = clock64();
    _Pragma("unroll 16") for (int i = 0; i < REP; i++) asm volatile("v_mov_b64 %0, %1\n\tv_mov_b64 %1, %0" : "+v"(a), "+v"(s));
    t1 = clock64(); if (threadIdx.x == 0) cyc[10] = t1 - t0;
    // 11: ds_read_b64 dependent (address from value) -> LDS latency
    __shared__ double L[64];
    L[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int ix = threadIdx.x;
    t0 = clock64();
    for (int i = 0; i < REP / 8; i++) { double v = L[ix]; ix = ((int)v + 1) & 63; }
    t1 = clock64(); if (threadIdx.x == 0) cyc[11] = (t1 - t0) * 8;
    for (int j = 0; j < 8; j++) a += acc[j];
    out[threadIdx.x] = a + r + s + ix;
}
int main() {
    double *o; long long *c;
    hipMalloc(&o, 64 * 8); hipMalloc(&c, 16 * 8);
    for (int rep = 0; rep < 3; rep++) {
        k<<<1, 64>>>(o, c, 1.0);
        hipDeviceSynchronize();
    }
    long long h[16];
    hipMemcpy(h, c, 16 * 8, hipMemcpyDeviceToHost);
    const char *nm[] = {"fma dep", "fma indep", "fmac_dpp dep(acc)", "fmac_dpp indep", "mov_b64_dpp dep(src)+nop1",
                        "s_nop 1", "rsq dep+nop0", "rsq indep", "mul dep", "fmac_dpp->mov->dpp src dep +nop1", "mov_b64 x2 dep", "ds_read dep"};
    for (int i = 0; i < 12; i++) printf("%-36s %.1f cyc/op\n", nm[i], (double)h[i] / REP);
    return 0;
}
