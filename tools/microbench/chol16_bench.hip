// The LocalBA diagonal-tile Cholesky + inverse alone on one wavefront: chol16_factor (lba.hip,
// the round-4 form) against chol16_pipe (lba_chol16.inc, tools/gen_chol16.py), cycles by s_memtime
// and the largest difference of the factors. Built against the library's sources:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../include -I../../orb-slam2-noted_amd/csrc
//         -I../../orb-slam2-noted_amd/build chol16_bench.hip -o chol16_bench
#include "lba.hip"
#include <cstdio>
#include <cmath>
using namespace lbaamd;
template <int V, bool COLD> __global__ void kb(const double *A, double *L, double *Li, long long *cyc, int lim) {
    const int lane = threadIdx.x, i = lane & 15;
    double row[16], li[16];
#pragma unroll
    for (int c = 0; c < 16; c++) row[c] = c <= i ? A[i * 16 + c] : 0.0;
    bool bad = false;
    if (COLD) asm volatile("s_icache_inv\n\ts_nop 15\n\ts_nop 15" ::: "memory");   // the code below fetched cold (from L2)
    long long t0 = clock64();
    if constexpr (V == 0) {
#pragma unroll
        for (int r = 0; r < 16; r++) li[r] = 0.0;
        chol16_factor<0, false>(row, li, i, lim, bad);
    } else {
#pragma unroll
        for (int r = 0; r < 16; r++) li[r] = r == i ? 1.0 : 0.0;
        chol16_pipe(row, li, lim, bad);
    }
    long long t1 = clock64();
    if (lane < 16) {
        for (int c = 0; c < 16; c++) L[i * 16 + c] = row[c];
        for (int r = 0; r < 16; r++) Li[r * 16 + i] = li[r];
    }
    if (lane == 0) cyc[0] = t1 - t0 + (bad ? 1000000000LL : 0);
}
int main() {
    double hA[256];
    srand(3);
    double M[256];
    for (int k = 0; k < 256; k++) M[k] = (rand() / (double)RAND_MAX) - 0.5;
    for (int r = 0; r < 16; r++)
        for (int c = 0; c < 16; c++) {
            double s = r == c ? 4.0 : 0.0;
            for (int k = 0; k < 16; k++) s += M[r * 16 + k] * M[c * 16 + k];
            hA[r * 16 + c] = s;
        }
    double *A, *L, *Li; long long *cy;
    (void)hipMalloc(&A, 2048); (void)hipMalloc(&L, 2048 * 2); (void)hipMalloc(&Li, 2048 * 2); (void)hipMalloc(&cy, 64);
    (void)hipMemcpy(A, hA, 2048, hipMemcpyHostToDevice);
    double hL[2][256], hLi[2][256];
    for (int cold = 0; cold < 2; cold++)
    for (int lim : {16, 9}) {
        long long best[2] = {1LL << 60, 1LL << 60};
        for (int rep = 0; rep < 20; rep++) {
            long long c;
            if (cold) kb<0, true><<<1, 64>>>(A, L, Li, cy, lim); else kb<0, false><<<1, 64>>>(A, L, Li, cy, lim);
            (void)hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost);
            best[0] = c < best[0] ? c : best[0];
            (void)hipMemcpy(hL[0], L, 2048, hipMemcpyDeviceToHost); (void)hipMemcpy(hLi[0], Li, 2048, hipMemcpyDeviceToHost);
            if (cold) kb<1, true><<<1, 64>>>(A, L + 256, Li + 256, cy + 1, lim); else kb<1, false><<<1, 64>>>(A, L + 256, Li + 256, cy + 1, lim);
            (void)hipMemcpy(&c, cy + 1, 8, hipMemcpyDeviceToHost);
            best[1] = c < best[1] ? c : best[1];
            (void)hipMemcpy(hL[1], L + 256, 2048, hipMemcpyDeviceToHost); (void)hipMemcpy(hLi[1], Li + 256, 2048, hipMemcpyDeviceToHost);
        }
        double dl = 0, dli = 0;
        for (int r = 0; r < lim; r++)
            for (int c = 0; c <= r; c++) {
                dl = fmax(dl, fabs(hL[0][r * 16 + c] - hL[1][r * 16 + c]));
                dli = fmax(dli, fabs(hLi[0][r * 16 + c] - hLi[1][r * 16 + c]));
            }
        printf("%s lim=%d chol16_factor %lld cyc, chol16_pipe %lld cyc, max|dL| %.3g max|dLinv| %.3g\n", cold ? "icache-cold" : "warm", lim, best[0], best[1], dl, dli);
    }
    return 0;
}
