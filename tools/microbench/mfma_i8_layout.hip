// Operand / accumulator lane maps of v_mfma_i32_16x16x64_i8 and v_mfma_i32_16x16x32_i8 on gfx950,
// checked with exact asymmetric integer data against a host product (the MFMA blur of
// fast_blur_kernel relies on them). Assumed maps: lane l holds A[m = l & 15][k = KL (l >> 4) + j]
// and B[k = KL (l >> 4) + j][n = l & 15] in byte j = 0..KL-1 of its fragment (KL = 16 for K = 64,
// 8 for K = 32); C/D element r of lane l is C[m = 4 (l >> 4) + r][n = l & 15].
// Build: hipcc -O2 --offload-arch=gfx950 -o mfma_i8_layout mfma_i8_layout.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));

// K = 32 form: 8 bytes per lane; A is read as the first 32 columns of the K = 64 data
__global__ void probe32(const int8_t *A, const int8_t *B, const int *C0, int *D) {
    const int l = threadIdx.x, m = l & 15, g = l >> 4;
    long a = 0, b = 0;
    int8_t *pa = (int8_t *)&a, *pb = (int8_t *)&b;
    for (int j = 0; j < 8; j++) {
        pa[j] = A[m * 64 + 8 * g + j];
        pb[j] = B[(8 * g + j) * 16 + m];
    }
    i32x4 c;
    for (int r = 0; r < 4; r++) c[r] = C0[(4 * g + r) * 16 + m];
    c = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[(4 * g + r) * 16 + m] = c[r];
}

__global__ void probe(const int8_t *A, const int8_t *B, const int *C0, int *D) {
    const int l = threadIdx.x, m = l & 15, g = l >> 4;
    i32x4 a, b;
    int8_t *pa = (int8_t *)&a, *pb = (int8_t *)&b;
    for (int j = 0; j < 16; j++) {
        pa[j] = A[m * 64 + 16 * g + j];
        pb[j] = B[(16 * g + j) * 16 + m];
    }
    i32x4 c;
    for (int r = 0; r < 4; r++) c[r] = C0[(4 * g + r) * 16 + m];
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(*(long long __attribute__((ext_vector_type(2))) *)&a,
                                              *(long long __attribute__((ext_vector_type(2))) *)&b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[(4 * g + r) * 16 + m] = c[r];
}

int main() {
    int8_t hA[16 * 64], hB[64 * 16];
    int hC[256], hD[256], ref[256];
    for (int m = 0; m < 16; m++)
        for (int k = 0; k < 64; k++) hA[m * 64 + k] = (int8_t)((m * 7 + k * 3 + (m * k) % 5) % 255 - 127);
    for (int k = 0; k < 64; k++)
        for (int n = 0; n < 16; n++) hB[k * 16 + n] = (int8_t)((k * 11 + n * 5 + (k ^ n)) % 253 - 126);
    for (int i = 0; i < 256; i++) hC[i] = i * 1000 - 77;
    for (int m = 0; m < 16; m++)
        for (int n = 0; n < 16; n++) {
            int s = hC[m * 16 + n];
            for (int k = 0; k < 64; k++) s += hA[m * 64 + k] * hB[k * 16 + n];
            ref[m * 16 + n] = s;
        }
    int8_t *dA, *dB;
    int *dC, *dD;
    if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dC, sizeof hC) || hipMalloc(&dD, sizeof hD))
        return 2;
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(dA, dB, dC, dD);
    if (hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int bad = 0;
    for (int i = 0; i < 256; i++) bad += hD[i] != ref[i];
    int ref32[256];
    for (int m = 0; m < 16; m++)
        for (int n = 0; n < 16; n++) {
            int s = hC[m * 16 + n];
            for (int k = 0; k < 32; k++) s += hA[m * 64 + k] * hB[k * 16 + n];
            ref32[m * 16 + n] = s;
        }
    probe32<<<1, 64>>>(dA, dB, dC, dD);
    if (hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int bad32 = 0;
    for (int i = 0; i < 256; i++) bad32 += hD[i] != ref32[i];
    printf("{\"mfma_i32_16x16x64_i8_layout_mismatches\": %d, \"mfma_i32_16x16x32_i8_layout_mismatches\": %d}\n", bad, bad32);
    return bad || bad32 ? 1 : 0;
}
