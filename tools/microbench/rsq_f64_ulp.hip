// v_rsq_f64's error against the correctly rounded 1 / sqrt(x) (long double on the host), over
// random doubles spread across exponents 2^-60 .. 2^60 and the Cholesky pivots' range: is the
// Newton step after it in chol16_pipe (lba_chol16.inc) needed for accuracy?
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/rsq_f64_ulp.hip -o tools/microbench/rsq_f64_ulp
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

__global__ void rsq(const double *x, double *y, double *yn, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    const double r = __builtin_amdgcn_rsq(d);
    y[i] = r;
    const double h = 0.5 * d;
    yn[i] = __builtin_fma(r, __builtin_fma(-(h * r), r, 0.5), r);   // the product's one Newton step
}

static double ulp_err(double got, long double want) {
    const double w = (double)want;
    const double u = std::nextafter(w, INFINITY) - w;
    return (double)(((long double)got - want) / (long double)u);
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), y(n), yn(n);
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> m(1.0, 2.0);
    std::uniform_int_distribution<int> e(-60, 60);
    for (int i = 0; i < n; i++) x[i] = std::ldexp(m(rng), e(rng));
    double *dx, *dy, *dyn;
    hipMalloc(&dx, n * 8); hipMalloc(&dy, n * 8); hipMalloc(&dyn, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    rsq<<<n / 256, 256>>>(dx, dy, dyn, n);
    hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(yn.data(), dyn, n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0;
    long ex0 = 0, ex1 = 0;
    for (int i = 0; i < n; i++) {
        const long double w = 1.0L / std::sqrt((long double)x[i]);
        const double a = std::fabs(ulp_err(y[i], w)), b = std::fabs(ulp_err(yn[i], w));
        m0 = std::max(m0, a); m1 = std::max(m1, b);
        ex0 += a < 0.5; ex1 += b < 0.5;
    }
    printf("{\"inputs\": %d, \"rsq_max_ulp\": %.3f, \"rsq_correctly_rounded_frac\": %.4f, "
           "\"rsq_newton_max_ulp\": %.3f, \"rsq_newton_correctly_rounded_frac\": %.4f}\n",
           n, m0, (double)ex0 / n, m1, (double)ex1 / n);
    return 0;
}
