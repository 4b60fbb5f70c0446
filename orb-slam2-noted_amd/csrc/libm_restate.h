// libm functions the triangulation of LocalMapping::CreateNewMapPoints calls, restated so the
// GPU returns the host's bits (compiled as HIP for the device and as C by the pin tool
// oracle/tools/check_atan2f_hypot.c, which compares them with the live glibc):
//   * atan2f(y, x) -- glibc 2.35 sysdeps/ieee754/flt-32/e_atan2f.c + s_atanf.c, the fdlibm float
//     algorithm (argument reduction into 4 intervals, 11-term odd/even polynomial in float);
//   * hypot(x, y) -- glibc 2.35 sysdeps/ieee754/dbl-64/e_hypot.c (scaling + Borges' corrected
//     kernel without FMA, as the x86-64 baseline build compiles it).
// Both are evaluated with -ffp-contract=off (every float / double operation rounded on its own).
#ifndef ORB_LIBM_RESTATE_H
#define ORB_LIBM_RESTATE_H
#include <stdint.h>
#ifdef __HIPCC__
#define LM_FN __host__ __device__ static inline
#else
#include <math.h>
#include <string.h>
#define LM_FN static inline
#endif

LM_FN float lm_f(uint32_t u) {
    float f;
#ifdef __HIPCC__
    f = __builtin_bit_cast(float, u);
#else
    memcpy(&f, &u, 4);
#endif
    return f;
}
LM_FN uint32_t lm_u(float f) {
#ifdef __HIPCC__
    return __builtin_bit_cast(uint32_t, f);
#else
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
#endif
}

LM_FN float lm_atanf(float x) {
    // the source's decimal literals (converted double -> float as the C compiler does)
    const float atanhi[4] = {(float)4.6364760399e-01, (float)7.8539812565e-01, (float)9.8279368877e-01,
                             (float)1.5707962513e+00};
    const float atanlo[4] = {(float)5.0121582440e-09, (float)3.7748947079e-08, (float)3.4473217170e-08,
                             (float)7.5497894159e-08};
    const float aT[11] = {(float)3.3333334327e-01, (float)-2.0000000298e-01, (float)1.4285714924e-01,
                          (float)-1.1111110449e-01, (float)9.0908870101e-02, (float)-7.6918758452e-02,
                          (float)6.6610731184e-02, (float)-5.8335702866e-02, (float)4.9768779427e-02,
                          (float)-3.6531571299e-02, (float)1.6285819933e-02};
    const float one = 1.0f;
    const int32_t hx = (int32_t)lm_u(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {   // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        const float z = atanhi[3] + atanlo[3];
        return hx > 0 ? z : -z;
    }
    if (ix < 0x3ee00000) {    // |x| < 0.4375
        if (ix < 0x31000000) return x;   // |x| < 2^-29
        id = -1;
    } else {
        x = lm_f((uint32_t)ix);   // fabsf
        if (ix < 0x3f980000) {        // |x| < 1.1875
            if (ix < 0x3f300000) {    // 7/16 <= |x| < 11/16
                id = 0;
                x = ((float)2.0 * x - one) / ((float)2.0 + x);
            } else {                  // 11/16 <= |x| < 19/16
                id = 1;
                x = (x - one) / (x + one);
            }
        } else {
            if (ix < 0x401c0000) {    // |x| < 2.4375
                id = 2;
                x = (x - (float)1.5) / (one + (float)1.5 * x);
            } else {                  // 2.4375 <= |x| < 2^25
                id = 3;
                x = -(float)1.0 / x;
            }
        }
    }
    float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -z : z;
}

LM_FN float lm_atan2f(float y, float x) {
    const float tiny = (float)1.0e-30, pi_o_4 = (float)7.8539818525e-01, pi_o_2 = (float)1.5707963705e+00,
                pi = (float)3.1415927410e+00, pi_lo = (float)-8.7422776573e-08;
    const int32_t hx = (int32_t)lm_u(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)lm_u(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return lm_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return (float)3.0 * pi_o_4 + tiny;
                default: return (float)-3.0 * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + (float)0.5 * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else {
        const float q = y / x;
        z = lm_atanf(lm_f(lm_u(q) & 0x7fffffffu));   // fabsf
    }
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// glibc 2.35 hypot (sysdeps/ieee754/dbl-64/e_hypot.c, x86-64 baseline build: the non-FMA
// kernel of Borges' corrected algorithm), finite inputs
LM_FN double lm_hypot_kernel(double ax, double ay) {
    double h = sqrt(ax * ax + ay * ay), t1, t2;
    if (h <= 2.0 * ay) {
        const double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        const double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

LM_FN double lm_hypot(double x, double y) {
    x = x < 0 ? -x : x;
    y = y < 0 ? -y : y;
    const double ax = x < y ? y : x, ay = x < y ? x : y;
    const double SCALE = 0x1p-600, EPS = 0x1p-54;
    if (ax > 0x1p+511) {
        if (ay <= ax * EPS) return ax + ay;
        return lm_hypot_kernel(ax * SCALE, ay * SCALE) / SCALE;
    }
    if (ay < 0x1p-459) {
        if (ax >= ay / EPS) return ax + ay;
        return lm_hypot_kernel(ax / SCALE, ay / SCALE) * SCALE;
    }
    if (ay <= ax * EPS) return ax + ay;
    return lm_hypot_kernel(ax, ay);
}

#endif
