// SE3Quat / Eigen quaternion helpers shared by the LocalBA and PoseOptimization kernels
// (g2o se3quat.h:60-285, Eigen Quaternion(Matrix3) + _transformVector), FP64.
#pragma once
#include <hip/hip_runtime.h>

namespace g2oamd {

struct Pose { double q[4]; double t[3]; double pad; };   // q = (x, y, z, w)

__host__ __device__ inline void quat_rotate(const double q[4], const double v[3], double o[3]) {
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const double cx = q[1] * uv[2] - q[2] * uv[1], cy = q[2] * uv[0] - q[0] * uv[2], cz = q[0] * uv[1] - q[1] * uv[0];
    o[0] = v[0] + q[3] * uv[0] + cx;
    o[1] = v[1] + q[3] * uv[1] + cy;
    o[2] = v[2] + q[3] * uv[2] + cz;
}

__host__ __device__ inline void quat_to_R(const double q[4], double R[9]) {
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

// Eigen::Quaternion(const Matrix3&) + SE3Quat::normalizeRotation
__host__ __device__ inline void quat_from_R_norm(const double m[9], double q[4]) {
    double t = m[0] + m[4] + m[8];
    double c[3], w;
    if (t > 0) {
        t = sqrt(t + 1.0);
        w = 0.5 * t;
        t = 0.5 / t;
        c[0] = (m[7] - m[5]) * t;
        c[1] = (m[2] - m[6]) * t;
        c[2] = (m[3] - m[1]) * t;
    } else {
        // branches spelled out per pivot i (j = i+1, k = i+2 mod 3) so no array is indexed
        // dynamically (a dynamically indexed local lands in scratch memory on the GPU)
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > (i == 0 ? m[0] : m[4])) i = 2;
        if (i == 0) {        // j = 1, k = 2
            t = sqrt(m[0] - m[4] - m[8] + 1.0);
            c[0] = 0.5 * t;
            t = 0.5 / t;
            w = (m[7] - m[5]) * t;
            c[1] = (m[3] + m[1]) * t;
            c[2] = (m[6] + m[2]) * t;
        } else if (i == 1) { // j = 2, k = 0
            t = sqrt(m[4] - m[8] - m[0] + 1.0);
            c[1] = 0.5 * t;
            t = 0.5 / t;
            w = (m[2] - m[6]) * t;
            c[2] = (m[7] + m[5]) * t;
            c[0] = (m[1] + m[3]) * t;
        } else {             // j = 0, k = 1
            t = sqrt(m[8] - m[0] - m[4] + 1.0);
            c[2] = 0.5 * t;
            t = 0.5 / t;
            w = (m[3] - m[1]) * t;
            c[0] = (m[2] + m[6]) * t;
            c[1] = (m[5] + m[7]) * t;
        }
    }
    if (w < 0) { c[0] = -c[0]; c[1] = -c[1]; c[2] = -c[2]; w = -w; }
    const double n = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2] + w * w);
    q[0] = c[0] / n; q[1] = c[1] / n; q[2] = c[2] / n; q[3] = w / n;
}

__device__ inline void pose_map(const Pose &T, const double X[3], double o[3]) {
    quat_rotate(T.q, X, o);
    o[0] += T.t[0]; o[1] += T.t[1]; o[2] += T.t[2];
}

// exp(u) * T  (VertexSE3Expmap::oplusImpl, se3quat.h:223-257 + operator*)
__device__ inline Pose pose_oplus(const Pose &T, const double u[6]) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9], R[9], V[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) { R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i]; V[i] = R[i]; }
    } else {
        const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        const double c = (theta - sin(theta)) / (theta * theta * theta);
        for (int i = 0; i < 9; i++) {
            const double I = i % 4 == 0 ? 1.0 : 0.0;
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + c * O2[i];
        }
    }
    double dq[4], dt[3];
    quat_from_R_norm(R, dq);
    for (int i = 0; i < 3; i++) dt[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
    Pose r;
    double rt[3];
    quat_rotate(dq, T.t, rt);
    r.t[0] = dt[0] + rt[0]; r.t[1] = dt[1] + rt[1]; r.t[2] = dt[2] + rt[2];
    const double *a = dq, *b = T.q;  // (x, y, z, w)
    double q[4];
    q[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    q[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    q[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    q[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    r.q[0] = q[0] / n; r.q[1] = q[1] / n; r.q[2] = q[2] / n; r.q[3] = q[3] / n;
    r.pad = 0;
    return r;
}

}  // namespace g2oamd
