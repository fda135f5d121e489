// SE3Quat on the device (Thirdparty/g2o/g2o/types/se3quat.h), shared by LocalBA and
// PoseOptimization.  Same operation order as the oracle (Eigen's quaternion formulas).
#pragma once

#include <hip/hip_runtime.h>

struct Q4 { double x, y, z, w; };

__device__ __forceinline__ Q4 q_from_R(const double* m) {   // Eigen::Quaterniond(Matrix3d)
    Q4 q;
    const double t = m[0] + m[4] + m[8];
    if (t > 0) {
        double s = sqrt(t + 1.0);
        q.w = 0.5 * s;
        s = 0.5 / s;
        q.x = (m[7] - m[5]) * s;
        q.y = (m[2] - m[6]) * s;
        q.z = (m[3] - m[1]) * s;
    } else {   // the largest diagonal i, (j, k) = (i+1, i+2) mod 3, spelled out per i
        const int i = m[4] > m[0] ? (m[8] > m[4] ? 2 : 1) : (m[8] > m[0] ? 2 : 0);
        if (i == 0) {
            double s = sqrt(m[0] - m[4] - m[8] + 1.0);
            q.x = 0.5 * s;
            s = 0.5 / s;
            q.w = (m[7] - m[5]) * s;
            q.y = (m[3] + m[1]) * s;
            q.z = (m[6] + m[2]) * s;
        } else if (i == 1) {
            double s = sqrt(m[4] - m[8] - m[0] + 1.0);
            q.y = 0.5 * s;
            s = 0.5 / s;
            q.w = (m[2] - m[6]) * s;
            q.z = (m[7] + m[5]) * s;
            q.x = (m[1] + m[3]) * s;
        } else {
            double s = sqrt(m[8] - m[0] - m[4] + 1.0);
            q.z = 0.5 * s;
            s = 0.5 / s;
            q.w = (m[3] - m[1]) * s;
            q.x = (m[2] + m[6]) * s;
            q.y = (m[5] + m[7]) * s;
        }
    }
    return q;
}
__device__ __forceinline__ void q_normalize_pos(Q4& q) {   // SE3Quat::normalizeRotation
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    if (n > 0) {   // one division, four multiplies (Eigen divides each: <= 1 ulp apart)
        const double in = 1.0 / n;
        q.x *= in; q.y *= in; q.z *= in; q.w *= in;
    }
}
__host__ __device__ __forceinline__ void q_to_R(const double* q4, double* R) {   // toRotationMatrix
    const double x = q4[0], y = q4[1], z = q4[2], w = q4[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
__device__ __forceinline__ void q_rotate(const double* q4, const double* v, double* o) {   // Eigen q*v
    const double qx = q4[0], qy = q4[1], qz = q4[2], qw = q4[3];
    double uv[3] = {qy * v[2] - qz * v[1], qz * v[0] - qx * v[2], qx * v[1] - qy * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const double c[3] = {qy * uv[2] - qz * uv[1], qz * uv[0] - qx * uv[2], qx * uv[1] - qy * uv[0]};
    for (int i = 0; i < 3; i++) o[i] = v[i] + qw * uv[i] + c[i];
}
__device__ __forceinline__ void se3_map(const double* q4, const double* t3, const double* X, double* o) {
    q_rotate(q4, X, o);
    o[0] += t3[0]; o[1] += t3[1]; o[2] += t3[2];
}
// pose <- SE3Quat::exp(upd) * pose   (se3quat.h:217-257, :99-105)
__device__ void se3_exp_update(const double* upd, double* q4, double* t3) {
    const double w0 = upd[0], w1 = upd[1], w2 = upd[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += O[3 * i + k] * O[3 * k + j];
            O2[3 * i + j] = s;
        }
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        double s, c;   // one sincos
        sincos(theta, &s, &c);
        const double it = 1.0 / theta;   // one division for a, b, d (<= 2 ulp from the reference's)
        const double a = s * it, b = (1 - c) * (it * it), d = (theta - s) * (it * it * it);
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * O[i] + b * O2[i];
        for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0 ? 1.0 : 0.0) + b * O[i] + d * O2[i];
    }
    Q4 E = q_from_R(R);
    q_normalize_pos(E);
    const double Eq[4] = {E.x, E.y, E.z, E.w};
    double Et[3];
    for (int i = 0; i < 3; i++) Et[i] = V[3 * i] * upd[3] + V[3 * i + 1] * upd[4] + V[3 * i + 2] * upd[5];
    double rt[3];
    q_rotate(Eq, t3, rt);
    for (int i = 0; i < 3; i++) t3[i] = Et[i] + rt[i];
    const double ax = E.x, ay = E.y, az = E.z, aw = E.w;
    const double bx = q4[0], by = q4[1], bz = q4[2], bw = q4[3];
    Q4 r{aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
         aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz};
    q_normalize_pos(r);
    q4[0] = r.x; q4[1] = r.y; q4[2] = r.z; q4[3] = r.w;
}

