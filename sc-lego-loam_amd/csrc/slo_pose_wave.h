// slo_pose_wave.h — the per-scan pose algebra of slo_pose.h run by one wave,
// for the kernels where one stream's scalar chain is the latency
// (k_fa_odo_finish).  The reference expressions are unchanged; only the
// independent trig calls run side by side: lane k evaluates sinf_ / cosf_ (or
// a double sin / cos / atan2) of input k, every lane receives every result,
// and the expressions then read those values where the scalar form calls the
// function again on the same argument — the same bits, in the same order
// (`-ffp-contract=off`, no fast-math).  A scalar call is ~0.7 us on one lane
// (the glibc tables are memory loads), so the chain of ~50 calls of
// integrate + transformFusion (53 us per scan) becomes ~15 rounds.
//   accumulate_rotation_w  featureAssociation.cpp:1015-1032
//   plugin_imu_rotation_w  featureAssociation.cpp:955-1013
//   integrate_w            featureAssociation.cpp:1697-1725
//   odom_handoff_w         featureAssociation.cpp:1728-1734 -> mapOptmization.cpp:658-666
//   associate_to_map_w     mapOptmization.cpp:397-482
// Every lane of the wave must call these together (shuffles); every lane
// returns the results.
#pragma once

#include "slo_pose.h"

namespace slo_pose {

// sinf_ / cosf_ of a[0..N) (lane k: a[k]), to every lane
template <int N>
__device__ inline void wave_sincos(const float (&a)[N], float (&s)[N], float (&c)[N]) {
    const int lane = threadIdx.x & 63;
    float x = a[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (lane == k) x = a[k];
    const float sv = sinf_(x), cv = cosf_(x);
#pragma unroll
    for (int k = 0; k < N; ++k) {
        s[k] = __shfl(sv, k, 64);
        c[k] = __shfl(cv, k, 64);
    }
}

// atan2f_(y0, x0) and atan2f_(y1, x1) on lanes 0 and 1
__device__ inline void wave_atan2f_2(float y0, float x0, float y1, float x1, float& r0, float& r1) {
    const bool one = (threadIdx.x & 63) == 1;
    const float r = atan2f_(one ? y1 : y0, one ? x1 : x0);
    r0 = __shfl(r, 0, 64);
    r1 = __shfl(r, 1, 64);
}

__device__ inline void accumulate_rotation_w(float scx, float ccx, float scy, float ccy, float scz, float ccz, float slx,
                                             float clx, float sly, float cly, float slz, float clz, float& ox, float& oy,
                                             float& oz) {
    float srx = clx * ccx * sly * scz - ccx * ccz * slx - clx * cly * scx;
    ox = -asinf_(srx);
    float srycrx = slx * (ccy * scz - ccz * scx * scy) +
                   clx * sly * (ccy * ccz + scx * scy * scz) + clx * cly * ccx * scy;
    float crycrx = clx * cly * ccx * ccy - clx * sly * (ccz * scy - ccy * scx * scz) -
                   slx * (scy * scz + ccy * ccz * scx);
    float srzcrx = scx * (clz * sly - cly * slx * slz) +
                   ccx * scz * (cly * clz + slx * sly * slz) + clx * ccx * ccz * slz;
    float crzcrx = clx * clz * ccx * ccz - ccx * scz * (cly * slz - clz * slx * sly) -
                   scx * (sly * slz + cly * clz * slx);
    const float cox = cosf_(ox);
    wave_atan2f_2(srycrx / cox, crycrx / cox, srzcrx / cox, crzcrx / cox, oy, oz);
}

__device__ inline void plugin_imu_rotation_w(float sbcx, float cbcx, float sbcy, float cbcy, float sbcz, float cbcz,
                                             float sblx, float cblx, float sbly, float cbly, float sblz, float cblz,
                                             float salx, float calx, float saly, float caly, float salz, float calz,
                                             float& acx, float& acy, float& acz) {
    float srx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
                cbcx * cbcz * (calx * saly * (cbly * sblz - cblz * sblx * sbly) - calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                cbcx * sbcz * (calx * caly * (cblz * sbly - cbly * sblx * sblz) - calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
    acx = -asinf_(srx);
    float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * (calx * saly * (cbly * sblz - cblz * sblx * sbly) - calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                   (cbcy * cbcz + sbcx * sbcy * sbcz) * (calx * caly * (cblz * sbly - cbly * sblx * sblz) - calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) +
                   cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
    float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * (calx * caly * (cblz * sbly - cbly * sblx * sblz) - calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) -
                   (sbcy * sbcz + cbcy * cbcz * sbcx) * (calx * saly * (cbly * sblz - cblz * sblx * sbly) - calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) +
                   cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
    float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) - cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                   cbcx * cbcz * ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) + (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) - calx * cblx * cblz * salz) +
                   cbcx * sbcz * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) + (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) + calx * cblx * salz * sblz);
    float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) - cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                   cbcx * cbcz * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) + (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) + calx * calz * cblx * cblz) -
                   cbcx * sbcz * ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) + (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) - calx * calz * cblx * sblz);
    const float cacx = cosf_(acx);
    wave_atan2f_2(srycrx / cacx, crycrx / cacx, srzcrx / cacx, crzcrx / cacx, acy, acz);
}

// integrate (slo_pose.h) into out[6] (sum is only read)
__device__ inline void integrate_w(const float* sum, const float* cur, const float* imu, float* out) {
    const float a[12] = {sum[0], sum[1], sum[2], -cur[0], -cur[1], -cur[2], imu[3], imu[4], imu[5], imu[6], imu[7], imu[8]};
    float S[12], C[12];
    wave_sincos<12>(a, S, C);
    float rx, ry, rz, tx, ty, tz;
    accumulate_rotation_w(S[0], C[0], S[1], C[1], S[2], C[2], S[3], C[3], S[4], C[4], S[5], C[5], rx, ry, rz);
    const float b[3] = {rx, ry, rz};
    float S2[3], C2[3];
    wave_sincos<3>(b, S2, C2);
    const float sx = imu[0], sy = imu[1], sz = imu[2];  // imuShiftFromStart*
    float x1 = C2[2] * (cur[3] - sx) - S2[2] * (cur[4] - sy);
    float y1 = S2[2] * (cur[3] - sx) + C2[2] * (cur[4] - sy);
    float z1 = cur[5] - sz;
    float x2 = x1;
    float y2 = C2[0] * y1 - S2[0] * z1;
    float z2 = S2[0] * y1 + C2[0] * z1;
    tx = sum[3] - (C2[1] * x2 + S2[1] * z2);
    ty = sum[4] - y2;
    tz = sum[5] - (-S2[1] * x2 + C2[1] * z2);
    plugin_imu_rotation_w(S2[0], C2[0], S2[1], C2[1], S2[2], C2[2], S[6], C[6], S[7], C[7], S[8], C[8], S[9], C[9],
                          S[10], C[10], S[11], C[11], rx, ry, rz);
    out[0] = rx; out[1] = ry; out[2] = rz;
    out[3] = tx; out[4] = ty; out[5] = tz;
}

// odom_handoff (slo_pose.h): tf_quat_rpy's three double sin / cos pairs and
// tf_rpy_of's two atan2 side by side
__device__ inline void odom_handoff_w(const float ts[6], float out[6]) {
    const int lane = threadIdx.x & 63;
    const double roll = (double)ts[2], pitch = (double)(-ts[0]), yaw = (double)(-ts[1]);
    const double h = lane == 0 ? yaw * 0.5 : (lane == 1 ? pitch * 0.5 : roll * 0.5);
    const double cv = slo_libm::cos_d(h), sv = slo_libm::sin_d(h);
    const double cy = __shfl(cv, 0, 64), sy = __shfl(sv, 0, 64);
    const double cp = __shfl(cv, 1, 64), sp = __shfl(sv, 1, 64);
    const double cr = __shfl(cv, 2, 64), sr = __shfl(sv, 2, 64);
    double q[4];
    q[0] = sr * cp * cy - cr * sp * sy;
    q[1] = cr * sp * cy + sr * cp * sy;
    q[2] = cr * cp * sy - sr * sp * cy;
    q[3] = cr * cp * cy + sr * sp * sy;
    // tf_rpy_of
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double k = 2.0 / (x * x + y * y + z * z + w * w);
    const double xs = x * k, ys = y * k, zs = z * k;
    const double r00 = 1.0 - (y * ys + z * zs), r01 = x * ys - w * zs, r02 = x * zs + w * ys;
    const double r10 = x * ys + w * zs;
    const double r20 = x * zs - w * ys, r21 = y * zs + w * xs, r22 = 1.0 - (x * xs + y * ys);
    double r, p, yw;
    if (fabs(r20) >= 1.0) {   // pitch at +-90 deg
        yw = 0.0;
        const double delta = slo_libm::atan2_d(r01, r02);
        p = r20 > 0 ? M_PI / 2.0 : -M_PI / 2.0;
        r = (r20 > 0 ? p : -p) + delta;
    } else {
        p = -slo_libm::asin_d(r20);
        const double c = slo_libm::cos_d(p);
        const double a = lane == 1 ? slo_libm::atan2_d(r10 / c, r00 / c) : slo_libm::atan2_d(r21 / c, r22 / c);
        r = __shfl(a, 0, 64);
        yw = __shfl(a, 1, 64);
    }
    out[0] = (float)(-p);
    out[1] = (float)(-yw);
    out[2] = (float)r;
    for (int i = 3; i < 6; ++i) out[i] = ts[i];
}

__device__ inline void associate_to_map_w(const float* sum, const float* bef, const float* aft, float* incre, float* tbm) {
    const float a[9] = {sum[0], sum[1], sum[2], bef[0], bef[1], bef[2], aft[0], aft[1], aft[2]};
    float S[9], C[9];
    wave_sincos<9>(a, S, C);
    float x1 = C[1] * (bef[3] - sum[3]) - S[1] * (bef[5] - sum[5]);
    float y1 = bef[4] - sum[4];
    float z1 = S[1] * (bef[3] - sum[3]) + C[1] * (bef[5] - sum[5]);
    float x2 = x1;
    float y2 = C[0] * y1 + S[0] * z1;
    float z2 = -S[0] * y1 + C[0] * z1;
    incre[3] = C[2] * x2 + S[2] * y2;
    incre[4] = -S[2] * x2 + C[2] * y2;
    incre[5] = z2;
    const float sbcx = S[0], cbcx = C[0], sbcy = S[1], cbcy = C[1], sbcz = S[2], cbcz = C[2];
    const float sblx = S[3], cblx = C[3], sbly = S[4], cbly = C[4], sblz = S[5], cblz = C[5];
    const float salx = S[6], calx = C[6], saly = S[7], caly = C[7], salz = S[8], calz = C[8];
    float srx = -sbcx * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz) -
                cbcx * sbcy * (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                cbcx * cbcy * (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx);
    tbm[0] = -asinf_(srx);
    float srycrx = sbcx * (cblx * cblz * (caly * salz - calz * salx * saly) - cblx * sblz * (caly * calz + salx * saly * salz) + calx * saly * sblx) -
                   cbcx * cbcy * ((caly * calz + salx * saly * salz) * (cblz * sbly - cbly * sblx * sblz) + (caly * salz - calz * salx * saly) * (sbly * sblz + cbly * cblz * sblx) - calx * cblx * cbly * saly) +
                   cbcx * sbcy * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) + (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) + calx * cblx * saly * sbly);
    float crycrx = sbcx * (cblx * sblz * (calz * saly - caly * salx * salz) - cblx * cblz * (saly * salz + caly * calz * salx) + calx * caly * sblx) +
                   cbcx * cbcy * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) + (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) + calx * caly * cblx * cbly) -
                   cbcx * sbcy * ((saly * salz + caly * calz * salx) * (cbly * sblz - cblz * sblx * sbly) + (calz * saly - caly * salx * salz) * (cbly * cblz + sblx * sbly * sblz) - calx * caly * cblx * sbly);
    float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) -
                   (cbcy * cbcz + sbcx * sbcy * sbcz) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) +
                   cbcx * sbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
    float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                   (sbcy * sbcz + cbcy * cbcz * sbcx) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) +
                   cbcx * cbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
    const float c0 = cosf_(tbm[0]);
    wave_atan2f_2(srycrx / c0, crycrx / c0, srzcrx / c0, crzcrx / c0, tbm[1], tbm[2]);
    const float b[3] = {tbm[2], tbm[0], tbm[1]};
    float S2[3], C2[3];
    wave_sincos<3>(b, S2, C2);
    x1 = C2[0] * incre[3] - S2[0] * incre[4];
    y1 = S2[0] * incre[3] + C2[0] * incre[4];
    z1 = incre[5];
    x2 = x1;
    y2 = C2[1] * y1 - S2[1] * z1;
    z2 = S2[1] * y1 + C2[1] * z1;
    tbm[3] = aft[3] - (C2[2] * x2 + S2[2] * z2);
    tbm[4] = aft[4] - y2;
    tbm[5] = aft[5] - (-S2[2] * x2 + C2[2] * z2);
}

}  // namespace slo_pose
