// slo_pose.h — scalar pose algebra of the FA / MO nodes for one GPU lane.
// All trig through slo_libm (glibc float bits); float evaluation order as
// in the reference expressions.
//   transform_to_start  featureAssociation.cpp:860-883
//   transform_to_end    featureAssociation.cpp:885-953 (the IMU terms from
//                       ImuEnd; without an IMU they are the reference's
//                       zero-IMU values, cos 1 / sin 0: Q17)
//   plugin_imu_rotation featureAssociation.cpp:955-1013
//   accumulate_rotation featureAssociation.cpp:1015-1032
//   integrate           featureAssociation.cpp:1697-1725
//   associate_to_map    mapOptmization.cpp:397-482
//   odom_handoff        featureAssociation.cpp:1728-1734 -> mapOptmization.cpp:658-666
//   keyframe_estimate   mapOptmization.cpp:1545-1556, 1588-1601
#pragma once

#include "slo_libm.h"
#include "slo_libm_d.h"

#if defined(__HIPCC__)
#define SLO_P_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define SLO_P_HD inline
#endif

namespace slo_pose {

using slo_libm::sinf_;
using slo_libm::cosf_;
using slo_libm::asinf_;
using slo_libm::atan2f_;

struct P4 { float x, y, z, w; };

SLO_P_HD P4 transform_to_start(P4 pi, const float* tc) {
    float s = 10 * (pi.w - (float)(int)pi.w);
    float rx = s * tc[0], ry = s * tc[1], rz = s * tc[2];
    float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
    float srx, crx, sry, cry, srz, crz;   // sin/cos pairs share one range reduction
    slo_libm::sincosf_(rx, &srx, &crx);
    slo_libm::sincosf_(ry, &sry, &cry);
    slo_libm::sincosf_(rz, &srz, &crz);
    float x1 = crz * (pi.x - tx) + srz * (pi.y - ty);
    float y1 = -srz * (pi.x - tx) + crz * (pi.y - ty);
    float z1 = (pi.z - tz);
    float x2 = x1;
    float y2 = crx * y1 + srx * z1;
    float z2 = -srx * y1 + crx * z1;
    P4 o;
    o.x = cry * x2 - sry * z2;
    o.y = y2;
    o.z = sry * x2 + cry * z2;
    o.w = pi.w;
    return o;
}

// The IMU terms of TransformToEnd as publishCloudsLast sees them:
// cos/sin of the scan's start angles (updateImuRollPitchYawStartSinCos),
// imuShiftFromStart*, and cos/sin of imu{Yaw,Pitch,Roll}Last (the reference
// evaluates these per point; one evaluation gives the same bits).  Without an
// IMU every angle and shift is 0.
struct ImuEnd {
    float cRS, cPS, cYS, sRS, sPS, sYS;   // start
    float shx, shy, shz;                  // imuShiftFromStart
    float cYL, sYL, cPL, sPL, cRL, sRL;   // last
};
SLO_P_HD ImuEnd imu_end(float rollStart, float pitchStart, float yawStart, const float* shift, float yawLast,
                        float pitchLast, float rollLast) {
    ImuEnd e;
    e.cRS = cosf_(rollStart); e.cPS = cosf_(pitchStart); e.cYS = cosf_(yawStart);
    e.sRS = sinf_(rollStart); e.sPS = sinf_(pitchStart); e.sYS = sinf_(yawStart);
    e.shx = shift[0]; e.shy = shift[1]; e.shz = shift[2];
    e.cYL = cosf_(yawLast); e.sYL = sinf_(yawLast);
    e.cPL = cosf_(pitchLast); e.sPL = sinf_(pitchLast);
    e.cRL = cosf_(rollLast); e.sRL = sinf_(rollLast);
    return e;
}

// tct = sin/cos of tc[0..2]: {srx, crx, sry, cry, srz, crz} (sincosf_)
SLO_P_HD P4 transform_to_end(P4 pi, const float* tc, const float* tct, const ImuEnd& im) {
    const float cosImuRollStart = im.cRS, cosImuPitchStart = im.cPS, cosImuYawStart = im.cYS;
    const float sinImuRollStart = im.sRS, sinImuPitchStart = im.sPS, sinImuYawStart = im.sYS;
    const float imuShiftFromStartX = im.shx, imuShiftFromStartY = im.shy, imuShiftFromStartZ = im.shz;
    float s = 10 * (pi.w - (float)(int)pi.w);
    float rx = s * tc[0], ry = s * tc[1], rz = s * tc[2];
    float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
    float srx, crx, sry, cry, srz, crz;   // sin/cos pairs share one range reduction
    slo_libm::sincosf_(rx, &srx, &crx);
    slo_libm::sincosf_(ry, &sry, &cry);
    slo_libm::sincosf_(rz, &srz, &crz);
    float x1 = crz * (pi.x - tx) + srz * (pi.y - ty);
    float y1 = -srz * (pi.x - tx) + crz * (pi.y - ty);
    float z1 = (pi.z - tz);
    float x2 = x1;
    float y2 = crx * y1 + srx * z1;
    float z2 = -srx * y1 + crx * z1;
    float x3 = cry * x2 - sry * z2;
    float y3 = y2;
    float z3 = sry * x2 + cry * z2;
    tx = tc[3]; ty = tc[4]; tz = tc[5];
    srx = tct[0]; crx = tct[1]; sry = tct[2]; cry = tct[3]; srz = tct[4]; crz = tct[5];
    float x4 = cry * x3 + sry * z3;
    float y4 = y3;
    float z4 = -sry * x3 + cry * z3;
    float x5 = x4;
    float y5 = crx * y4 - srx * z4;
    float z5 = srx * y4 + crx * z4;
    float x6 = crz * x5 - srz * y5 + tx;
    float y6 = srz * x5 + crz * y5 + ty;
    float z6 = z5 + tz;
    float x7 = cosImuRollStart * (x6 - imuShiftFromStartX) - sinImuRollStart * (y6 - imuShiftFromStartY);
    float y7 = sinImuRollStart * (x6 - imuShiftFromStartX) + cosImuRollStart * (y6 - imuShiftFromStartY);
    float z7 = z6 - imuShiftFromStartZ;
    float x8 = x7;
    float y8 = cosImuPitchStart * y7 - sinImuPitchStart * z7;
    float z8 = sinImuPitchStart * y7 + cosImuPitchStart * z7;
    float x9 = cosImuYawStart * x8 + sinImuYawStart * z8;
    float y9 = y8;
    float z9 = -sinImuYawStart * x8 + cosImuYawStart * z8;
    float x10 = im.cYL * x9 - im.sYL * z9;
    float y10 = y9;
    float z10 = im.sYL * x9 + im.cYL * z9;
    float x11 = x10;
    float y11 = im.cPL * y10 + im.sPL * z10;
    float z11 = -im.sPL * y10 + im.cPL * z10;
    P4 o;
    o.x = im.cRL * x11 + im.sRL * y11;
    o.y = -im.sRL * x11 + im.cRL * y11;
    o.z = z11;
    o.w = (float)(int)pi.w;
    return o;
}

SLO_P_HD void tc_trig(const float* tc, float* tct) {
    slo_libm::sincosf_(tc[0], &tct[0], &tct[1]);
    slo_libm::sincosf_(tc[1], &tct[2], &tct[3]);
    slo_libm::sincosf_(tc[2], &tct[4], &tct[5]);
}

SLO_P_HD P4 transform_to_end(P4 pi, const float* tc, const ImuEnd& im) {
    float tct[6];
    tc_trig(tc, tct);
    return transform_to_end(pi, tc, tct, im);
}

SLO_P_HD void plugin_imu_rotation(float bcx, float bcy, float bcz, float blx, float bly, float blz, float alx,
                                  float aly, float alz, float& acx, float& acy, float& acz) {
    float sbcx = sinf_(bcx), cbcx = cosf_(bcx), sbcy = sinf_(bcy), cbcy = cosf_(bcy), sbcz = sinf_(bcz), cbcz = cosf_(bcz);
    float sblx = sinf_(blx), cblx = cosf_(blx), sbly = sinf_(bly), cbly = cosf_(bly), sblz = sinf_(blz), cblz = cosf_(blz);
    float salx = sinf_(alx), calx = cosf_(alx), saly = sinf_(aly), caly = cosf_(aly), salz = sinf_(alz), calz = cosf_(alz);
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
    acy = atan2f_(srycrx / cosf_(acx), crycrx / cosf_(acx));
    float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) - cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                   cbcx * cbcz * ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) + (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) - calx * cblx * cblz * salz) +
                   cbcx * sbcz * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) + (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) + calx * cblx * salz * sblz);
    float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) - cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                   cbcx * cbcz * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) + (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) + calx * calz * cblx * cblz) -
                   cbcx * sbcz * ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) + (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) - calx * calz * cblx * sblz);
    acz = atan2f_(srzcrx / cosf_(acx), crzcrx / cosf_(acx));
}

SLO_P_HD void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz, float& ox, float& oy, float& oz) {
    float srx = cosf_(lx) * cosf_(cx) * sinf_(ly) * sinf_(cz) - cosf_(cx) * cosf_(cz) * sinf_(lx) - cosf_(lx) * cosf_(ly) * sinf_(cx);
    ox = -asinf_(srx);
    float srycrx = sinf_(lx) * (cosf_(cy) * sinf_(cz) - cosf_(cz) * sinf_(cx) * sinf_(cy)) +
                   cosf_(lx) * sinf_(ly) * (cosf_(cy) * cosf_(cz) + sinf_(cx) * sinf_(cy) * sinf_(cz)) + cosf_(lx) * cosf_(ly) * cosf_(cx) * sinf_(cy);
    float crycrx = cosf_(lx) * cosf_(ly) * cosf_(cx) * cosf_(cy) - cosf_(lx) * sinf_(ly) * (cosf_(cz) * sinf_(cy) - cosf_(cy) * sinf_(cx) * sinf_(cz)) -
                   sinf_(lx) * (sinf_(cy) * sinf_(cz) + cosf_(cy) * cosf_(cz) * sinf_(cx));
    oy = atan2f_(srycrx / cosf_(ox), crycrx / cosf_(ox));
    float srzcrx = sinf_(cx) * (cosf_(lz) * sinf_(ly) - cosf_(ly) * sinf_(lx) * sinf_(lz)) +
                   cosf_(cx) * sinf_(cz) * (cosf_(ly) * cosf_(lz) + sinf_(lx) * sinf_(ly) * sinf_(lz)) + cosf_(lx) * cosf_(cx) * cosf_(cz) * sinf_(lz);
    float crzcrx = cosf_(lx) * cosf_(lz) * cosf_(cx) * cosf_(cz) - cosf_(cx) * sinf_(cz) * (cosf_(ly) * sinf_(lz) - cosf_(lz) * sinf_(lx) * sinf_(ly)) -
                   sinf_(cx) * (sinf_(ly) * sinf_(lz) + cosf_(ly) * cosf_(lz) * sinf_(lx));
    oz = atan2f_(srzcrx / cosf_(ox), crzcrx / cosf_(ox));
}

// integrateTransformation: sum <- sum (+) cur; imu = {imuShiftFromStart x, y,
// z, imuPitchStart, imuYawStart, imuRollStart, imuPitchLast, imuYawLast,
// imuRollLast} (all 0 without an IMU)
SLO_P_HD void integrate(float* sum, const float* cur, const float* imu) {
    float rx, ry, rz, tx, ty, tz;
    accumulate_rotation(sum[0], sum[1], sum[2], -cur[0], -cur[1], -cur[2], rx, ry, rz);
    const float sx = imu[0], sy = imu[1], sz = imu[2];  // imuShiftFromStart*
    float x1 = cosf_(rz) * (cur[3] - sx) - sinf_(rz) * (cur[4] - sy);
    float y1 = sinf_(rz) * (cur[3] - sx) + cosf_(rz) * (cur[4] - sy);
    float z1 = cur[5] - sz;
    float x2 = x1;
    float y2 = cosf_(rx) * y1 - sinf_(rx) * z1;
    float z2 = sinf_(rx) * y1 + cosf_(rx) * z1;
    tx = sum[3] - (cosf_(ry) * x2 + sinf_(ry) * z2);
    ty = sum[4] - y2;
    tz = sum[5] - (-sinf_(ry) * x2 + cosf_(ry) * z2);
    plugin_imu_rotation(rx, ry, rz, imu[3], imu[4], imu[5], imu[6], imu[7], imu[8], rx, ry, rz);
    sum[0] = rx; sum[1] = ry; sum[2] = rz;
    sum[3] = tx; sum[4] = ty; sum[5] = tz;
}

// transformAssociateToMap: predicted map pose tbm from odometry sum and the
// last (before, after) mapping pair
SLO_P_HD void associate_to_map(const float* sum, const float* bef, const float* aft, float* incre, float* tbm) {
    float x1 = cosf_(sum[1]) * (bef[3] - sum[3]) - sinf_(sum[1]) * (bef[5] - sum[5]);
    float y1 = bef[4] - sum[4];
    float z1 = sinf_(sum[1]) * (bef[3] - sum[3]) + cosf_(sum[1]) * (bef[5] - sum[5]);
    float x2 = x1;
    float y2 = cosf_(sum[0]) * y1 + sinf_(sum[0]) * z1;
    float z2 = -sinf_(sum[0]) * y1 + cosf_(sum[0]) * z1;
    incre[3] = cosf_(sum[2]) * x2 + sinf_(sum[2]) * y2;
    incre[4] = -sinf_(sum[2]) * x2 + cosf_(sum[2]) * y2;
    incre[5] = z2;
    float sbcx = sinf_(sum[0]), cbcx = cosf_(sum[0]), sbcy = sinf_(sum[1]), cbcy = cosf_(sum[1]), sbcz = sinf_(sum[2]), cbcz = cosf_(sum[2]);
    float sblx = sinf_(bef[0]), cblx = cosf_(bef[0]), sbly = sinf_(bef[1]), cbly = cosf_(bef[1]), sblz = sinf_(bef[2]), cblz = cosf_(bef[2]);
    float salx = sinf_(aft[0]), calx = cosf_(aft[0]), saly = sinf_(aft[1]), caly = cosf_(aft[1]), salz = sinf_(aft[2]), calz = cosf_(aft[2]);
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
    tbm[1] = atan2f_(srycrx / cosf_(tbm[0]), crycrx / cosf_(tbm[0]));
    float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) -
                   (cbcy * cbcz + sbcx * sbcy * sbcz) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) +
                   cbcx * sbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
    float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                   (sbcy * sbcz + cbcy * cbcz * sbcx) * (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) +
                   cbcx * cbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
    tbm[2] = atan2f_(srzcrx / cosf_(tbm[0]), crzcrx / cosf_(tbm[0]));
    x1 = cosf_(tbm[2]) * incre[3] - sinf_(tbm[2]) * incre[4];
    y1 = sinf_(tbm[2]) * incre[3] + cosf_(tbm[2]) * incre[4];
    z1 = incre[5];
    x2 = x1;
    y2 = cosf_(tbm[0]) * y1 - sinf_(tbm[0]) * z1;
    z2 = sinf_(tbm[0]) * y1 + cosf_(tbm[0]) * z1;
    tbm[3] = aft[3] - (cosf_(tbm[1]) * x2 + sinf_(tbm[1]) * z2);
    tbm[4] = aft[4] - y2;
    tbm[5] = aft[5] - (-sinf_(tbm[1]) * x2 + cosf_(tbm[1]) * z2);
}

// ---------------------------------------------------------------- f64 angle round trips
// The mapping node never sees FA's float angles directly: the odometry
// crosses a tf quaternion (createQuaternionMsgFromRollPitchYaw -> Matrix3x3
// getRPY) and every keyframe pose a GTSAM Rot3 (RzRyRx -> pitch/yaw/roll).
// Both are identities inside (-pi, pi] and wrap outside, so a heading that
// has turned past pi reaches mapping wrapped, as in the reference.  Double
// evaluation order as in tf's LinearMath and GTSAM's Rot3M/Rot3 (RQ); the
// double sin/cos/atan2/asin are slo_libm_d.h's, shared with the oracle, so
// the float casts agree bit for bit even where a tiny angle exposes the last
// double bit.

// tf::Quaternion::setRPY(roll, pitch, yaw) -> (x, y, z, w)
SLO_P_HD void tf_quat_rpy(double roll, double pitch, double yaw, double q[4]) {
    const double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
    const double cy = slo_libm::cos_d(hy), sy = slo_libm::sin_d(hy);
    const double cp = slo_libm::cos_d(hp), sp = slo_libm::sin_d(hp);
    const double cr = slo_libm::cos_d(hr), sr = slo_libm::sin_d(hr);
    q[0] = sr * cp * cy - cr * sp * sy;
    q[1] = cr * sp * cy + sr * cp * sy;
    q[2] = cr * cp * sy - sr * sp * cy;
    q[3] = cr * cp * cy + sr * sp * sy;
}

// Matrix3x3(q).getRPY(roll, pitch, yaw): setRotation, then getEulerYPR solution 1
SLO_P_HD void tf_rpy_of(const double q[4], double& roll, double& pitch, double& yaw) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double k = 2.0 / (x * x + y * y + z * z + w * w);
    const double xs = x * k, ys = y * k, zs = z * k;
    const double r00 = 1.0 - (y * ys + z * zs), r01 = x * ys - w * zs, r02 = x * zs + w * ys;
    const double r10 = x * ys + w * zs;
    const double r20 = x * zs - w * ys, r21 = y * zs + w * xs, r22 = 1.0 - (x * xs + y * ys);
    if (fabs(r20) >= 1.0) {   // pitch at +-90 deg
        yaw = 0.0;
        const double delta = slo_libm::atan2_d(r01, r02);
        pitch = r20 > 0 ? M_PI / 2.0 : -M_PI / 2.0;
        roll = (r20 > 0 ? pitch : -pitch) + delta;
        return;
    }
    pitch = -slo_libm::asin_d(r20);
    const double c = slo_libm::cos_d(pitch);
    roll = slo_libm::atan2_d(r21 / c, r22 / c);
    yaw = slo_libm::atan2_d(r10 / c, r00 / c);
}

// laserOdometryHandler's transformSum from FA's (publishOdometry's message
// carries (-q.y, -q.z, q.x, q.w); the handler's Quaternion(o.z, -o.x, -o.y,
// o.w) is q again)
SLO_P_HD void odom_handoff(const float ts[6], float out[6]) {
    double q[4], r, p, y;
    tf_quat_rpy((double)ts[2], (double)(-ts[0]), (double)(-ts[1]), q);
    tf_rpy_of(q, r, p, y);
    out[0] = (float)(-p);
    out[1] = (float)(-y);
    out[2] = (float)r;
    for (int i = 3; i < 6; ++i) out[i] = ts[i];
}

// row-major A * B, entries summed left to right (Eigen's 3x3 coefficient product)
SLO_P_HD void mat3_mul(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = (A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j]) + A[3 * i + 2] * B[6 + j];
}

// Pose3(Rot3::RzRyRx(t[2], t[0], t[1]), ..) read back with pitch()/yaw()/roll()
SLO_P_HD void keyframe_estimate(const float t[6], float out[6]) {
    const double ax = (double)t[2], ay = (double)t[0], az = (double)t[1];
    const double cx = slo_libm::cos_d(ax), sx = slo_libm::sin_d(ax);
    const double cy = slo_libm::cos_d(ay), sy = slo_libm::sin_d(ay);
    const double cz = slo_libm::cos_d(az), sz = slo_libm::sin_d(az);
    const double ssx = sx * sy, csx = cx * sy;
    const double A[9] = {cy * cz, -(cx * sz) + ssx * cz, sx * sz + csx * cz,
                         cy * sz, cx * cz + ssx * sz,    -(sx * cz) + csx * sz,
                         -sy,     sx * cy,               cx * cy};
    // RQ (Rot3.cpp): peel Rx, then Ry, then Rz
    const double rx = -slo_libm::atan2_d(-A[7], A[8]);
    const double c1 = slo_libm::cos_d(-rx), s1 = slo_libm::sin_d(-rx);
    const double Qx[9] = {1, 0, 0, 0, c1, -s1, 0, s1, c1};
    double B[9], C[9];
    mat3_mul(A, Qx, B);
    const double ry = -slo_libm::atan2_d(B[6], B[8]);
    const double c2 = slo_libm::cos_d(-ry), s2 = slo_libm::sin_d(-ry);
    const double Qy[9] = {c2, 0, s2, 0, 1, 0, -s2, 0, c2};
    mat3_mul(B, Qy, C);
    const double rz = -slo_libm::atan2_d(-C[3], C[4]);
    out[0] = (float)ry;
    out[1] = (float)rz;
    out[2] = (float)rx;
    for (int i = 3; i < 6; ++i) out[i] = t[i];
}

}  // namespace slo_pose
