// oracle_tf.h — TEST INFRASTRUCTURE (CPU restatement; only tests/, smoke()
// and bench.py's cpu_baseline use it).
//
// The two f64 angle round trips of the reference's mapping node:
//
// 1. FA -> MO hand-off.  FeatureAssociation::publishOdometry (FA:1727-1737)
//    encodes transformSum with tf::createQuaternionMsgFromRollPitchYaw(
//    ts[2], -ts[0], -ts[1]) and mapOptimization::laserOdometryHandler
//    (MO:655-667) decodes it with tf::Matrix3x3(q).getRPY.  tf (ROS
//    geometry, LinearMath Quaternion.h / Matrix3x3.h) is not in this image;
//    its published algorithm is restated: Quaternion::setRPY,
//    Matrix3x3::setRotation, Matrix3x3::getEulerYPR(solution 1).
// 2. Keyframe save.  saveKeyFramesAndFactor (MO:1545-1611) stores the iSAM2
//    estimate of the new node: Pose3(Rot3::RzRyRx(t[2], t[0], t[1]), ..) read
//    back through Rot3::pitch()/yaw()/roll() (GTSAM 4 Rot3M.cpp RzRyRx,
//    Rot3.cpp RQ).  With only a prior and consistent between-factors the
//    estimate is the initial value (no GTSAM here: the optimiser's
//    rounding-level update is not reproduced).
//
// Inside (-pi, pi] (pitch inside [-pi/2, pi/2]) both round trips give back
// the input float; outside they wrap, which is why they matter: the heading
// of a vehicle driving a loop leaves (-pi, pi] and the reference's mapping
// then sees the wrapped angle.  The double sin/cos/atan2/asin are the host
// glibc's (oracle_libm.h), as tf's are in the reference; the device uses the
// fdlibm restatement (slo_libm_d.h, within 1 ulp of glibc), and the float casts
// are where the two must agree.
#pragma once
#include <cmath>
#include "oracle_libm.h"

namespace oracle {

struct TfQuat { double x, y, z, w; };

// tf::Quaternion::setRPY
inline TfQuat tf_set_rpy(double roll, double pitch, double yaw) {
    const double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
    const double cy = oracle_libm::cos_d(hy), sy = oracle_libm::sin_d(hy);
    const double cp = oracle_libm::cos_d(hp), sp = oracle_libm::sin_d(hp);
    const double cr = oracle_libm::cos_d(hr), sr = oracle_libm::sin_d(hr);
    return {sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
            cr * cp * cy + sr * sp * sy};
}

// tf::Matrix3x3(q) (setRotation) then getRPY(roll, pitch, yaw) (getEulerYPR, solution 1)
inline void tf_get_rpy(const TfQuat& q, double& roll, double& pitch, double& yaw) {
    const double d = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    const double s = 2.0 / d;
    const double xs = q.x * s, ys = q.y * s, zs = q.z * s;
    const double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
    const double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
    const double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
    const double m00 = 1.0 - (yy + zz), m01 = xy - wz, m02 = xz + wy;
    const double m10 = xy + wz;
    const double m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
    if (std::fabs(m20) >= 1) {   // gimbal lock (pitch = +-90 deg; unreachable for a ground vehicle, unpinned)
        yaw = 0;
        const double delta = oracle_libm::atan2_d(m01, m02);
        if (m20 > 0) { pitch = M_PI / 2.0; roll = pitch + delta; }
        else { pitch = -M_PI / 2.0; roll = -pitch + delta; }
        return;
    }
    double a = m20;
    if (a < -1) a = -1;
    if (a > 1) a = 1;   // tfAsin clamps
    pitch = -oracle_libm::asin_d(a);
    const double c = oracle_libm::cos_d(pitch);
    roll = oracle_libm::atan2_d(m21 / c, m22 / c);
    yaw = oracle_libm::atan2_d(m10 / c, m00 / c);
}

// publishOdometry (FA:1728-1734) -> laserOdometryHandler (MO:658-666)
inline void odom_handoff(const float ts[6], float out[6]) {
    const TfQuat g = tf_set_rpy((double)ts[2], (double)(-ts[0]), (double)(-ts[1]));
    // message orientation (-g.y, -g.z, g.x, g.w); the handler rebuilds
    // Quaternion(o.z, -o.x, -o.y, o.w) = g
    double roll, pitch, yaw;
    tf_get_rpy(g, roll, pitch, yaw);
    out[0] = (float)(-pitch);
    out[1] = (float)(-yaw);
    out[2] = (float)roll;
    out[3] = ts[3];
    out[4] = ts[4];
    out[5] = ts[5];
}

// Rot3::RzRyRx(x, y, z) = Rz(z) Ry(y) Rx(x), row-major
inline void gtsam_rzryrx(double x, double y, double z, double R[9]) {
    const double cx = oracle_libm::cos_d(x), sx = oracle_libm::sin_d(x);
    const double cy = oracle_libm::cos_d(y), sy = oracle_libm::sin_d(y);
    const double cz = oracle_libm::cos_d(z), sz = oracle_libm::sin_d(z);
    const double ss_ = sx * sy, cs_ = cx * sy, sc_ = sx * cy, cc_ = cx * cy;
    const double c_s = cx * sz, s_s = sx * sz, _cs = cy * sz, _cc = cy * cz;
    const double s_c = sx * cz, c_c = cx * cz;
    const double ssc = ss_ * cz, csc = cs_ * cz, sss = ss_ * sz, css = cs_ * sz;
    const double M[9] = {_cc, -c_s + ssc, s_s + csc, _cs, c_c + sss, -s_c + css, -sy, sc_, cc_};
    for (int i = 0; i < 9; ++i) R[i] = M[i];
}

// 3x3 product, each entry ((a0 b0 + a1 b1) + a2 b2)
inline void mul33(const double A[9], const double B[9], double C[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = (A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j]) + A[3 * i + 2] * B[6 + j];
}

// Rot3::xyz() through RQ(A) (Rot3.cpp): x = roll(), y = pitch(), z = yaw()
inline void gtsam_xyz(const double A[9], double& x, double& y, double& z) {
    x = -oracle_libm::atan2_d(-A[7], A[8]);
    const double c1 = oracle_libm::cos_d(-x), s1 = oracle_libm::sin_d(-x);
    const double Qx[9] = {1, 0, 0, 0, c1, -s1, 0, s1, c1};
    double B[9];
    mul33(A, Qx, B);
    y = -oracle_libm::atan2_d(B[6], B[8]);
    const double c2 = oracle_libm::cos_d(-y), s2 = oracle_libm::sin_d(-y);
    const double Qy[9] = {c2, 0, s2, 0, 1, 0, -s2, 0, c2};
    double C[9];
    mul33(B, Qy, C);
    z = -oracle_libm::atan2_d(-C[3], C[4]);
}

// the new keyframe's iSAM2 estimate read back (MO:1545-1548/1555-1556, 1588-1601)
inline void keyframe_estimate(const float t[6], float out[6]) {
    double R[9];
    gtsam_rzryrx((double)t[2], (double)t[0], (double)t[1], R);
    double x, y, z;
    gtsam_xyz(R, x, y, z);
    out[0] = (float)y;   // pitch()
    out[1] = (float)z;   // yaw()
    out[2] = (float)x;   // roll()
    out[3] = t[3];
    out[4] = t[4];
    out[5] = t[5];
}

}  // namespace oracle
