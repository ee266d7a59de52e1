// slo_imu.h — FeatureAssociation's IMU path for one GPU lane, in the
// reference's float / double evaluation order (featureAssociation.cpp):
//   imu_handler      imuHandler (FA:459-486) + AccumulateIMUShiftAndRotation (FA:417-457)
//   imu_at           the ring lookup and interpolation of adjustDistortion (FA:532-590)
//   imu_velo_to_start VeloToStartIMU (FA:349-365)
//   imu_to_start     TransformToStartIMU (FA:367-392)
// Trig as everywhere in the path: slo_libm's glibc restatements (cos(float)
// is cosf; the handler's sin/cos of the double tf angles are double).
#pragma once

#include "slo_internal.h"
#include "slo_libm.h"
#include "slo_libm_d.h"
#include "slo_pose.h"

namespace slo_imu {

using slo::ImuState;
constexpr int Q = SLO_IMU_QUE;

__device__ inline void imu_handler(ImuState& m, const slo_imu_msg& in, float scanPeriod) {
    using namespace slo_libm;
    const double q[4] = {in.qx, in.qy, in.qz, in.qw};   // tf::quaternionMsgToTF
    double roll, pitch, yaw;
    slo_pose::tf_rpy_of(q, roll, pitch, yaw);            // Matrix3x3(orientation).getRPY
    const float accX0 = (float)(in.ay - sin_d(roll) * cos_d(pitch) * 9.81);
    const float accY0 = (float)(in.az - cos_d(roll) * cos_d(pitch) * 9.81);
    const float accZ0 = (float)(in.ax + sin_d(pitch) * 9.81);
    const int L = (m.last + 1) % Q;
    m.last = L;
    m.time[L] = in.stamp;
    m.roll[L] = (float)roll;
    m.pitch[L] = (float)pitch;
    m.yaw[L] = (float)yaw;
    m.acc[0][L] = accX0;
    m.acc[1][L] = accY0;
    m.acc[2][L] = accZ0;
    m.angVelo[0][L] = (float)in.wx;
    m.angVelo[1][L] = (float)in.wy;
    m.angVelo[2][L] = (float)in.wz;
    // AccumulateIMUShiftAndRotation
    const float r = m.roll[L], p = m.pitch[L], y = m.yaw[L];
    float accX = m.acc[0][L], accY = m.acc[1][L], accZ = m.acc[2][L];
    const float x1 = cosf_(r) * accX - sinf_(r) * accY;
    const float y1 = sinf_(r) * accX + cosf_(r) * accY;
    const float z1 = accZ;
    const float x2 = x1;
    const float y2 = cosf_(p) * y1 - sinf_(p) * z1;
    const float z2 = sinf_(p) * y1 + cosf_(p) * z1;
    accX = cosf_(y) * x2 + sinf_(y) * z2;
    accY = y2;
    accZ = -sinf_(y) * x2 + cosf_(y) * z2;
    const int B = (L + Q - 1) % Q;
    const double td = m.time[L] - m.time[B];
    if (td < (double)scanPeriod) {
        const float a[3] = {accX, accY, accZ};
        for (int k = 0; k < 3; ++k) {
            m.shift[k][L] = (float)((double)m.shift[k][B] + (double)m.velo[k][B] * td + (double)a[k] * td * td / 2);
            m.velo[k][L] = (float)((double)m.velo[k][B] + (double)a[k] * td);
            m.angRot[k][L] = (float)((double)m.angRot[k][B] + (double)m.angVelo[k][B] * td);
        }
    }
}

// the IMU quantities at time t = timeScanCur + pointTime (FA:532-590): the
// ring is walked from `it` (imuPointerLastIteration) to the first message not
// older than t; after the newest one the newest values are taken, otherwise
// the two messages around t are interpolated
struct ImuAt {
    float roll, pitch, yaw;
    float velo[3];
    float ang[3];       // imuAngularRotation*Cur (read only for the first point)
};

__device__ inline ImuAt imu_at(const ImuState& m, int it, double tscan, float pointTime) {
    int front = it;
    while (front != m.last) {
        if (tscan + pointTime < m.time[front]) break;
        front = (front + 1) % Q;
    }
    ImuAt o;
    if (tscan + pointTime > m.time[front]) {
        o.roll = m.roll[front];
        o.pitch = m.pitch[front];
        o.yaw = m.yaw[front];
        for (int k = 0; k < 3; ++k) { o.velo[k] = m.velo[k][front]; o.ang[k] = m.angRot[k][front]; }
    } else {
        const int back = (front + Q - 1) % Q;
        const float rf = (float)((tscan + pointTime - m.time[back]) / (m.time[front] - m.time[back]));
        const float rb = (float)((m.time[front] - tscan - pointTime) / (m.time[front] - m.time[back]));
        o.roll = m.roll[front] * rf + m.roll[back] * rb;
        o.pitch = m.pitch[front] * rf + m.pitch[back] * rb;
        if (m.yaw[front] - m.yaw[back] > M_PI)
            o.yaw = (float)(m.yaw[front] * rf + ((double)m.yaw[back] + 2 * M_PI) * rb);
        else if (m.yaw[front] - m.yaw[back] < -M_PI)
            o.yaw = (float)(m.yaw[front] * rf + ((double)m.yaw[back] - 2 * M_PI) * rb);
        else
            o.yaw = m.yaw[front] * rf + m.yaw[back] * rb;
        for (int k = 0; k < 3; ++k) {
            o.velo[k] = m.velo[k][front] * rf + m.velo[k][back] * rb;
            o.ang[k] = m.angRot[k][front] * rf + m.angRot[k][back] * rb;
        }
    }
    return o;
}

// sin/cos of the scan's start angles (updateImuRollPitchYawStartSinCos, FA:317-324)
struct ImuStartTrig { float cr, cp, cy, sr, sp, sy; };
__device__ inline ImuStartTrig start_trig(float rollStart, float pitchStart, float yawStart) {
    using namespace slo_libm;
    return ImuStartTrig{cosf_(rollStart), cosf_(pitchStart), cosf_(yawStart),
                        sinf_(rollStart), sinf_(pitchStart), sinf_(yawStart)};
}

// VeloToStartIMU (FA:349-365)
__device__ inline void imu_velo_to_start(const float* veloCur, const float* veloStart, const ImuStartTrig& t,
                                         float* out) {
    const float vx = veloCur[0] - veloStart[0], vy = veloCur[1] - veloStart[1], vz = veloCur[2] - veloStart[2];
    const float x1 = t.cy * vx - t.sy * vz;
    const float y1 = vy;
    const float z1 = t.sy * vx + t.cy * vz;
    const float x2 = x1;
    const float y2 = t.cp * y1 + t.sp * z1;
    const float z2 = -t.sp * y1 + t.cp * z1;
    out[0] = t.cr * x2 + t.sr * y2;
    out[1] = -t.sr * x2 + t.cr * y2;
    out[2] = z2;
}

// TransformToStartIMU (FA:367-392); imuShiftFromStart*Cur is always 0
__device__ inline void imu_to_start(float& px, float& py, float& pz, const ImuAt& c, const ImuStartTrig& t) {
    using namespace slo_libm;
    const float shx = 0.0f, shy = 0.0f, shz = 0.0f;
    const float x1 = cosf_(c.roll) * px - sinf_(c.roll) * py;
    const float y1 = sinf_(c.roll) * px + cosf_(c.roll) * py;
    const float z1 = pz;
    const float x2 = x1;
    const float y2 = cosf_(c.pitch) * y1 - sinf_(c.pitch) * z1;
    const float z2 = sinf_(c.pitch) * y1 + cosf_(c.pitch) * z1;
    const float x3 = cosf_(c.yaw) * x2 + sinf_(c.yaw) * z2;
    const float y3 = y2;
    const float z3 = -sinf_(c.yaw) * x2 + cosf_(c.yaw) * z2;
    const float x4 = t.cy * x3 - t.sy * z3;
    const float y4 = y3;
    const float z4 = t.sy * x3 + t.cy * z3;
    const float x5 = x4;
    const float y5 = t.cp * y4 + t.sp * z4;
    const float z5 = -t.sp * y4 + t.cp * z4;
    px = t.cr * x5 + t.sr * y5 + shx;
    py = -t.sr * x5 + t.cr * y5 + shy;
    pz = z5 + shz;
}

}  // namespace slo_imu
