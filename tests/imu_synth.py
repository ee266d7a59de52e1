"""Synthetic IMU messages for the IMU-path parity tests (test infrastructure).

slo_imu_msg / sensor_msgs/Imu records (stamp, orientation quaternion, linear
acceleration, angular velocity) at 100 Hz.  Orientation: small roll / pitch
oscillations and a heading that, for `wrap` streams, oscillates across +-pi
(so adjustDistortion's yaw interpolation takes its +-2pi branches,
featureAssociation.cpp:567-573).  Linear acceleration is gravity plus a small
motion term (imuHandler subtracts gravity, FA:466-468); angular velocity is
the derivative of the angles.  Scan k (stamp 0.1 k) receives the messages
stamped in (0.1 k, 0.1 k + 0.1] — the sweep it covers — and scan 0 also the
ones since -0.05 s, so the ring holds data before the first point."""
import math

import numpy as np

RATE = 100.0
G = 9.81


def _quat_rpy(roll, pitch, yaw):
    """tf::Quaternion::setRPY -> (x, y, z, w)"""
    hy, hp, hr = yaw * 0.5, pitch * 0.5, roll * 0.5
    cy, sy, cp, sp, cr, sr = math.cos(hy), math.sin(hy), math.cos(hp), math.sin(hp), math.cos(hr), math.sin(hr)
    return (sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
            cr * cp * cy + sr * sp * sy)


def message(stream, t, wrap=False):
    ph = 0.7 * stream
    roll = 0.02 * math.sin(1.3 * t + ph)
    pitch = 0.015 * math.cos(0.9 * t + 2 * ph)
    if wrap:
        yaw = math.pi + 0.2 * math.sin(0.8 * t + ph)
        dyaw = 0.16 * math.cos(0.8 * t + ph)
    else:
        yaw = 0.3 * math.sin(0.2 * t + ph)
        dyaw = 0.06 * math.cos(0.2 * t + ph)
    droll = 0.026 * math.cos(1.3 * t + ph)
    dpitch = -0.0135 * math.sin(0.9 * t + 2 * ph)
    qx, qy, qz, qw = _quat_rpy(roll, pitch, yaw)
    ax = -math.sin(pitch) * G + 0.05 * math.sin(2.1 * t + ph)
    ay = math.sin(roll) * math.cos(pitch) * G + 0.03 * math.cos(1.7 * t)
    az = math.cos(roll) * math.cos(pitch) * G + 0.02 * math.sin(3.0 * t)
    return (t, qx, qy, qz, qw, ax, ay, az, droll, dpitch, dyaw)


def scan_messages(stream, k, period=0.1, wrap=False, every=1):
    """(n, 11) float64: the messages delivered before scan k; with every > 1
    only every `every`-th scan gets its messages (an IMU dropout)"""
    if k % every:
        return np.zeros((0, 11), np.float64)
    j0 = -5 if k == 0 else int(round(k * period * RATE)) + 1
    j1 = int(round((k + 1) * period * RATE))
    if k > 0 and every > 1:   # the messages of the skipped scans arrive late, with this scan
        j0 = int(round((k - every + 1) * period * RATE)) + 1
    return np.array([message(stream, j / RATE, wrap) for j in range(j0, j1 + 1)], np.float64).reshape(-1, 11)
