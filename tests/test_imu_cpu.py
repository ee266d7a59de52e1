"""IMU path of FeatureAssociation in the oracle (CPU): imuHandler +
AccumulateIMUShiftAndRotation (featureAssociation.cpp:417-486), the IMU
branch of adjustDistortion (FA:525-616), updateInitialGuess (FA:1639-1664)
and the IMU terms of TransformToEnd / integrateTransformation.  The GPU is
compared with this restatement in tests/test_gpu_imu.py.  The reference has no
IMU fixtures and ROS/tf are absent, so these pin properties of the published
algorithm; parity with the reference's binary stays unpinned."""
import math

import numpy as np

import imu_synth
import oracle_py as O

PID, CID = 0, 1   # VLP-16: small and fast


def _run(n_scans, imu_fn=None, stream=0):
    o = O.OracleStream(O.preset(PID), stable_voxel=False)
    out = []
    for k in range(n_scans):
        if imu_fn is not None:
            o.imu(imu_fn(k))
        o.step(O.gen_scan(PID, CID, stream, k), 0.1 * k)
        out.append({n: o.get(n).copy() for n in ("fa_seg_pts", "transform_sum", "transform_cur", "mapped", "imu")})
    return out


def _level(k):
    """a stationary, level IMU: identity orientation, gravity only, no rotation rate"""
    m = imu_synth.scan_messages(0, k)
    m[:, 1:5] = (0.0, 0.0, 0.0, 1.0)
    m[:, 5:8] = (0.0, 0.0, 9.81)
    m[:, 8:11] = 0.0
    return m


def test_stationary_level_imu_changes_nothing():
    """with every IMU angle, velocity and rotation 0 the IMU terms are the
    reference's zero-IMU values: the same odometry and map as without messages"""
    a, b = _run(8), _run(8, _level)
    for k, (x, y) in enumerate(zip(a, b)):
        for n in ("fa_seg_pts", "transform_sum", "transform_cur", "mapped"):
            assert np.array_equal(x[n], y[n]), (k, n)
        assert y["imu"][0] >= 0 and x["imu"][0] == -1   # the ring is in use only with messages


def test_imu_ring_pointers_and_dropout():
    """imuPointerLast advances one slot per message modulo imuQueLength = 200;
    imuPointerLastIteration follows it after each scan (FA:616), also across a
    dropout where a scan receives no message"""
    o = O.OracleStream(O.preset(PID), stable_voxel=False)
    total = 0
    for k in range(30):
        m = imu_synth.scan_messages(1, k, every=3)
        o.imu(m)
        total += len(m)
        o.step(O.gen_scan(PID, CID, 1, k), 0.1 * k)
        st = o.get("imu")
        assert st[0] == (total - 1) % 200 and st[1] == st[0], (k, st[:2])
    assert total > 200   # the ring wrapped


def test_imu_deskews_and_seeds_the_odometry():
    """a rotating IMU changes the deskewed cloud (TransformToStartIMU) and the
    initial guess (updateInitialGuess: transformCur[0..2] = -imuAngularFromStart)"""
    fn = lambda k: imu_synth.scan_messages(0, k)   # noqa: E731
    a, b = _run(6), _run(6, fn)
    assert not np.array_equal(a[3]["fa_seg_pts"], b[3]["fa_seg_pts"])
    st = b[3]["imu"]
    assert np.all(np.isfinite(st)) and np.any(st[17:20] != 0)   # imuAngularFromStart
    # the odometry still tracks: the two runs stay within a few centimetres
    assert np.max(np.abs(a[5]["transform_sum"][3:] - b[5]["transform_sum"][3:])) < 0.2


def test_yaw_interpolation_across_pi():
    """a heading oscillating across +-pi: the interpolated yaw takes the +-2pi
    branch (FA:567-573) and stays near +-pi instead of averaging to ~0"""
    fn = lambda k: imu_synth.scan_messages(0, k, wrap=True)   # noqa: E731
    out = _run(12, fn)
    yaws = np.array([r["imu"][10] for r in out])   # imuYawCur of each scan's last point
    assert np.all(np.abs(np.abs(yaws) - math.pi) < 0.5), yaws
