"""GPU parity of FeatureAssociation's IMU path (slo_batch_imu /
slo_imu_handler): imuHandler + AccumulateIMUShiftAndRotation
(featureAssociation.cpp:417-486), the IMU deskew of adjustDistortion
(FA:525-616), updateInitialGuess (FA:1639-1664), TransformToEnd's and
integrateTransformation's IMU terms — against the oracle restatement, bit
for bit, on synthetic IMU streams (tests/imu_synth.py): a smooth one, one
whose heading crosses +-pi, one with dropouts; the ring wraps (> 200
messages)."""
import os
import sys

import numpy as np
import pytest

import imu_synth
import oracle_py as O
import slo_amd
from parity_util import mismatch

pytestmark = pytest.mark.gpu
_TOOLS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
if _TOOLS not in sys.path:
    sys.path.insert(0, _TOOLS)


def _imu(k, s):
    if s % 3 == 1:
        return imu_synth.scan_messages(s, k, wrap=True)
    if s % 3 == 2:
        return imu_synth.scan_messages(s, k, every=3)
    return imu_synth.scan_messages(s, k)


def _clean(rep, worst, counts):
    bad = [r for r in rep if any(isinstance(v, int) and v != 0 and k not in
                                 ("scan", "stream", "flags_cpu", "flags_gpu") for k, v in r.items())]
    assert not bad, bad[:2]
    assert counts["flag_mismatch"] == 0 and counts["detect_mismatch"] == 0
    assert worst == {"odom": 0.0, "map": 0.0, "keypose": 0.0}


@pytest.mark.parametrize("preset,config,streams,scans", [
    (6, 3, 3, 26),   # C3 hdl64_1800: 6 mapping rounds, > 200 IMU messages per stream
    (0, 1, 3, 30),   # VLP-16
])
def test_imu_pipeline_bit_exact(preset, config, streams, scans):
    import torch
    assert torch.cuda.is_available()
    import parity_report
    rep, worst, counts = parity_report.run(preset, config, streams, scans, verbose=False, imu_fn=_imu)
    assert all("imu" in r for r in rep)
    _clean(rep, worst, counts)


def test_imu_single_scan_api():
    """FeatureAssociation.imuHandler + runFeatureAssociation(t) on a one-stream
    context == the oracle's nodes"""
    import torch
    assert torch.cuda.is_available()
    pid, cid = 0, 1
    cfg = slo_amd.preset(pid)
    ctx = slo_amd.Context(cfg, 0, 1)
    ip, fa = slo_amd.ImageProjection(ctx), slo_amd.FeatureAssociation(ctx)
    orc = O.OracleStream(O.preset(pid), stable_voxel=False)
    try:
        for k in range(12):
            msgs = imu_synth.scan_messages(0, k, wrap=True)
            for m in msgs:
                fa.imuHandler(m)
            orc.imu(msgs)
            pts = O.gen_scan(pid, cid, 0, k)
            orc.step(pts, 0.1 * k)
            ip.cloudHandler(pts)
            f = fa.runFeatureAssociation(0.1 * k)
            for key in ("sharp", "flat", "corner_last", "surf_last"):
                assert mismatch(f[key], orc.get(key)) == 0, (k, key)
            assert mismatch(f["transform_sum"], orc.get("transform_sum")) == 0, k
            assert mismatch(ctx.get(0, "imu"), orc.get("imu")) == 0, k
    finally:
        ctx.close()
