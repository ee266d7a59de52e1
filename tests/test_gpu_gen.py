"""The device generator (csrc/slo_gendev.hip) against the host one
(slo_gen.h, slo_gen_batch): bench.py feeds the GPU from the device
generator and times the CPU baseline on host-generated scans, so the two
must be the same workload bit for bit."""
import numpy as np
import pytest

import slo_amd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,cid,stream0,S,scan0,K", [
    ("hdl64_1800", 3, 0, 5, 0, 3),      # C3 shape
    ("hdl64_1800", 3, 40, 3, 597, 2),   # second lap of the loop
    (0, 1, 2, 4, -7, 2),                # VLP-16, negative scan indices (SC history seeding)
    (7, 5, 1, 2, 11, 1),                # 128 x 2048 (C5 shape)
])
def test_device_generator_matches_host(preset, cid, stream0, S, scan0, K):
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    pid = slo_amd.PRESETS.get(preset, preset)
    want = slo_amd.gen_batch(pid, cid, stream0, S, scan0, K, P, 8)
    g = slo_amd.DeviceGenerator(pid, cid, stream0, S, 0)
    try:
        dev = torch.full((K, S, P, 4), 7.0, dtype=torch.float32, device="cuda")
        g.scans(scan0, K, dev.data_ptr())
        torch.cuda.synchronize()
        got = dev.cpu().numpy()
    finally:
        g.close()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert np.isnan(got[..., 0]).mean() > 0.01
