"""VoxelGrid over many wide streams: (stream << voxel bits) needs more than
32 bits, so the batched sort runs on 64-bit keys (csrc/slo_vg.hip), with
empty streams in between.  Every stream's downsampled cloud must equal the
oracle's PCL VoxelGrid restatement (stable in-voxel order) bit for bit, with
the default LSD passes and with the single-pass scatters."""
import numpy as np
import pytest

import oracle_py as O
import slo_amd
from parity_util import mismatch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("onesweep", ["0", "1"])
def test_wide_streams_voxel_grid_matches_oracle(onesweep, monkeypatch):
    # onesweep = 1: the single-pass scatter sort (decoupled look-back,
    # SLO_VG_ONESWEEP, read when the context is created)
    monkeypatch.setenv("SLO_VG_ONESWEEP", onesweep)
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    pid, S = 0, 64
    cfg = slo_amd.preset(pid)
    cfg.voxel_order = 1   # the radix sort (SLO_VOXEL_STABLE): what this test is about
    P = cfg.max_points
    rng = np.random.default_rng(5)
    clouds = []
    for s in range(S):
        p = O.gen_scan(pid, 1, s, 0).copy()
        p[:, :2] *= np.float32(6.0)                    # ~600 m across
        p[:, 2] *= np.float32(3.0)
        p[:, :3] += rng.uniform(-50, 50, 3).astype(np.float32)
        if s % 17 == 3:
            p[:, :3] = np.nan                          # empty streams inside the groups
        clouds.append(p)
    # the key width this workload needs: voxel index bits + stream bits > 32
    cells = 0.0
    for c in clouds:
        f = c[np.isfinite(c[:, :3]).all(1)]
        if len(f):
            cells = max(cells, float(np.prod((f[:, :3].max(0) - f[:, :3].min(0)) / cfg.leaf_sc + 1)))
    assert np.log2(cells) + np.log2(S) > 33
    ctx = slo_amd.Context(cfg, 0, S)
    try:
        dev = torch.from_numpy(np.stack(clouds)).cuda()
        cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
        ctx.batch_sc_make(dev.data_ptr(), cnt.data_ptr())
        ctx.synchronize()
        for s in range(S):
            want = O.voxel_grid(clouds[s], cfg.leaf_sc, stable=True)
            got = ctx.get(s, "raw_ds")
            assert mismatch(got, want) == 0, s
    finally:
        ctx.close()


def test_voxel_grid_int32_overflow_returns_the_input():
    # PCL's guard: when the bounding box holds more than
    # INT32_MAX cells the filter returns its input unchanged.  Streams whose
    # clouds are stretched to ~40 km x 40 km x 1.5 km (> 2^31 cells at 0.5 m)
    # sit between ordinary streams in one batched call.
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    pid, S = 0, 6
    cfg = slo_amd.preset(pid)
    P = cfg.max_points
    clouds = []
    for s in range(S):
        p = O.gen_scan(pid, 1, s, 0).copy()
        if s % 2 == 1:
            p[:, :2] *= np.float32(400.0)
            p[:, 2] *= np.float32(100.0)
        clouds.append(p)
    ctx = slo_amd.Context(cfg, 0, S)
    try:
        dev = torch.from_numpy(np.stack(clouds)).cuda()
        cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
        ctx.batch_sc_make(dev.data_ptr(), cnt.data_ptr())
        ctx.synchronize()
        for s in range(S):
            fin = clouds[s][np.isfinite(clouds[s][:, :3]).all(1)]
            want = O.voxel_grid(fin, cfg.leaf_sc, stable=False)
            if s % 2 == 1:
                assert want.tobytes() == fin.tobytes()      # the oracle takes the overflow branch
            got = ctx.get(s, "raw_ds")
            assert mismatch(got, want) == 0, s
    finally:
        ctx.close()


def _stable(cfg):
    cfg.voxel_order = 1   # SLO_VOXEL_STABLE: the radix sort, input order inside a voxel


@pytest.mark.parametrize("onesweep", ["0", "1"])
def test_pipeline_with_stable_voxel_order(monkeypatch, onesweep):
    """C3 (hdl64_1800) pipeline, two mapping rounds per stream, every
    VoxelGrid in the stable order (cfg.voxel_order = 1) by the LSD radix
    passes or by the single-pass scatters: bit-exact vs the oracle in its
    stable mode."""
    import os
    import sys
    monkeypatch.setenv("SLO_VG_ONESWEEP", onesweep)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import parity_report
    rep, worst, counts = parity_report.run(6, 3, 2, 14, verbose=False, cfg_edit=_stable)
    bad = [r for r in rep if any(isinstance(v, int) and v != 0 and k not in
                                 ("scan", "stream", "flags_cpu", "flags_gpu") for k, v in r.items())]
    assert not bad and not counts["flag_mismatch"] and not counts["detect_mismatch"], (bad[:2], counts)
    assert not any(worst.values()), worst
    assert sum(1 for r in rep if r["flags_cpu"] & 2) >= 1
