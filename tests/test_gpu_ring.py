"""useCloudRing (utility.h:64; IP:172-178, 225-226) on the MI355X: rows from
the points' "ring" field instead of their elevation, against the oracle.
The reference ships the option disabled; these cases run it on synthetic
rings (true rows for most points, a few out of range, which IP:232 drops)."""
import numpy as np
import pytest

import oracle_py as O
import slo_amd
from parity_util import mismatch
from slo_amd import wire

pytestmark = pytest.mark.gpu
KEYS = ("seg_pts", "seg_ground", "seg_col", "seg_range", "ring_start", "ring_end", "orient", "outlier")


def _torch():
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    return torch


def _rings(pts, R, seed):
    """ring per point: the generator's firing order is ring-major within a
    column, so index % R is the laser; 2 % of the points get an out-of-range ring"""
    rng = np.random.default_rng(seed)
    r = (np.arange(len(pts)) % R).astype(np.uint16)
    bad = rng.random(len(pts)) < 0.02
    r[bad] = R + rng.integers(0, 5, bad.sum())
    return r


def _cfg(mod, pid):
    c = mod.preset(pid)
    c.use_cloud_ring = 1
    return c


def test_message_rings_follow_the_reference_indexing():
    # the message path: uint16 "ring" of PointXYZIR read at the index AFTER
    # NaN removal (laserCloudInRing->points[i]); the generator's scans have
    # NaNs, so a message flagged is_dense reproduces the reference's shift
    _torch()
    pid, cid = 0, 1
    cfg = _cfg(slo_amd, pid)
    ctx = slo_amd.Context(cfg, 0, 1)
    ip = slo_amd.ImageProjection(ctx)
    orc = O.OracleStream(_cfg(O, pid), stable_voxel=False)
    try:
        for k in range(3):
            pts = O.gen_scan(pid, cid, 0, k)
            rings = _rings(pts, cfg.n_scan, k)
            msg = wire.pack(pts, "velodyne", height=16, ring=rings)
            msg.is_dense = True
            orc.set_rings(rings)
            orc.image_projection(pts)
            seg = ip.cloudHandler(msg)
            for key in KEYS:
                assert mismatch(seg[key], orc.get(key)) == 0, (k, key)
        msg.is_dense = False   # the reference shuts down (IP:174-177)
        with pytest.raises(slo_amd.SloError):
            ip.cloudHandler(msg)
    finally:
        ctx.close()


def test_batched_rings_through_the_pipeline():
    torch = _torch()
    pid, cid, S, K = 0, 1, 2, 8
    cfg = _cfg(slo_amd, pid)
    P = cfg.max_points
    ctx = slo_amd.Context(cfg, 0, S)
    orcs = [O.OracleStream(_cfg(O, pid), stable_voxel=False) for _ in range(S)]
    d_cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
    try:
        for k in range(K):
            scans = [O.gen_scan(pid, cid, s, k) for s in range(S)]
            rings = [_rings(p, cfg.n_scan, 100 * s + k) for s, p in enumerate(scans)]
            d_pts = torch.from_numpy(np.stack(scans)).cuda()
            d_rng = torch.from_numpy(np.stack(rings).astype(np.int16)).cuda()
            ctx.batch_set_rings(d_rng.data_ptr())
            ctx.batch_process(d_pts.data_ptr(), d_cnt.data_ptr(), 0.1 * k)
            ctx.synchronize()
            for s in range(S):
                # device rings are indexed like the points; the oracle reads
                # them at the filtered index, so hand it the finite points' rings
                fin = np.isfinite(scans[s][:, :3]).all(axis=1)
                orcs[s].set_rings(rings[s][fin])
                orcs[s].step(scans[s], 0.1 * k)
                for key in ("seg_pts", "seg_col", "transform_sum"):
                    assert mismatch(ctx.get(s, key), orcs[s].get(key)) == 0, (k, s, key)
    finally:
        ctx.close()


def test_ring_mode_needs_rings():
    _torch()
    cfg = _cfg(slo_amd, 0)
    ctx = slo_amd.Context(cfg, 0, 1)
    try:
        with pytest.raises(slo_amd.SloError):
            slo_amd.ImageProjection(ctx).cloudHandler(O.gen_scan(0, 1, 0, 0))
    finally:
        ctx.close()


def test_batch_unpack_delivers_rings():
    # slo_batch_pc2_unpack's ring output: PointXYZIR's uint16 "ring" per point
    # (an Ouster uint8 ring does not match the reference's uint16 field -> 0)
    torch = _torch()
    cfg = _cfg(slo_amd, 0)
    P = cfg.max_points
    scans = [O.gen_scan(0, 1, s, 1) for s in range(2)]
    rings = [_rings(p, cfg.n_scan, s) for s, p in enumerate(scans)]
    for layout, want in (("velodyne", rings), ("ouster", [np.zeros_like(r) for r in rings])):
        msgs = [wire.pack(p, layout, height=16, ring=r) for p, r in zip(scans, rings)]
        stride = len(msgs[0].data)
        raw = torch.from_numpy(np.stack([np.frombuffer(m.data, np.uint8) for m in msgs])).cuda()
        dims = torch.tensor([[m.width, m.height, m.row_step] for m in msgs], dtype=torch.int32, device="cuda")
        ctx = slo_amd.Context(cfg, 0, 2)
        try:
            d_pts = torch.zeros((2, P, 4), dtype=torch.float32, device="cuda")
            d_cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
            d_rng = torch.full((2, P), -1, dtype=torch.int16, device="cuda")
            ctx.batch_pc2_unpack(raw.data_ptr(), stride, dims.data_ptr(), wire.layout_of(msgs[0]), d_pts.data_ptr(),
                                 d_cnt.data_ptr(), d_rng.data_ptr())
            ctx.synchronize()
            got = d_rng.cpu().numpy().view(np.uint16)
            for s in range(2):
                assert (got[s, :len(want[s])] == want[s]).all(), (layout, s)
        finally:
            ctx.close()
