"""PointCloud2 ingestion on the MI355X: the message
path of ImageProjection::cloudHandler (fromROSMsg, IP:167) and the batched
device unpack, both against the host conversion / the oracle."""
import numpy as np
import pytest

import oracle_py as O
import slo_amd
from parity_util import mismatch
from slo_amd import wire

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    return torch


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32).tobytes()


def test_cloud_handler_takes_pointcloud2():
    _torch()
    pid, cid = 0, 1
    ctx = slo_amd.Context(slo_amd.preset(pid), 0, 1)
    ip = slo_amd.ImageProjection(ctx)
    orc = O.OracleStream(O.preset(pid), stable_voxel=False)
    try:
        for k in range(3):
            pts = O.gen_scan(pid, cid, 0, k)
            orc.step(pts, 0.1 * k)
            seg = ip.cloudHandler(wire.pack(pts, "ouster", height=16, row_pad=8))
            for key in ("seg_pts", "seg_ground", "seg_col", "seg_range", "ring_start", "ring_end", "orient",
                        "outlier"):
                assert mismatch(seg[key], orc.get(key)) == 0, (k, key)
    finally:
        ctx.close()


def _upload(torch, msgs):
    stride = (max(len(m.data) for m in msgs) + 255) // 256 * 256
    raw = np.zeros((len(msgs), stride), np.uint8)
    for s, m in enumerate(msgs):
        raw[s, :len(m.data)] = np.frombuffer(m.data, np.uint8)
    dims = np.array([[m.width, m.height, m.row_step] for m in msgs], np.int32)
    return torch.from_numpy(raw).cuda(), stride, torch.from_numpy(dims).cuda()


@pytest.mark.parametrize("packed", [False, True])
def test_batch_unpack_matches_host_conversion(packed):
    torch = _torch()
    cfg = slo_amd.preset(0)
    P = cfg.max_points
    scans = [O.gen_scan(0, 1, s, 2) for s in range(3)]
    msgs = [wire.pack(scans[0], "ouster", height=16), wire.pack(scans[1], "ouster", height=1),
            wire.pack(scans[2][:16 * 1000], "ouster", height=16, row_pad=4)]
    if packed:   # a 17-byte point: every field misaligned, byte loads
        for m in msgs:
            pts = wire.fromROSMsg(m)
            h = m.height
            step = 17
            buf = np.zeros((len(pts), step), np.uint8)
            buf[:, 1:17] = pts.view(np.uint8).reshape(len(pts), 16)
            m.fields = [wire.PointField(n, 1 + 4 * k, wire.FLOAT32, 1) for k, n in
                        enumerate(("x", "y", "z", "intensity"))]
            m.point_step, m.row_step, m.data = step, step * m.width, buf.tobytes()
            assert m.height == h
    ctx = slo_amd.Context(cfg, 0, 3)
    try:
        d_raw, stride, d_dims = _upload(torch, msgs)
        layout = wire.layout_of(msgs[0])
        d_pts = torch.full((3, P, 4), -7.0, dtype=torch.float32, device="cuda")
        d_cnt = torch.zeros(3, dtype=torch.int32, device="cuda")
        ctx.batch_pc2_unpack(d_raw.data_ptr(), stride, d_dims.data_ptr(), layout, d_pts.data_ptr(),
                             d_cnt.data_ptr())
        ctx.synchronize()
        got, cnt = d_pts.cpu().numpy(), d_cnt.cpu().numpy()
        for s, m in enumerate(msgs):
            want = wire.fromROSMsg(m)
            assert cnt[s] == len(want)
            assert bits(got[s, :cnt[s]]) == bits(want), s
            assert (got[s, cnt[s]:] == -7.0).all()   # nothing written past the count
            assert int(ctx.get(s, "err")[0]) & 8 == 0
    finally:
        ctx.close()


def test_batch_unpack_clips_to_capacity_and_flags_it():
    torch = _torch()
    cfg = slo_amd.preset(0)
    P = cfg.max_points
    pts = np.tile(O.gen_scan(0, 1, 0, 0), (2, 1))[:P + 100]
    msgs = [wire.pack(pts, "xyzi"), wire.pack(pts[:50], "xyzi")]
    ctx = slo_amd.Context(cfg, 0, 2)
    try:
        d_raw, stride, d_dims = _upload(torch, msgs)
        d_pts = torch.zeros((2, P, 4), dtype=torch.float32, device="cuda")
        d_cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
        ctx.batch_pc2_unpack(d_raw.data_ptr(), stride, d_dims.data_ptr(), wire.layout_of(msgs[0]),
                             d_pts.data_ptr(), d_cnt.data_ptr())
        ctx.synchronize()
        cnt = d_cnt.cpu().numpy()
        assert cnt.tolist() == [P, 50]
        assert bits(d_pts[0].cpu().numpy()) == bits(pts[:P])
        assert int(ctx.get(0, "err")[0]) & 8 == 8 and int(ctx.get(1, "err")[0]) & 8 == 0
        # a row_step that would read past the message slot: nothing is read
        d_dims[1, 2] = stride
        d_dims[1, 1] = 2
        ctx.batch_pc2_unpack(d_raw.data_ptr(), stride, d_dims.data_ptr(), wire.layout_of(msgs[0]),
                             d_pts.data_ptr(), d_cnt.data_ptr())
        ctx.synchronize()
        assert d_cnt.cpu().numpy().tolist() == [P, 0]
        assert int(ctx.get(1, "err")[0]) & 8 == 8
    finally:
        ctx.close()
