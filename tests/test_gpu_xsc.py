"""Multi-GPU record exchange on the device: slo_pack_records against the
oracle's record (bit for bit, descriptor included), the RCCL all-gather of the
records (a one-rank NCCL group: the N > 1 code path), and the cross-stream
Scan Context store (slo_xsc) against its oracle restatement — candidate
stream / keyframe, distance and yaw bit for bit — on two sessions of one
world (stream 0's first lap and, 590 scans later, its second lap) — on the
VLP-16 preset and on C4's OS1-64 64x1024."""
import os
import socket

import numpy as np
import pytest

import oracle_py as O
import slo_amd
from slo_amd import xsc as X

pytestmark = pytest.mark.gpu
LAG = 590


@pytest.mark.parametrize("pid,nscans,min_loops", [(0, 64, 3), (4, 64, 3)], ids=["vlp16", "os1_64"])
def test_records_allgather_and_cross_session_match(pid, nscans, min_loops):
    import torch
    import torch.distributed as dist
    from slo_amd import dist as sdist
    assert torch.cuda.is_available(), "no HIP device"
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    cfg = slo_amd.preset(pid)
    P = cfg.max_points
    ctx = slo_amd.Context(cfg, 0, 2)
    xs = X.CrossSession(cfg, 2, 64, 0)
    ors = [O.OracleStream(O.preset(pid), stable_voxel=False) for _ in range(2)]
    xo = O.XscOracle(O.preset(pid), 2, 64)
    rec = torch.zeros((2, slo_amd._abi.RECORD_FLOATS), dtype=torch.float32, device="cuda")
    gathered = torch.zeros_like(rec)
    out = torch.zeros((2, X.MATCH_DTYPE.itemsize // 4), dtype=torch.int32, device="cuda")
    ext = torch.cuda.ExternalStream(ctx.stream_handle)
    cnt = torch.full((2,), P, dtype=torch.int32, device="cuda")
    loops = 0
    try:
        for k in range(nscans):
            scans = [O.gen_scan(pid, 1, 0, k), O.gen_scan(pid, 1, 0, k + LAG)]
            pts = torch.from_numpy(np.stack(scans)).cuda()
            ctx.batch_process(pts.data_ptr(), cnt.data_ptr(), 0.1 * k)
            ctx.pack_records(rec.data_ptr())
            with torch.cuda.stream(ext):
                sdist.gather_records(rec, gathered)
                xs.ingest(gathered.data_ptr(), ctx.stream_handle)
                xs.query(gathered.data_ptr(), 2, 0, out.data_ptr(), ctx.stream_handle)
            ctx.synchronize()
            want = np.stack([O.record(o, bool(o.step(s, 0.1 * k) & 4)) for o, s in zip(ors, scans)])
            got = rec.cpu().numpy()
            assert got.view(np.uint32).tolist() == want.view(np.uint32).tolist(), k
            assert np.array_equal(gathered.cpu().numpy().view(np.uint32), got.view(np.uint32))
            xo.ingest(want)
            oi, of = xo.query(want, 0)
            m = out.cpu().numpy().view(X.MATCH_DTYPE).reshape(2)
            for q in range(2):
                assert [m[q][f] for f in ("valid", "n_cand", "nn_stream", "nn_keyframe", "loop")] == oi[q].tolist(), k
                if oi[q, 0]:
                    assert np.float32(m[q]["yaw"]) == np.float32(of[q, 0]) and \
                        np.float64(m[q]["min_dist"]).tobytes() == of[q, 1].tobytes(), k
            loops += int(oi[1, 4])
        assert loops >= min_loops   # session B closes loops against session A
    finally:
        xs.close()
        ctx.close()
        dist.destroy_process_group()
