"""Sharding equivalence (SURVEY §4 / §8(e) mode M): the streams a rank owns
run the same whatever else shares the device.  Four streams in one context
against the same streams split over two contexts (the per-rank layout of
bench.py / slo_amd.dist): the per-stream records that the multi-GPU path
all-gathers (slo_pack_records: poses, keyframe count, loop result, newest
ring key) must be bit-identical after every scan."""
import numpy as np
import pytest

import oracle_py as O
import slo_amd

pytestmark = pytest.mark.gpu


def test_split_contexts_give_identical_records():
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    pid, cid, S, K = 0, 1, 4, 12
    cfg = slo_amd.preset(pid)
    P = cfg.max_points
    whole = slo_amd.Context(cfg, 0, S)
    halves = [slo_amd.Context(cfg, 0, 2), slo_amd.Context(cfg, 0, 2)]
    F = whole.L.slo_record_floats()
    rec_w = torch.zeros((S, F), dtype=torch.float32, device="cuda")
    rec_h = [torch.zeros((2, F), dtype=torch.float32, device="cuda") for _ in halves]
    cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
    mapped = 0
    try:
        for k in range(K):
            pts = torch.from_numpy(np.stack([O.gen_scan(pid, cid, s, k) for s in range(S)])).cuda()
            whole.batch_process(pts.data_ptr(), cnt.data_ptr(), 0.1 * k)
            for h, c in enumerate(halves):
                c.batch_process(pts[2 * h].data_ptr(), cnt[2 * h].data_ptr(), 0.1 * k)
            whole.pack_records(rec_w.data_ptr())
            for h, c in enumerate(halves):
                c.pack_records(rec_h[h].data_ptr())
            whole.synchronize()
            for c in halves:
                c.synchronize()
            got = torch.cat(rec_h).cpu().numpy()
            want = rec_w.cpu().numpy()
            assert got.view(np.uint32).tobytes() == want.view(np.uint32).tobytes(), k
            mapped += int(int(whole.get(0, "flags")[0]) & 2 != 0)
        assert mapped >= 2   # mapping and keyframes ran inside the compared window
    finally:
        whole.close()
        for c in halves:
            c.close()
