"""World-size-2 rehearsal of the multi-GPU layout on CPU (gloo): stream
sharding, the per-step record all-gather (rank-major = global stream order)
of real per-stream records (the oracle's slo_pack_records layout after three
VLP-16 scans of each global stream) and the max-over-ranks timing bench.py
reports."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_py as O
from slo_amd import dist as sdist

S, PID, NSCAN = 3, 0, 3


def _records(s0, n):
    """the record of each of streams s0 .. s0 + n - 1 after NSCAN scans"""
    out = []
    for s in range(s0, s0 + n):
        o = O.OracleStream(O.preset(PID), stable_voxel=False)
        for k in range(NSCAN):
            saved = bool(o.step(O.gen_scan(PID, 1, s, k), 0.1 * k) & 4)
        out.append(O.record(o, saved))
    return torch.from_numpy(np.stack(out))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s0, n = sdist.stream_shard(rank, world, S)
        out = sdist.gather_records(_records(s0, n))
        t = sdist.max_over_ranks(0.5 + rank)
        q.put((rank, out.numpy().copy(), t, s0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_record_allgather_and_timing(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    ref = _records(0, world * S).numpy()      # every global stream, in one process
    assert len({r.tobytes() for r in ref}) == world * S        # the streams' records differ
    for rank, out, t, s0 in res:
        assert s0 == rank * S
        assert out.shape == ref.shape
        assert out.view(np.uint32).tolist() == ref.view(np.uint32).tolist()   # global stream order, bit for bit
        assert t == 0.5 + (world - 1)                           # slowest rank's time


def test_stream_shard_bounds():
    assert sdist.stream_shard(3, 8, 64) == (192, 64)
    with pytest.raises(ValueError):
        sdist.stream_shard(8, 8, 64)


def test_group_slices_cover_the_rank():
    from slo_amd.dist import group_slices
    for S, G in [(256, 2), (192, 1), (7, 3), (5, 5)]:
        sl = group_slices(S, G)
        assert len(sl) == G
        assert sl[0][0] == 0 and sum(n for _, n in sl) == S
        assert all(sl[i][0] + sl[i][1] == sl[i + 1][0] for i in range(G - 1))
        assert max(n for _, n in sl) - min(n for _, n in sl) <= 1
    with pytest.raises(ValueError):
        group_slices(2, 3)
