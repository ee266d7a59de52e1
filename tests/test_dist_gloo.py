"""World-size-2 rehearsal of the multi-GPU layout on CPU (gloo): stream
sharding, the per-step record all-gather (rank-major = global stream order)
and the max-over-ranks timing bench.py reports."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from slo_amd import dist as sdist

S, F = 5, 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s0, n = sdist.stream_shard(rank, world, S)
        # record = (global stream id, rank, ...) as slo_pack_records would lay out per stream
        rec = torch.zeros((n, F), dtype=torch.float32)
        rec[:, 0] = torch.arange(s0, s0 + n, dtype=torch.float32)
        rec[:, 1] = rank
        rec[:, 2:] = torch.randn(n, F - 2, generator=torch.Generator().manual_seed(rank))
        out = sdist.gather_records(rec)
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
    ref = res[0][1]
    for rank, out, t, s0 in res:
        assert s0 == rank * S
        assert out.shape == (world * S, F)
        assert (out[:, 0] == range(world * S)).all()          # global stream order
        assert (out[:, 1] == [r for r in range(world) for _ in range(S)]).all()
        assert (out == ref).all()                              # every rank holds the same table
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
