"""Cross-stream Scan Context over the gathered records, CPU side:
the oracle's restatement of slo_xsc (oracle_api.cpp XscOracle) on two
sessions of one world — stream 0's first lap, and the same stream 590 scans
later (its second lap) — and the world-size-2 gloo rehearsal of the exchange
(each rank runs one session, all-gathers its records, and every rank's store
answers the same)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_py as O

LAG = 590          # session B = scans LAG.. of the same stream: the second lap, 16 m behind A
SCANS = 70


def _session_records(k, streams, offsets, flags_out=None):
    recs = []
    for o, off in zip(streams, offsets):
        fl = o.step(O.gen_scan(0, 1, 0, k + off), 0.1 * k)
        recs.append(O.record(o, bool(fl & 4)))
    return np.stack(recs)


def test_second_session_finds_the_first():
    cfg = O.preset(0)
    A, B = O.OracleStream(cfg, stable_voxel=False), O.OracleStream(cfg, stable_voxel=False)
    x = O.XscOracle(cfg, 2, 64)
    found = []
    for k in range(SCANS):
        recs = _session_records(k, [A, B], [0, LAG])
        x.ingest(recs)
        oi, of = x.query(recs, 0)
        assert not oi[:, 0].any() or (oi[oi[:, 0] == 1, 2] != np.nonzero(oi[:, 0])[0]).all()   # never itself
        if oi[1, 0] and oi[1, 1] > 0:
            # B at scan LAG + k is where A was at scan k - 16 (606-scan loop); A keyframes every 4th scan
            found.append((k, int(oi[1, 3]), float(of[1, 1]), int(oi[1, 4])))
    late = [f for f in found if f[0] >= 40]
    assert late and all(f[3] == 1 and f[2] < 0.15 for f in late)
    assert all(abs(f[1] - (f[0] - 16) / 4) <= 3 for f in late)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from slo_amd import dist as sdist
        cfg = O.preset(0)
        o = O.OracleStream(cfg, stable_voxel=False)
        x = O.XscOracle(cfg, world, 64)
        answers = []
        for k in range(48):
            fl = o.step(O.gen_scan(0, 1, 0, k + rank * LAG), 0.1 * k)
            rec = torch.from_numpy(O.record(o, bool(fl & 4))[None])
            table = sdist.gather_records(rec).numpy()           # [world][RECORD_FLOATS], rank-major
            x.ingest(table)
            oi, of = x.query(table, 0)                          # every rank can answer for every stream
            answers.append((oi.copy(), of.copy()))
        q.put((rank, answers))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_record_exchange():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # both ranks hold the same store and give the same answers, step by step
    for (oi0, of0), (oi1, of1) in zip(res[0], res[1]):
        assert np.array_equal(oi0, oi1)
        assert of0.tobytes() == of1.tobytes()
    # and they equal a single-process run of the same two sessions
    cfg = O.preset(0)
    A, B = O.OracleStream(cfg, stable_voxel=False), O.OracleStream(cfg, stable_voxel=False)
    x = O.XscOracle(cfg, 2, 64)
    for k in range(48):
        recs = _session_records(k, [A, B], [0, LAG])
        x.ingest(recs)
        oi, of = x.query(recs, 0)
        assert np.array_equal(oi, res[0][k][0]) and of.tobytes() == res[0][k][1].tobytes()
    assert any(a[0][1, 4] for a in res[0])     # session B found session A
