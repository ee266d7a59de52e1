"""Mode S rehearsed on CPU (slo_amd/modes.py): one VLP-16
stream's front ends dealt round-robin over 2 and 3 gloo ranks, its back ends
on rank 0, the carry and the features sent point to point.  The restatement
runs the compute (oracle OracleStream.front / back), so this checks the
protocol — what travels, in which order — against a one-process run of the
same stream: odometry and mapped poses, keyframes and Scan Context detects
bit for bit at every scan.  The rank drivers are the product's
(modes.run_rank / run_rank3); the oracle engine is tests/mode_engines.py.  tests/test_gpu_modes.py checks libslo's own
front / back split the same way on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_py as O
from mode_engines import OracleEngine
from slo_amd import modes

PID, CID, N = 0, 1, 220   # C1 VLP-16; >= 51 keyframes by the end, so Scan Context detects run


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scan(k):
    return O.gen_scan(PID, CID, 0, k), 0.1 * k


def _worker(rank, world, port, q, split=False, transport="dist"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = O.preset(PID)
        eng = OracleEngine(cfg, split_back=split)
        ref = O.OracleStream(cfg) if rank == 0 else None
        bad, detects, kf = [], 0, 0

        def check(k, fl):
            nonlocal detects, kf
            pts, t = _scan(k)
            fr = ref.step(pts, t)
            if fr != fl:
                bad.append((k, "flags", fr, fl))
            names = ["transform_sum", "integrated"] + (["mapped", "keyposes"] if fr & 2 else []) + \
                    (["detect", "detect_f"] if fr & 8 else [])
            for name in names:
                a, b = ref.get(name), eng.owner.get(name)
                if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                    bad.append((k, name))
            detects += int(bool(fr & 8))
            kf = len(ref.get("keyposes")) // 6

        run = modes.run_rank3 if split else modes.run_rank
        tr = modes.DistTransport() if transport == "dist" else modes.HostTransport()
        run(eng, rank, world, _scan, N, tr, on_back=check if rank == 0 else None)
        q.put((rank, bad, detects, kf))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,split,transport", [(2, False, "dist"), (3, False, "dist"), (3, True, "dist"),
                                                   (4, True, "dist"), (3, True, "host")])
def test_mode_s_owner_matches_one_process(world, split, transport):
    """split: the reference's three processes as ranks (modes.run_rank3:
    mapping on rank 0, odometry on rank 1, front ends on the rest); "host":
    modes.HostTransport, bench.py's gloo fallback for the Mode S leg"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, split, transport)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    rank, bad, detects, kf = res[0]
    assert bad == [], bad[:5]
    assert kf >= 52 and detects >= 1, (kf, detects)


def test_split_back_end_matches_one_object():
    """OracleStream.odom / mapstage on two objects equal back() on one: flags,
    odometry, fused and mapped poses, keyframes at every scan (C1, 120 scans)"""
    cfg = O.preset(PID)
    one, two = OracleEngine(cfg), OracleEngine(cfg, split_back=True)
    for k in range(120):
        pts, t = _scan(k)
        _, f = one.front(0, pts, t, None)
        _, f2 = two.front(0, pts, t, None)
        assert one.back(f, pts, t) == two.back(f2, pts, t), k
        for name in ("transform_sum", "integrated", "mapped", "keyposes"):
            assert np.array_equal(one.owner.get(name).view(np.uint8), two.owner.get(name).view(np.uint8)), (k, name)


def test_carry_is_the_one_object_state():
    """the carry a front end hands on is exactly the stale state one object
    running every front end would hold: two front objects taking turns, each
    starting from the carry, leave the same carry bytes as one object after
    every scan — also after one of them ran another stream first (its own
    stale state is then wrong for this stream; the carry replaces it).  (On
    these synthetic streams the stale reads never change a feature — 0 of 100
    scans, measured with and without the carry — so the carry buys
    exactness in the Q5 corner cases, not a visible difference here.)"""
    cfg = O.preset(PID)
    one, two = OracleEngine(cfg, fronts=1), OracleEngine(cfg, fronts=2)
    c = None
    for k in range(5):   # front object 1 first sees another stream
        c, _ = two.fronts[1].front(O.gen_scan(PID, CID, 7, k), 0.1 * k, c)
    c1 = c2 = None
    for k in range(40):
        pts, t = _scan(k)
        c1, f1 = one.front(0, pts, t, None)   # one object: its own state carries over
        c2, f2 = two.front(k % 2, pts, t, c2)
        assert np.array_equal(c1, c2), k
        assert np.array_equal(f1, f2), k


@pytest.mark.parametrize("world,split", [(2, False), (4, True)])
def test_mode_s_threads_local_transport(world, split):
    """the same drivers with the ranks as threads of one process
    (modes.LocalTransport), the form tests/test_gpu_modes.py runs on one GPU"""
    import threading
    cfg = O.preset(PID)
    n = 60
    tr = modes.LocalTransport.group(world)
    engs = [OracleEngine(cfg, split_back=split) for _ in range(world)]
    run = modes.run_rank3 if split else modes.run_rank
    out, errs = {}, []

    def go(r):
        try:
            out[r] = run(engs[r], r, world, _scan, n, tr[r])
        except BaseException as e:   # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=go, args=(r,)) for r in range(world)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs, errs
    ref = O.OracleStream(cfg)
    for k in range(n):
        pts, t = _scan(k)
        assert ref.step(pts, t) == out[0][k], k
    for name in ("transform_sum", "integrated", "mapped", "keyposes"):
        assert np.array_equal(ref.get(name).view(np.uint8), engs[0].owner.get(name).view(np.uint8)), name
