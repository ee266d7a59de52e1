"""Mode S on the GPU (include/slo_abi.h "Mode S", slo_amd/modes.py): one
stream's front ends (slo_front_process) dealt round-robin over 2 and 3 front
contexts, every back end (slo_back_process) on an owner context, the carry
and the features handed over as device buffers — what the ranks of a
multi-GPU run send each other.  The owner's odometry and mapped poses, key
poses, Scan Context descriptors and detect records equal a one-context run of
the same stream (slo_batch_process, itself bit-exact against the oracle in
test_gpu_parity.py) bit for bit at every scan."""
import numpy as np
import pytest

import slo_amd
from slo_amd import modes

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    return torch


@pytest.mark.parametrize("preset,config,scans,world,split", [
    (0, 1, 220, 2, False),   # C1 VLP-16 past 51 keyframes: Scan Context detects run on the owner
    (6, 3, 40, 3, False),    # C3 hdl64_1800, three front contexts
    (0, 1, 220, 1, True),    # the back end split: odometry context | mapping context (slo_odom/map_process)
    (6, 3, 40, 2, True),
])
def test_mode_s_owner_matches_one_context(preset, config, scans, world, split):
    torch = _torch()
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(preset, config, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    one = slo_amd.Context(cfg, 0, 1)
    eng = modes.SloEngine(cfg, fronts=world, split_back=split)
    bad, detects = [], 0
    try:
        def check(k):
            nonlocal detects
            one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            fl = int(one.get(0, "flags")[0])
            if fl != int(eng.owner.get(0, "flags")[0]):
                bad.append((k, "flags"))
            names = ["transform_sum", "integrated", "err"]
            if fl & 2:
                names += ["mapped", "keyposes", "map_surf_ds", "surf_total_ds"]
            if fl & 4:
                names += ["sc_desc", "ring_key"]
            if fl & 8:
                names += ["detect", "detect_f"]
                detects += 1
            for name in names:
                a, b = one.get(0, name), eng.owner.get(0, name)
                if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                    bad.append((k, name))

        modes.run_local_slo(eng, world, [buf[k].data_ptr() for k in range(scans)], cnt.data_ptr(),
                            [0.1 * k for k in range(scans)], on_back=check)
        assert bad == [], bad[:5]
        assert int(one.get(0, "err")[0]) == 0
        kf = len(one.get(0, "keyposes")) // 6
        print(f"Mode S {world} fronts{', split back end' if split else ''}: {scans} scans, {kf} keyframes, {detects} detects, owner bit-identical")
        if preset == 0:
            assert detects >= 1
    finally:
        eng.close()
        one.close()


@pytest.mark.parametrize("world", [1, 2])
def test_mode_s_pipelined_matches_one_context(world):
    """the two-stage pipeline on one GPU (modes.run_pipelined_slo: a host
    thread per stage, scan k + 1's front end beside scan k's back end)
    changes when the work runs, not what: C3 hdl64_1800 for 60 scans, the
    owner's records equal a one-context run's bit for bit"""
    torch = _torch()
    preset, config, scans = 6, 3, 60
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(preset, config, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    one = slo_amd.Context(cfg, 0, 1)
    eng = modes.SloEngine(cfg, fronts=world)
    try:
        ref = {}
        for k in range(scans):
            one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            ref[k] = {n: one.get(0, n).copy() for n in ("transform_sum", "mapped", "keyposes", "flags")}
        got = {}

        def grab(k):
            got[k] = {n: eng.owner.get(0, n).copy() for n in ref[k]}

        tf, tb = modes.run_pipelined_slo(eng, world, [buf[k].data_ptr() for k in range(scans)], cnt.data_ptr(),
                                         [0.1 * k for k in range(scans)], on_back=grab)
        for k in range(scans):
            for n in ref[k]:
                assert np.array_equal(ref[k][n].view(np.uint8), got[k][n].view(np.uint8)), (k, n)
        print(f"pipelined Mode S, {world} front context(s): front {tf / scans * 1e3:.3f} ms, "
              f"back {tb / scans * 1e3:.3f} ms per scan")
    finally:
        eng.close()
        one.close()


def test_mode_s_three_stage_pipeline_matches_one_context():
    """the three-stage pipeline (modes.run_pipelined3_slo: front | odometry |
    mapping, a host thread and context each, the reference's three
    processes): C3 hdl64_1800 for 60 scans, the mapping context's odometry,
    fused and mapped poses, keyframes and flags equal a one-context run's bit
    for bit"""
    torch = _torch()
    preset, config, scans = 6, 3, 60
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(preset, config, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    one = slo_amd.Context(cfg, 0, 1)
    eng = modes.SloEngine(cfg, fronts=1, split_back=True)
    names = ("transform_sum", "integrated", "mapped", "keyposes", "flags", "err")
    try:
        ref = {}
        for k in range(scans):
            one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            ref[k] = {n: one.get(0, n).copy() for n in names}
        got = {}

        def grab(k):
            got[k] = {n: eng.owner.get(0, n).copy() for n in names}

        tf, to, tm = modes.run_pipelined3_slo(eng, 1, [buf[k].data_ptr() for k in range(scans)], cnt.data_ptr(),
                                              [0.1 * k for k in range(scans)], on_back=grab)
        for k in range(scans):
            for n in names:
                assert np.array_equal(ref[k][n].view(np.uint8), got[k][n].view(np.uint8)), (k, n)
        print(f"three-stage Mode S: front {tf / scans * 1e3:.3f}, odometry {to / scans * 1e3:.3f}, "
              f"mapping {tm / scans * 1e3:.3f} ms per scan")
    finally:
        eng.close()
        one.close()


@pytest.mark.parametrize("world,split,preset,config,scans", [
    (1, False, 0, 1, 80),    # world 1: the owner runs every front end itself, nothing travels
    (3, False, 6, 3, 40),    # three ranks: carry from rank to rank, features to the owner
    (4, True, 6, 3, 40),     # the three processes as ranks: mapping 0, odometry 1, front ends 2 and 3
])
def test_rank_drivers_match_one_context(world, split, preset, config, scans):
    """the multi-GPU drivers (modes.run_rank / run_rank3, the ones the gloo
    rehearsal runs on the oracle) with SloEngine ranks as threads of one
    process on one GPU, the buffers moved by modes.LocalTransport: the
    owner's poses, key poses, descriptors and detects equal a one-context run
    bit for bit at every scan"""
    import threading
    torch = _torch()
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(preset, config, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    one = slo_amd.Context(cfg, 0, 1)
    engs = [modes.SloEngine.for_rank(cfg, r, world, split_back=split) for r in range(world)]
    tr = modes.LocalTransport.group(world)
    run = modes.run_rank3 if split else modes.run_rank
    bad, errs, out = [], [], {}

    def check(k, fl):
        one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ref = int(one.get(0, "flags")[0])
        if ref != fl:
            bad.append((k, "flags", ref, fl))
        names = ["transform_sum", "integrated", "err"] + (["mapped", "keyposes"] if ref & 2 else []) + \
                (["sc_desc", "ring_key"] if ref & 4 else []) + (["detect", "detect_f"] if ref & 8 else [])
        for name in names:
            a, b = one.get(0, name), engs[0].owner.get(0, name)
            if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                bad.append((k, name))

    def go(r):
        try:
            out[r] = run(engs[r], r, world, lambda k: ((buf[k].data_ptr(), cnt.data_ptr()), 0.1 * k), scans, tr[r],
                         on_back=check if r == 0 else None)
        except BaseException as e:   # noqa: BLE001
            errs.append((r, e))
            for q in tr:   # unblock the others: their receives time out
                q.timeout = 1.0

    try:
        ths = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errs, errs
        assert bad == [], bad[:5]
        assert len(out[0]) == scans
    finally:
        for e in engs:
            e.close()
        one.close()


def test_mode_s_three_streams_ragged_matches_one_context():
    """n_streams vehicles split the same way: a context of three
    streams with different point counts (so each stream's carry tail past its
    own seg_count differs), front ends over two front contexts, every stream
    against a three-stream one-context run bit for bit"""
    torch = _torch()
    preset, config, scans, S = 6, 3, 30, 3
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(preset, config, 0, S)
    buf = torch.empty((scans, S, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.tensor([P, P - 20011, P // 2 + 7], dtype=torch.int32, device="cuda")
    one = slo_amd.Context(cfg, 0, S)
    eng = modes.SloEngine(cfg, fronts=2, n_streams=S)
    bad = []
    try:
        def check(k):
            one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            for s in range(S):
                fl = int(one.get(s, "flags")[0])
                names = ["transform_sum", "integrated", "err", "flags"] + (["mapped", "keyposes"] if fl & 2 else [])
                for name in names:
                    a, b = one.get(s, name), eng.owner.get(s, name)
                    if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                        bad.append((k, s, name))

        modes.run_local_slo(eng, 2, [buf[k].data_ptr() for k in range(scans)], cnt.data_ptr(),
                            [0.1 * k for k in range(scans)], on_back=check)
        assert bad == [], bad[:5]
        assert len({int(one.get(s, "seg_pts").shape[0]) for s in range(S)}) == S   # the streams differ
    finally:
        eng.close()
        one.close()


def test_pipelined_raises_when_the_back_end_fails():
    """run_pipelined_slo with a back end that raises: the error
    surfaces instead of the front thread waiting for a free slot forever"""
    torch = _torch()
    cfg = slo_amd.preset(0)
    P = cfg.max_points
    scans = 12
    gen = slo_amd.DeviceGenerator(0, 1, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    eng = modes.SloEngine(cfg, fronts=1)
    try:
        def boom(k):
            if k == 1:
                raise RuntimeError("back end failed")

        with pytest.raises(RuntimeError, match="back end failed"):
            modes.run_pipelined_slo(eng, 1, [buf[k].data_ptr() for k in range(scans)], cnt.data_ptr(),
                                    [0.1 * k for k in range(scans)], depth=2, on_back=boom)
    finally:
        eng.close()


def test_mode_s_and_imu_refuse_each_other():
    """Mode S carries no IMU ring: a context fed IMU messages
    refuses slo_front_process / slo_back_process (SLO_E_STATE, with the
    reason in the error text), and a context Mode S ran on refuses IMU
    messages — instead of odometry that silently differs from one context"""
    torch = _torch()
    from slo_amd import _abi
    cfg = slo_amd.preset(0)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(0, 1, 0, 1)
    buf = torch.empty((1, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, 1, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    msg = np.zeros(1, _abi.IMU_DTYPE)
    eng = modes.SloEngine(cfg, fronts=1)
    try:
        eng.fronts[0].imu_handler(msg)   # fed IMU: Mode S refused
        c, f = eng.buffers()
        with pytest.raises(slo_amd.SloError, match="IMU"):
            eng.front(0, buf[0].data_ptr(), cnt.data_ptr(), 0.0, None, c, f)
        # the owner ran Mode S: IMU refused
        g = eng.buffers()[1]
        eng2 = modes.SloEngine(cfg, fronts=1)
        try:
            eng2.front(0, buf[0].data_ptr(), cnt.data_ptr(), 0.0, None, None, g)
            eng2.back(g, buf[0].data_ptr(), cnt.data_ptr(), 0.0)
            for ctx in (eng2.fronts[0], eng2.owner):
                with pytest.raises(slo_amd.SloError, match="IMU"):
                    ctx.imu_handler(msg)
        finally:
            eng2.close()
    finally:
        eng.close()


def test_mode_s_leg_as_processes_gloo(tmp_path):
    """bench.py's Mode S leg as separate processes (bench.py --modes-leg,
    slo_amd.dist.launch_ranks): three ranks of run_rank3 — mapping, odometry,
    front end — moving device buffers through modes.HostTransport over gloo
    (the leg's fallback when RCCL is unavailable; RCCL itself needs one GPU per
    rank), all three on this GPU; the owner's final state and every scan's
    flags equal one context's bit for bit"""
    import json
    import os
    import sys
    import tempfile
    from slo_amd import dist as sdist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    argv = ["--modes-leg", "--gpus", "3", "--preset", "hdl64_1800", "--config-id", "3", "--preroll", "24",
            "--warmup", "2", "--modes-steps", "16", "--modes-transport", "gloo"]
    with tempfile.TemporaryFile("w+") as f:
        rc = sdist.launch_ranks(3, argv, os.path.join(root, "bench.py"), stdout=f, timeout_s=240)
        f.seek(0)
        lines = [x for x in f.read().splitlines() if x.startswith("{")]
    assert rc == 0 and lines, rc
    rec = json.loads(lines[-1])
    assert rec["bit_exact_vs_one_context"] is True, rec
    assert rec["ranks"] == 3 and rec["err"] == 0 and rec["value"] > 0
    print(rec, file=sys.stderr)


def _pipe_names(fl):
    n = ["transform_sum", "integrated", "err", "flags", "n_keyframes", "seg_pts", "curvature", "sharp", "less_flat",
         "transform_cur", "fa_iters", "corner_last"]
    if fl & 2:
        n += ["mapped", "keyposes", "map_surf_ds", "surf_total_ds", "raw_ds"]
    if fl & 4:
        n += ["sc_desc", "ring_key"]
    if fl & 8:
        n += ["detect", "detect_f"]
    return n


@pytest.mark.parametrize("preset,config,scans,depth", [
    (0, 1, 220, 2),   # C1 VLP-16 past 51 keyframes (Scan Context detects), the smallest rings
    (6, 3, 60, 6),    # C3 hdl64_1800 at the bench's depth
])
def test_pipeline_one_context_matches_plain(preset, config, scans, depth):
    """slo_pipeline: one context whose front end, odometry and mapping stage
    run on three HIP streams (the reference's three processes inside one
    context).  Scan by scan (read after each) every pose, flag, feature cloud,
    keyframe, descriptor and detect equals a plain context's bit for bit —
    each field read from the stage that computes it — and, enqueued back to
    back with no host wait (the stages overlapping through the rings), the
    final state is the same too."""
    torch = _torch()
    cfg = slo_amd.preset(preset)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(preset, config, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    one = slo_amd.Context(cfg, 0, 1)
    pipe = slo_amd.Context(cfg, 0, 1)
    pipe.pipeline(depth)
    fast = slo_amd.Context(cfg, 0, 1)
    fast.pipeline(depth)
    bad, detects, ref = [], 0, None
    try:
        for k in range(scans):
            one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            pipe.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            fl = int(one.get(0, "flags")[0])
            detects += int(bool(fl & 8))
            for name in _pipe_names(fl):
                a, b = one.get(0, name), pipe.get(0, name)
                if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                    bad.append((k, name))
        ref = {n: one.get(0, n).copy() for n in _pipe_names(7)}
        for k in range(scans):   # back to back: the host only enqueues
            fast.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        fast.synchronize()
        for n, a in ref.items():
            b = fast.get(0, n)
            if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                bad.append(("async", n))
        assert bad == [], bad[:8]
        assert int(one.get(0, "n_keyframes")[0]) > 5
        if preset == 0:
            assert detects > 0
    finally:
        for c in (one, pipe, fast):
            c.close()


def test_pipeline_refusals():
    """slo_pipeline only on a fresh context, and not with the paths whose host
    round trips need one context (loop verification here)"""
    torch = _torch()
    cfg = slo_amd.preset(0)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(0, 1, 0, 1)
    buf = torch.empty((1, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, 1, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    a = slo_amd.Context(cfg, 0, 1)
    try:
        a.batch_process(buf[0].data_ptr(), cnt.data_ptr(), 0.0)
        with pytest.raises(slo_amd.SloError, match="first scan|processed a scan"):
            a.pipeline(4)
    finally:
        a.close()
    cfg2 = slo_amd.preset(0)
    cfg2.loop_verify = 1
    cfg2.loop_archive_points = 4096
    b = slo_amd.Context(cfg2, 0, 1)
    try:
        with pytest.raises(slo_amd.SloError, match="loop verification"):
            b.pipeline(4)
    finally:
        b.close()
