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
