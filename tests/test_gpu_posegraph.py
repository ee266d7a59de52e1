"""The pose-graph back end wired into the batched pipeline (cfg.pose_graph,
csrc/slo_pgwire.hip), on the VLP-16 stream driven twice around the synthetic
loop (tests/golden/make_loop_golden.py), whose second lap closes loops:
accepted RS / SC candidates become Cauchy loop factors (MO:1030-1046,
1078-1091); the next mapping step takes the graph's estimate for its
keyframe and rewrites every key pose (saveKeyFramesAndFactor + correctPoses,
MO:1541-1611, 1642-1664).

1. The wiring: the GPU pipeline against the oracle pipeline driven in the
   same order (oracle/oracle_pg.py PipelineWithGraph), whose graph is the
   same SE(3) solver (slo_pg's host code through its C ABI) — so every
   device write-back, factor construction (the RS correction composed on the
   device side and restated in the oracle) and correctPoses must agree bit
   for bit, before and after the loops close.
2. The solver: the graph that run built, replayed into the independent numpy
   restatement (oracle_pg.Graph, dense Gauss-Newton with numeric
   Jacobians): its optimum and slo_pg's agree within the north-star
   tolerance, 1e-4 m / 1e-4 rad.  (GTSAM itself is absent: parity with iSAM2
   is unpinned.  Two independent solvers inside the closed loop would drift
   apart through the mapping that follows each correction, which is why the
   pipeline check of (1) uses one solver.)"""
import os
import sys

import numpy as np
import pytest

import oracle_py as O
import slo_amd

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_loop_golden as G  # noqa: E402


class ProductGraph:
    """slo_pg (host code, C ABI) behind oracle_pg.Graph's interface, recording
    every factor so the graph can be replayed into the numpy restatement"""

    def __init__(self):
        from slo_amd import pose_graph as PGP
        self.g = PGP.PoseGraph()
        self.est, self.last, self.calls = [], None, []

    def add_keyframe(self, t):
        out, _ = self.g.add_keyframe(t)
        self.est.append(None)
        self.last = out
        self.calls.append(("kf", np.array(t, np.float32)))

    def add_loop(self, i, j, a, b):
        self.g.add_loop(i, j, a, b)
        self.calls.append(("loop", i, j, np.array(a, np.float32), np.array(b, np.float32)))

    def optimize(self):
        self.calls.append(("opt",))
        return self.g.optimize()

    def key_poses(self):
        return self.g.key_poses()


def _ang(d):
    return np.abs((np.asarray(d, np.float64) + np.pi) % (2 * np.pi) - np.pi)


def test_pose_graph_pipeline():
    import ctypes
    import torch
    import oracle_pg as PG
    assert torch.cuda.is_available(), "no HIP device"
    ocfg = G.loop_config()
    gcfg = slo_amd.preset(0)
    ctypes.memmove(ctypes.byref(gcfg), ctypes.byref(ocfg), ctypes.sizeof(gcfg))
    gcfg.pose_graph = 1
    ctx = slo_amd.Context(gcfg, 0, 1)
    pgraph = ProductGraph()
    orc = PG.PipelineWithGraph(O.OracleStream(ocfg, stable_voxel=False), pgraph)
    cnt = torch.full((1,), gcfg.max_points, dtype=torch.int32, device="cuda")
    loops_gpu, corrected = 0, 0
    try:
        for k in range(G.LOOP_SCANS):
            pts = O.gen_scan(G.LOOP_PRESET, G.LOOP_CONFIG, G.LOOP_STREAM, k * G.LOOP_STRIDE)
            ctx.batch_process(torch.from_numpy(pts[None]).cuda().data_ptr(), cnt.data_ptr(), 0.1 * k)
            was_pending = orc.pending
            fo = orc.step(pts, 0.1 * k)
            fg = int(ctx.get(0, "flags")[0])
            assert (fo & 14) == fg, k
            if fg & 8:
                lp = ctx.get(0, "loop")
                loops_gpu += int(any(r["ran"] and r["accepted"] and r["id"] >= 0 for r in lp))
            if fg & 2:
                corrected += int(was_pending)
                kg, ko = ctx.get(0, "keyposes"), orc.st.get("keyposes")
                assert kg.tobytes() == ko.tobytes(), k
                assert ctx.get(0, "mapped").tobytes() == orc.st.get("mapped").tobytes(), k
                for name in ("map_corner_ds", "map_surf_ds"):
                    assert ctx.get(0, name).tobytes() == orc.st.get(name).tobytes(), (k, name)
        assert loops_gpu == orc.loops >= 5 and corrected >= 5
        assert int(ctx.get(0, "err")[0]) == 0
    finally:
        ctx.close()
    # the same graph in the independent numpy solver
    ng = PG.Graph()
    for c in pgraph.calls:   # the odometry factors depend on the estimates so far: optimise where it did
        if c[0] == "kf":
            ng.add_keyframe(c[1])
        elif c[0] == "loop":
            ng.add_loop(*c[1:])
        else:
            ng.optimize()
    ng.optimize(iters=200)
    pgraph.optimize()
    kp, kn = pgraph.key_poses().astype(np.float64), ng.key_poses()
    dpos, dang = float(np.abs(kp[:, :3] - kn[:, :3]).max()), float(_ang(kp[:, 3:] - kn[:, 3:]).max())
    print(f"pose graph: {len(kp)} key poses, {orc.loops} loop steps, {corrected} corrections; "
          f"slo_pg vs numpy {dpos:.2e} m / {dang:.2e} rad")
    assert dpos < 1e-4 and dang < 1e-4
