"""The pose-graph back end wired into the batched pipeline (cfg.pose_graph,
csrc/slo_pgwire.hip) against the oracle pipeline driving its own numpy
restatement of the graph (oracle/oracle_pg.py PipelineWithGraph) — the
VLP-16 stream driven twice around the synthetic loop (tests/golden
make_loop_golden.py), where the second lap closes loops: accepted RS / SC
candidates become Cauchy loop factors (MO:1030-1046, 1078-1091), the next
mapping step takes the graph's estimate for its keyframe and rewrites every
key pose (saveKeyFramesAndFactor + correctPoses, MO:1541-1611, 1642-1664).

Until the first loop closes the two pipelines are bit-identical.  After it,
the two solvers (skyline Levenberg-Marquardt in C++, dense Gauss-Newton in
numpy; GTSAM itself is absent, so parity with iSAM2 is unpinned) agree to
rounding, and the north-star tolerance applies: key poses and mapped poses
within 1e-4 m / 1e-4 rad at every mapping step, the same loops accepted."""
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


def _ang(d):
    return np.abs((np.asarray(d, np.float64) + np.pi) % (2 * np.pi) - np.pi)


def test_pose_graph_pipeline_matches_oracle():
    import ctypes
    import torch
    import oracle_pg as PG
    assert torch.cuda.is_available(), "no HIP device"
    ocfg = G.loop_config()
    gcfg = slo_amd.preset(0)
    ctypes.memmove(ctypes.byref(gcfg), ctypes.byref(ocfg), ctypes.sizeof(gcfg))
    gcfg.pose_graph = 1
    ctx = slo_amd.Context(gcfg, 0, 1)
    orc = PG.PipelineWithGraph(O.OracleStream(ocfg, stable_voxel=True))
    P = gcfg.max_points
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    worst = {"pos": 0.0, "ang": 0.0, "mapped_pos": 0.0, "mapped_ang": 0.0}
    loops_gpu = 0
    first_loop = None
    try:
        for k in range(G.LOOP_SCANS):
            pts = O.gen_scan(G.LOOP_PRESET, G.LOOP_CONFIG, G.LOOP_STREAM, k * G.LOOP_STRIDE)
            ctx.batch_process(torch.from_numpy(pts[None]).cuda().data_ptr(), cnt.data_ptr(), 0.1 * k)
            fo = orc.step(pts, 0.1 * k)
            fg = int(ctx.get(0, "flags")[0])
            assert (fo & 14) == fg, k
            if fg & 8:
                lp = ctx.get(0, "loop")
                loops_gpu += int(any(r["ran"] and r["accepted"] and r["id"] >= 0 for r in lp))
            if not fg & 2:
                continue
            kg = ctx.get(0, "keyposes").reshape(-1, 6).astype(np.float64)
            ko = orc.st.get("keyposes").reshape(-1, 6).astype(np.float64)
            assert kg.shape == ko.shape, k
            if orc.loops == 0:
                assert kg.tobytes() == ko.tobytes(), k          # no loop yet: bit for bit
                continue
            first_loop = first_loop if first_loop is not None else k
            worst["pos"] = max(worst["pos"], float(np.abs(kg[:, :3] - ko[:, :3]).max()))
            worst["ang"] = max(worst["ang"], float(_ang(kg[:, 3:] - ko[:, 3:]).max()))
            mg, mo = ctx.get(0, "mapped").astype(np.float64), orc.st.get("mapped").astype(np.float64)
            worst["mapped_pos"] = max(worst["mapped_pos"], float(np.abs(mg[3:] - mo[3:]).max()))
            worst["mapped_ang"] = max(worst["mapped_ang"], float(_ang(mg[:3] - mo[:3]).max()))
        print("pose graph pipeline:", loops_gpu, "loop steps;", "first at scan", first_loop, worst)
        assert loops_gpu == orc.loops and orc.loops >= 5
        assert worst["pos"] < 1e-4 and worst["mapped_pos"] < 1e-4
        assert worst["ang"] < 1e-4 and worst["mapped_ang"] < 1e-4
        assert int(ctx.get(0, "err")[0]) == 0
    finally:
        ctx.close()
