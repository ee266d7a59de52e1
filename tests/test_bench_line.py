"""bench.py's output contract on CPU: the one JSON line the driver parses
stays small (round 5's 33 KB line went unparsed), carries the contract's
fields, the roofline and the CPU baseline, and the HBM budget arithmetic
(slo_amd.budget) leaves the reserve free at every world size."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))

import bench  # noqa: E402
from slo_amd import budget  # noqa: E402

FULL = os.path.join(ROOT, "tests", "golden", "bench_full_r05.json")
LIMIT = 8 * 1024


def _full_result():
    """round 5's whole result (every per-kernel table, three config lines,
    the ICP leg) plus the records added since (Mode S over ranks, hbm)"""
    out = json.load(open(FULL))
    out["single_stream_ranks"] = {"value": 1234.5, "unit": "scans/s", "ranks": 8, "streams": 1, "scans_timed": 100,
                                  "owner_ms_per_scan": 0.81, "bit_exact_vs_one_context": True, "keyframes_at_end": 79,
                                  "err": 0, "layout": "x" * 120, "transport": "RCCL point-to-point over 8 GPUs"}
    out["hbm"] = {"context_gb": 186.48, "window_gb": 70.3, "xsc_store_gb": 2.6, "free_after_window_gb": 8.1}
    return out


def test_line_fits_and_keeps_the_contract():
    out = _full_result()
    assert len(json.dumps(out)) > 4 * LIMIT   # the fixture is the oversized kind
    line = bench.contract_line(out)
    line["detail"] = "gpurun_out/bench_detail.json"
    s = json.dumps(line)
    assert len(s) < LIMIT, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    r = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["path"]["achieved"] > 0
    c = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["A_reference_topology"]["value"] > 0
    assert line["mfma"]["unit"] == "TFLOP/s"
    assert line["single_stream_ranks"]["bit_exact_vs_one_context"] is True
    assert set(line["config_lines"]) == {"c2", "c4", "c5"}
    for j in line["config_lines"].values():
        assert j["value"] > 0 and j["roofline"]["frac"] > 0
    for k in ("kernels_ms", "kernels_algo_gbs", "roofline_also", "loop_verify_icp"):
        assert k not in line   # the side file's


def test_line_survives_missing_legs():
    out = _full_result()
    for k in ("cpu_baseline", "single_stream", "single_stream_pipelined", "single_stream_pipelined3",
              "config_lines", "roofline_also"):
        out[k] = None
    out["single_stream_ranks"] = {"error": "Mode S ranks exited with 124", "ranks": 8}
    line = bench.contract_line(out)
    assert line["cpu_baseline"] is None
    assert "error" in line["single_stream_ranks"]
    assert len(json.dumps(line)) < LIMIT


# measured context HBM per GPU (rounds 5-6: C3 512 streams 186.48 GiB, C4 512 OS1-64 streams 153.81 GiB, C5 128
# streams 92.48 GiB, the mapping workspaces included), the runtime's own ~1 GiB, 288 GB of HBM
HBM = 288e9
CASES = {"c3": (186.48, 512, 115200, 64), "c4": (153.81, 512, 65536, 64), "c5": (92.48, 128, 262144, 64)}


@pytest.mark.parametrize("cfg", sorted(CASES))
@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("steps", [20, 100, 400])
def test_hbm_budget_leaves_the_reserve(cfg, world, steps):
    ctx_gib, S, P, cap = CASES[cfg]
    free = HBM - ctx_gib * budget.GIB - budget.GIB
    store = budget.xsc_bytes(world * S, cap) if world > 1 else 0
    step = budget.step_bytes(S, P)
    need = 8 + 5 + steps
    w = budget.window_scans(free, step, need, 0, store, 8 * budget.GIB)
    assert 1 <= w <= need
    assert free - store - w * step >= 8 * budget.GIB
    segs = budget.segments(8 + 5, need, w)
    assert sum(n for _, n in segs) == steps and all(n <= w for _, n in segs)
    if steps == 20:   # the driver's run: one segment
        assert len(segs) == 1


def test_hbm_budget_refuses_clearly():
    with pytest.raises(MemoryError, match="HBM budget"):
        budget.window_scans(10 * budget.GIB, 3 * budget.GIB, 20, 0, 0, 8 * budget.GIB)
    assert budget.window_scans(100 * budget.GIB, budget.GIB, 20, 2, 0, 8 * budget.GIB, cap_scans=5) == 7


def test_xsc_bytes_match_the_allocation():
    # csrc/slo_xsc.hip:199-203 for 8 ranks x 512 streams x 64 keyframes: ~2.6 GB
    b = budget.xsc_bytes(8 * 512, 64)
    assert b == 8 * 512 * 64 * (20 * 60 * 8 + 60 * 8 + 20 * 4 + 4) + 8 * 512 * 4
    assert 2.6e9 < b < 2.8e9
