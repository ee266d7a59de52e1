"""How far two oracle variants drift apart on the same stream, CPU only.

Default: the stable in-voxel order (round 2's GPU) against the
reference-faithful oracle (PCL's std::sort in-voxel order, FA:779-780,
MO:1224-1262).  --gemm: both in the faithful voxel order, the normal
equations summed in double-double and rounded once (what the GPU computes)
against OpenCV 3.x's own GEMM order (sequential double for matAtA, four
interleaved accumulators for matAtB; FA:1324-1326, 1425-1427, MO:1445-1447;
oracle_common.h gemm_AtA).
python tools/faithful_drift.py --preset 6 --config 3 --scans 240 [--gemm]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402


def angdiff(a, b):
    d = np.asarray(a, np.float64) - np.asarray(b, np.float64)
    return np.abs((d + np.pi) % (2 * np.pi) - np.pi)


def pose_dev(a, b):
    """(max rotation deviation rad, max translation deviation m) of 6-vectors
    (rx, ry, rz, tx, ty, tz) — rows of them."""
    a = np.asarray(a, np.float64).reshape(-1, 6)
    b = np.asarray(b, np.float64).reshape(-1, 6)
    if a.size == 0:
        return 0.0, 0.0
    return float(angdiff(a[:, :3], b[:, :3]).max()), float(np.abs(a[:, 3:] - b[:, 3:]).max())


def run(pid, cid, n_scans, cfg_edit=None, verbose=False, gemm=False):
    cfg = O.preset(pid)
    if cfg_edit:
        cfg_edit(cfg)
    if gemm:
        a = O.OracleStream(cfg, stable_voxel=False, gemm_mode=0)
        b = O.OracleStream(cfg, stable_voxel=False, gemm_mode=1)
    else:
        a = O.OracleStream(cfg, stable_voxel=True)
        b = O.OracleStream(cfg, stable_voxel=False)
    worst = {"odom_rad": 0.0, "odom_m": 0.0, "map_rad": 0.0, "map_m": 0.0, "key_rad": 0.0, "key_m": 0.0}
    flags_diff = detect_diff = ringbin_diff = 0
    first_div = None
    O.gemm_tally(gemm)
    O.gemm_stats()   # reset the tallies
    for k in range(n_scans):
        pts = O.gen_scan(pid, cid, 0, k)
        fa, fb = a.step(pts, 0.1 * k), b.step(pts, 0.1 * k)
        if first_div is None and not np.array_equal(a.get("transform_sum").view(np.uint32),
                                                    b.get("transform_sum").view(np.uint32)):
            first_div = k
        flags_diff += int((fa & 14) != (fb & 14))
        r, t = pose_dev(a.get("transform_sum"), b.get("transform_sum"))
        worst["odom_rad"], worst["odom_m"] = max(worst["odom_rad"], r), max(worst["odom_m"], t)
        if fa & 2:
            r, t = pose_dev(a.get("mapped"), b.get("mapped"))
            worst["map_rad"], worst["map_m"] = max(worst["map_rad"], r), max(worst["map_m"], t)
            ka, kb = a.get("keyposes"), b.get("keyposes")
            if len(ka) == len(kb):
                # keyposes are PointTypePose rows (x, y, z, roll, pitch, yaw)
                r, t = pose_dev(ka.reshape(-1, 6)[:, [3, 4, 5, 0, 1, 2]], kb.reshape(-1, 6)[:, [3, 4, 5, 0, 1, 2]])
                worst["key_rad"], worst["key_m"] = max(worst["key_rad"], r), max(worst["key_m"], t)
            else:
                flags_diff += 1
        if fa & 4 and fb & 4:
            ringbin_diff += int(not np.array_equal(a.get("ring_key"), b.get("ring_key")))
        if fa & 8:
            da, db = a.get("detect"), b.get("detect")
            detect_diff += int(len(da) == 0 or len(db) == 0 or da[0] != db[0])
        if verbose and (k % 20 == 0):
            print(k, json.dumps(worst), flush=True)
    ent, dif = O.gemm_stats()
    return {"worst": worst, "flags_diff": flags_diff, "detect_diff": detect_diff, "ring_key_diff": ringbin_diff,
            "first_divergence_scan": first_div, "normal_equation_entries": ent, "entries_modes_differ": dif}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", type=int, default=6)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--scans", type=int, default=240)
    ap.add_argument("--sc-off", action="store_true")
    ap.add_argument("--k50", action="store_true")
    ap.add_argument("--gemm", action="store_true", help="double-double vs OpenCV's GEMM order (faithful voxel order)")
    a = ap.parse_args()

    def edit(c):
        if a.sc_off:
            c.loop_closure_enable = 0
        if a.k50:
            c.sc_num_candidates = 50
    print(json.dumps(run(a.preset, a.config, a.scans, edit, verbose=True, gemm=a.gemm)))
