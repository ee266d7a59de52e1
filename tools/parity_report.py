"""Run synthetic streams through libslo (GPU) and the oracle (CPU) side by
side and report per-stage parity.  Used by tests/test_gpu_parity.py and run
directly on the GPU box:  python tools/parity_report.py --streams 2 --scans 12
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sc-lego-loam_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
import slo_amd  # noqa: E402
from parity_util import canon_smooth, mismatch, seg_class  # noqa: E402

FRONT = ["range", "ground", "seg_pts", "seg_ground", "seg_col", "seg_range", "ring_start", "ring_end", "orient",
         "outlier", "fa_seg_pts", "sharp", "flat", "corner_last", "surf_last"]
MAPPED = ["raw_ds", "corner_ds", "surf_total_ds", "map_corner_ds", "map_surf_ds"]
SC = ["sc_desc", "ring_key", "sector_key"]


def posediff(a, b):
    return float(np.max(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)))) if len(a) else 0.0


def run(preset_id=5, config_id=2, n_streams=2, n_scans=6, verbose=True, front=True, every=1, n_points=None,
        scan_fn=None, cfg_edit=None, imu_fn=None, compare=None, device_gen=False, map_every=1):
    """n_points(k, s) -> points of stream s's scan k handed over (ragged and
    empty scans; default: all); scan_fn(k, s) -> the scan itself (default: the
    synthetic generator); cfg_edit(cfg) changes both configs (GPU and oracle);
    imu_fn(k, s) -> (n, 11) float64 IMU messages (slo_imu_msg) stream s's
    imuHandler receives before scan k (both sides).  compare: the streams run
    on the oracle and compared (default: all); device_gen: the GPU's scans come
    from the device generator (slo_gen_device_*, bit-identical to the host
    generator), so a context of hundreds of streams costs no host staging;
    map_every: mapping results compared at every map_every-th mapping step."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    cfg = slo_amd.preset(preset_id)
    ocfg = O.preset(preset_id)
    if cfg_edit:
        cfg_edit(cfg)
        cfg_edit(ocfg)
    P = cfg.max_points
    ctx = slo_amd.Context(cfg, 0, n_streams)
    cmp = list(range(n_streams)) if compare is None else list(compare)
    ors = {s: O.OracleStream(ocfg, stable_voxel=cfg.voxel_order == 1) for s in cmp}
    pool = ThreadPoolExecutor(max_workers=min(8, len(cmp))) if len(cmp) > 1 else None
    gen = slo_amd.DeviceGenerator(preset_id, config_id, 0, n_streams) if device_gen else None
    dbuf = torch.empty((1, n_streams, P, 4), dtype=torch.float32, device="cuda") if device_gen else None
    report = []
    worst = {"odom": 0.0, "map": 0.0, "keypose": 0.0}
    counts = {"bit_mismatch": 0, "detect_mismatch": 0, "detects": 0, "loops": 0, "flag_mismatch": 0,
              "stream_errors": 0}
    n_map = 0
    for k in range(n_scans):
        if device_gen:
            scans = {s: O.gen_scan(preset_id, config_id, s, k) for s in cmp}
            gen.scans(k, 1, dbuf.data_ptr())
            pts = dbuf[0]
        else:
            scans = [scan_fn(k, s) if scan_fn else O.gen_scan(preset_id, config_id, s, k) for s in range(n_streams)]
            pts = torch.from_numpy(np.stack(scans)).cuda()
        ns = [min(P, n_points(k, s)) if n_points else P for s in range(n_streams)]
        cnt = torch.tensor(ns, dtype=torch.int32, device="cuda")
        if imu_fn:
            msgs = [np.asarray(imu_fn(k, s), np.float64).reshape(-1, 11) for s in range(n_streams)]
            per = max(1, max(len(m) for m in msgs))
            buf = np.zeros((n_streams, per, 11), np.float64)
            for s, m in enumerate(msgs):
                buf[s, :len(m)] = m
                ors[s].imu(m)
            d_imu = torch.from_numpy(buf).cuda()
            d_n = torch.tensor([len(m) for m in msgs], dtype=torch.int32, device="cuda")
            ctx.batch_imu(d_imu.data_ptr(), per, d_n.data_ptr())
        ctx.batch_process(pts.data_ptr(), cnt.data_ptr(), 0.1 * k)
        step = lambda s: ors[s].step(scans[s][:ns[s]], 0.1 * k)  # noqa: E731
        fls = dict(zip(cmp, pool.map(step, cmp))) if pool else {s: step(s) for s in cmp}
        ctx.synchronize()
        mapped = any(fl & 2 for fl in fls.values())
        n_map += int(mapped)
        check_map = mapped and (n_map - 1) % map_every == 0
        for s in cmp:
            fl_o = fls[s]
            fl_g = int(ctx.get(s, "flags")[0])
            row = {"scan": k, "stream": s, "flags_cpu": fl_o & 14, "flags_gpu": fl_g}
            counts["flag_mismatch"] += int((fl_o & 14) != fl_g)
            check_front = front and (k % every == 0)
            if check_front:
                for name in FRONT:
                    row[name] = mismatch(ctx.get(s, name), ors[s].get(name))
                row["label_class"] = int((seg_class(ctx.get(s, "label")) != seg_class(ors[s].get("label"))).sum())
                S = len(ors[s].get("seg_pts"))
                for name in ("curvature", "picked", "cloud_label"):
                    row[name] = mismatch(ctx.get(s, name)[:S], ors[s].get(name)[:S])
                cfg_o = ocfg
                cv, sg = ors[s].get("curvature"), ors[s].get("seg_ground")
                rso, reo = ors[s].get("ring_start"), ors[s].get("ring_end")
                cs = [canon_smooth(x[:S], cv, sg, rso, reo, cfg_o.edge_threshold, cfg_o.surf_threshold)
                      for x in (ctx.get(s, "smooth_ind"), ors[s].get("smooth_ind"))]
                row["smooth_ind"] = mismatch(cs[0], cs[1])
            if fl_o & 1:   # transformFusion's /integrated_to_init for this scan
                row["integrated"] = mismatch(ctx.get(s, "integrated"), ors[s].get("integrated"))
            if imu_fn:   # FA's IMU scalars (ring pointers, start / current / last angles, velocities)
                row["imu"] = mismatch(ctx.get(s, "imu"), ors[s].get("imu"))
            row["odom"] = posediff(ctx.get(s, "transform_sum"), ors[s].get("transform_sum"))
            worst["odom"] = max(worst["odom"], row["odom"])
            if fl_o & 2 and check_map:
                row["mapped"] = posediff(ctx.get(s, "mapped"), ors[s].get("mapped"))
                worst["map"] = max(worst["map"], row["mapped"])
                row["mo_iters"] = [int(ctx.get(s, "mo_iters")[0]), int(ors[s].get("mo_iters")[0])]
                for name in MAPPED:
                    g, o = ctx.get(s, name), ors[s].get(name)
                    row[name] = mismatch(g, o)
                    if row[name] < 0:
                        row[name + "_len"] = [len(g), len(o)]
                if not cfg.loop_closure_enable:   # surroundingExistingKeyPosesID (MO:1181-1214)
                    ig, io = ctx.get(s, "map_ids"), ors[s].get("map_ids")
                    row["map_ids"] = mismatch(ig, io)
                    row["n_map_ids"] = [len(ig), len(io)]
                row["map_raw_n"] = ctx.get(s, "map_raw_n").tolist()
                kg, ko = ctx.get(s, "keyposes"), ors[s].get("keyposes")
                row["n_kf"] = [len(kg) // 6, len(ko) // 6]
                if len(kg) == len(ko):
                    worst["keypose"] = max(worst["keypose"], posediff(kg, ko))
            if fl_o & 4 and check_map:
                for name in SC:
                    row[name] = mismatch(ctx.get(s, name), ors[s].get(name))
            if fl_o & 8:
                dg, do = ctx.get(s, "detect"), ors[s].get("detect")
                row["detect_gpu"] = dg.tolist()
                row["detect_cpu"] = do.tolist()
                counts["detects"] += 1
                if len(dg) == 0 or len(do) == 0 or dg[0] != do[0] or not np.array_equal(dg, do):
                    counts["detect_mismatch"] += 1
                if len(do) and do[0] >= 0:
                    counts["loops"] += 1
                fg, fo = ctx.get(s, "detect_f"), ors[s].get("detect_f")
                row["sc_min_dist"] = [float(fg[1]) if len(fg) else None, float(fo[1]) if len(fo) else None]
            counts["bit_mismatch"] += sum(v for kk, v in row.items() if isinstance(v, int) and v != 0 and kk not in
                                          ("scan", "stream", "flags_cpu", "flags_gpu"))
            report.append(row)
            if verbose:
                print(json.dumps(row), flush=True)
    # sticky error bits of every stream (capacity clips, the VoxelGrid sorts' guards), compared or not
    counts["stream_errors"] = sum(int(ctx.get(s, "err")[0]) != 0 for s in range(n_streams))
    if pool:
        pool.shutdown()
    if gen:
        gen.close()
    ctx.close()
    return report, worst, counts


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", type=int, default=5)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--scans", type=int, default=12)
    ap.add_argument("--every", type=int, default=1, help="front-end bit checks every N scans")
    a = ap.parse_args()
    rep, worst, counts = run(a.preset, a.config, a.streams, a.scans, every=a.every)
    print("SUMMARY", json.dumps({"worst": worst, "counts": counts}))
