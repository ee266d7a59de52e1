"""Run synthetic streams through libslo (GPU) and the oracle (CPU) side by
side and report per-stage parity.  Used by tests/test_gpu_parity.py and run
directly on the GPU box:  python tools/parity_report.py --streams 2 --scans 6
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
from parity_util import mismatch, seg_class  # noqa: E402

FRONT = ["range", "ground", "seg_pts", "seg_ground", "seg_col", "seg_range", "ring_start", "ring_end", "orient",
         "outlier", "fa_seg_pts", "sharp", "flat", "corner_last", "surf_last"]


def run(preset_id=5, config_id=2, n_streams=2, n_scans=6, verbose=True):
    import torch
    cfg = slo_amd.preset(preset_id)
    P = cfg.max_points
    ctx = slo_amd.Context(cfg, 0, n_streams)
    ors = [O.OracleStream(O.preset(preset_id), stable_voxel=True) for _ in range(n_streams)]
    report = []
    max_pose = 0.0
    for k in range(n_scans):
        scans = [O.gen_scan(preset_id, config_id, s, k) for s in range(n_streams)]
        pts = torch.from_numpy(np.stack(scans)).cuda()
        cnt = torch.full((n_streams,), P, dtype=torch.int32, device="cuda")
        ctx.batch_image_projection(pts.data_ptr(), cnt.data_ptr())
        ctx.batch_feature_association()
        ctx.synchronize()
        for s in range(n_streams):
            ors[s].step(scans[s], 0.1 * k)
            row = {"scan": k, "stream": s}
            for name in FRONT:
                row[name] = mismatch(ctx.get(s, name), ors[s].get(name))
            lab_g, lab_o = ctx.get(s, "label"), ors[s].get("label")
            row["label_class"] = int((seg_class(lab_g) != seg_class(lab_o)).sum())
            S = len(ors[s].get("seg_pts"))
            for name in ("curvature", "picked", "cloud_label", "smooth_ind"):
                row[name] = mismatch(ctx.get(s, name)[:S], ors[s].get(name)[:S])
            tg, to = ctx.get(s, "transform_sum"), ors[s].get("transform_sum")
            d = float(np.max(np.abs(tg.astype(np.float64) - to.astype(np.float64))))
            row["pose_maxdiff"] = d
            row["fa_iters_gpu"] = ctx.get(s, "fa_iters").tolist()
            row["fa_iters_cpu"] = ors[s].get("fa_iters").tolist()
            max_pose = max(max_pose, d)
            report.append(row)
            if verbose:
                print(json.dumps(row), flush=True)
    ctx.close()
    return report, max_pose


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", type=int, default=5)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--scans", type=int, default=6)
    a = ap.parse_args()
    rep, mp = run(a.preset, a.config, a.streams, a.scans)
    print("max pose diff", mp)
