"""VoxelGrid sort microbenchmark on the GPU: S streams of a map-like cloud
(5 hdl64 scans side by side, ~570 k points, leaf 0.3) and of raw scans
(115 k points with NaNs, leaf 0.5), through slo_batch_voxel_grid, per voxel
order; per-kernel times from the context's timing table.
python tools/vg_bench.py --streams 170 --reps 3"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "sc-lego-loam_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
import slo_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=170)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--which", default="map,raw")
    a = ap.parse_args()
    import torch
    parts = []
    for k in range(5):
        p = O.gen_scan(6, 3, 0, 4 * k)
        p = p[np.isfinite(p[:, :3]).all(1)].copy()
        p[:, 0] += np.float32(2.0 * k)
        parts.append(p)
    clouds = {"map": (np.concatenate(parts), 0.3), "raw": (O.gen_scan(6, 3, 1, 7), 0.5)}
    res = {}
    for name in a.which.split(","):
        cloud, leaf = clouds[name]
        S, n = a.streams, len(cloud)
        d_in = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(cloud, (S, n, 4)))).cuda()
        d_n = torch.full((S,), n, dtype=torch.int32, device="cuda")
        d_out = torch.zeros((S, n, 4), dtype=torch.float32, device="cuda")
        d_no = torch.zeros(S, dtype=torch.int32, device="cuda")
        for vo in (0, 1):
            cfg = slo_amd.preset(6)
            cfg.voxel_order = vo
            ctx = slo_amd.Context(cfg, 0, S)
            run = lambda: ctx.batch_voxel_grid(d_in.data_ptr(), n, d_n.data_ptr(), leaf, d_out.data_ptr(), n,  # noqa
                                               d_no.data_ptr(), n)
            run()
            ctx.synchronize()
            t0 = time.time()
            for _ in range(a.reps):
                run()
            ctx.synchronize()
            wall = (time.time() - t0) / a.reps * 1e3
            ctx.timing(True)
            ctx.timing_reset()
            for _ in range(a.reps):
                run()
            ctx.synchronize()
            t = ctx.timing_read()
            st = ctx.get(0, "pcl_work").tolist()
            vs = ctx.get(0, "vg_stats").tolist()
            ctx.close()
            res[f"{name}_vo{vo}"] = {"wall_ms": round(wall, 3), "items": S * n,
                                     "kernels_ms": {k: round(v[0] / a.reps, 3) for k, v in
                                                    sorted(t.items(), key=lambda kv: -kv[1][0])[:12]},
                                     "pcl_work": st, "vg_stats": vs}
            print(name, vo, json.dumps(res[f"{name}_vo{vo}"]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
