"""Graph replay vs eager launches on the same scans: two contexts side by side
(slo_graph_mode on / off), every readable field compared per scan.
python tools/graph_check.py [preset] [config] [streams] [scans]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import slo_amd  # noqa: E402

pid = int(sys.argv[1]) if len(sys.argv) > 1 else 6
cid = int(sys.argv[2]) if len(sys.argv) > 2 else 3
S = int(sys.argv[3]) if len(sys.argv) > 3 else 2
K = int(sys.argv[4]) if len(sys.argv) > 4 else 12
FIELDS = ["range", "ground", "seg_pts", "outlier", "fa_seg_pts", "curvature", "sharp", "flat", "corner_last",
          "surf_last", "transform_sum", "flags", "mapped", "raw_ds", "corner_ds", "surf_total_ds", "map_corner_ds",
          "map_surf_ds", "keyposes", "sc_desc"]
cfg = slo_amd.preset(pid)
P = cfg.max_points
host = slo_amd.gen_batch(pid, cid, 0, S, 0, K, P, 8)
g = slo_amd.Context(cfg, 0, S)
e = slo_amd.Context(cfg, 0, S)
e.graph_mode(False)
cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
bad = 0
for k in range(K):
    pts = torch.from_numpy(host[k]).cuda()
    g.batch_process(pts.data_ptr(), cnt.data_ptr(), 0.1 * k)
    e.batch_process(pts.data_ptr(), cnt.data_ptr(), 0.1 * k)
    g.synchronize()
    e.synchronize()
    diffs = []
    for s in range(S):
        for f in FIELDS:
            try:
                a, b = g.get(s, f), e.get(s, f)
            except Exception as ex:  # noqa: BLE001
                diffs.append(f"{f}:err {ex}")
                continue
            if a.shape != b.shape:
                diffs.append(f"s{s}:{f}:shape {a.shape} vs {b.shape}")
            elif not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
                diffs.append(f"s{s}:{f}:{int((a != b).sum())}")
    print(k, "ok" if not diffs else diffs, flush=True)
    bad += bool(diffs)
print("graph_check", "PASS" if not bad else f"FAIL {bad} scans")
g.close()
e.close()
