"""Print libslo's per-stream diagnostic counters (StreamState::dbg) after a
short batched run — phase cycle sums of whichever kernel is instrumented.
python tools/dbg_counters.py [preset] [streams] [scans]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import slo_amd  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hdl64_1800"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 16
K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
cfg = slo_amd.preset(name)
pid = slo_amd.PRESETS[name]
P = cfg.max_points
host = slo_amd.gen_batch(pid, 3, 0, S, 0, K, P, 8)
dev = torch.from_numpy(host).cuda()
cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
ctx = slo_amd.Context(cfg, 0, S)
for k in range(K):
    ctx.batch_process(dev[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
ctx.synchronize()
d = np.array([ctx.get(s, "dbg") for s in range(S)], np.float64)
print("per stream-scan averages:", (d.sum(0) / (S * K)).round(1).tolist())
print("per ring (R=%d):" % cfg.n_scan, (d.sum(0) / (S * K * cfg.n_scan)).round(1).tolist())
ctx.close()
