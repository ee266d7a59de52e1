"""Steady-state diagnostic counters of a libslo variant built with a
SLO_DIAG_* flag (StreamState::dbg): S hdl64_1800 streams are pre-rolled on
the device generator, then the counters' growth over a window of scans is
printed per stream-scan.
SLO_LIB=<variant.so> python tools/knn_diag.py [streams] [preroll] [window]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import slo_amd  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
PRE = int(sys.argv[2]) if len(sys.argv) > 2 else 210
WIN = int(sys.argv[3]) if len(sys.argv) > 3 else 40
name = "hdl64_1800"
cfg = slo_amd.preset(name)
cfg.keyframe_cloud_cap = 32768
P = cfg.max_points
gen = slo_amd.DeviceGenerator(name, 3, 0, S)
CH = 16
buf = torch.empty((CH, S, P, 4), dtype=torch.float32, device="cuda")
cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
ctx = slo_amd.Context(cfg, 0, S)


def run(k0, n):
    for c in range(k0, k0 + n, CH):
        m = min(CH, k0 + n - c)
        gen.scans(c, m, buf.data_ptr())
        torch.cuda.synchronize()
        for j in range(m):
            ctx.batch_process(buf[j].data_ptr(), cnt.data_ptr(), 0.1 * (c + j))
        ctx.synchronize()


def dbg():
    return np.array([ctx.get(s, "dbg") for s in range(S)], np.float64).sum(0)


run(0, PRE)
d0 = dbg()
run(PRE, WIN)
d = dbg() - d0
print(f"{S} streams, counters over scans {PRE}..{PRE + WIN - 1}, per stream-scan:",
      (d / (S * WIN)).round(2).tolist(), flush=True)
if d[0] + d[1] > 0:
    print(f"  units staged {d[0]:.0f}, global walk {d[1]:.0f} ({100 * d[1] / (d[0] + d[1]):.1f} %), "
          f"candidates/unit {d[2] / max(1, d[0] + d[1]):.0f}, members/unit {d[3] / max(1, d[0] + d[1]):.0f}")
ctx.close()
gen.close()
