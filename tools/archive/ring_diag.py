"""fa_ring_ds sort counters (SLO_DIAG_RING build: StreamState::dbg) for one
C3 stream: where the per-ring PCL-order VoxelGrid spends its time.  GPU.
SLO_LIB=sc-lego-loam_amd/variants/libslo_ring.so python tools/ring_diag.py
(make -C sc-lego-loam_amd BUILD=build_ring LIB=variants/libslo_ring.so DEFS=-DSLO_DIAG_RING=1)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sc-lego-loam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import slo_amd  # noqa: E402


def main():
    scans = 40
    for S in [int(x) for x in sys.argv[1:]] or (1, 64):
        cfg = slo_amd.preset(6)
        P = cfg.max_points
        gen = slo_amd.DeviceGenerator(6, 3, 0, S)
        buf = torch.empty((scans, S, P, 4), dtype=torch.float32, device="cuda")
        gen.scans(0, scans, buf.data_ptr())
        gen.close()
        cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
        ctx = slo_amd.Context(cfg, 0, S)
        ctx.graph_mode(False)
        ctx.timing(True)
        for k in range(scans):
            if k == 10:
                d0 = ctx.get(0, "dbg").astype(np.int64)
                ctx.timing_reset()
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        d = ctx.get(0, "dbg").astype(np.int64)
        mx_sort, slow_n, slow_ring = int(d[1]), int(d[6] >> 4) & 0xfff, int(d[7]) & 0xff
        d = d - d0
        t = ctx.timing_read()
        m = scans - 10
        R = cfg.n_scan
        print(f"S={S}: fa_ring_ds {t['fa_ring_ds'][0] / m * 1e3:.1f} us/launch; stream 0, per ring: sort {d[0] / m / R:.0f} "
              f"cycles (slowest ever {mx_sort}: ring {slow_ring}, {slow_n} points); block_sort phases: group levels "
              f"{d[2] / m / R:.0f}, wave level {d[3] / m / R:.0f}, bookkeeping {d[4] / m / R:.0f}, queue "
              f"{d[5] / m / R:.0f}", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
