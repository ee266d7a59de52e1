"""One C3 stream through the three-stage Mode S pipeline at several ring
depths (slo_amd.modes.run_pipelined3_slo): scans/s and per-stage busy time.
GPU.  python tools/pipe_depth.py [scans] [depth ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sc-lego-loam_amd"))
import torch  # noqa: E402

import slo_amd  # noqa: E402
from slo_amd import modes  # noqa: E402


def main():
    scans = int(sys.argv[1]) if len(sys.argv) > 1 else 220
    depths = [int(x) for x in sys.argv[2:]] or [3, 6, 12]
    cfg = slo_amd.preset(6)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(6, 3, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    ptr = [buf[k].data_ptr() for k in range(scans)]
    tim = [0.1 * k for k in range(scans)]
    warm = 20
    for d in depths:
        eng = modes.SloEngine(cfg, fronts=1, split_back=True)
        modes.run_pipelined3_slo(eng, 1, ptr[:warm], cnt.data_ptr(), tim[:warm], depth=d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = modes.run_pipelined3_slo(eng, 1, ptr[warm:], cnt.data_ptr(), tim[warm:], depth=d)
        el = time.perf_counter() - t0
        m = scans - warm
        print(f"depth {d:3d}: {m / el:7.1f} scans/s  stages ms/scan " +
              " ".join(f"{t / m * 1e3:.3f}" for t in ts), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
