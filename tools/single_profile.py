"""Per-kernel times of one C3 stream in ONE context (bench.py's single_stream
leg), from the context's launch timing, beside the graph-mode latency of the
same scans: where a lone stream's per-scan time goes.  GPU.
python tools/single_profile.py [scans] [preroll]   (preroll: untimed scans first, e.g.
210 for the bench's steady state with 50-keyframe local maps)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sc-lego-loam_amd"))
import torch  # noqa: E402

import slo_amd  # noqa: E402


def main():
    scans = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    pre = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    cfg = slo_amd.preset(6)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(6, 3, 0, 1)
    scans += pre
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    ctx = slo_amd.Context(cfg, 0, 1)
    ctx.graph_mode(True)
    warm = 60 + pre
    for k in range(warm):
        ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
    ctx.synchronize()
    half = (scans - warm) // 2
    lat = []
    for k in range(warm, warm + half):   # graph mode, one at a time
        t1 = time.perf_counter()
        ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ctx.synchronize()
        lat.append(time.perf_counter() - t1)
    lat = np.array(lat) * 1e3
    print(f"graph latency ms: mean {lat.mean():.3f} p50 {np.median(lat):.3f} p90 {np.percentile(lat, 90):.3f}")
    ctx.graph_mode(False)
    ctx.timing(True)
    ctx.timing_reset()
    m = scans - warm - half
    t0 = time.perf_counter()
    for k in range(warm + half, scans):
        ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / m * 1e3
    t = ctx.timing_read()
    tot = sum(v[0] for v in t.values())
    print(f"timed (eager): {tot / m * 1e3:.1f} us/scan of kernels over {sum(v[1] for v in t.values()) / m:.1f} "
          f"launches/scan, wall {wall:.3f} ms/scan")
    for k, (ms, n) in sorted(t.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"   {k:28s} {ms / m * 1e3:8.1f} us/scan  {n / m:5.2f}/scan  {ms / max(n, 1) * 1e3:7.1f} us/launch")
    ctx.close()


if __name__ == "__main__":
    main()
