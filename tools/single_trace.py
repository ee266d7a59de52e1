"""One C3 stream, one plain context: per-scan latency (graph mode, synchronised
after each scan) classed by what the scan ran (flags: mapping, keyframe,
loop detection), then the same scans eager with per-kernel HIP-event timing,
summed per class.  Writes gpurun_out/single_trace.json."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
import torch  # noqa: E402
import slo_amd  # noqa: E402


def run(graphs, timing, n0, n, buf, cnt, cfg, pid):
    ctx = slo_amd.Context(cfg, 0, 1)
    ctx.graph_mode(graphs)
    lat, cls, ker = [], [], []
    try:
        for k in range(n0):
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ctx.synchronize()
        if timing:
            ctx.timing(True)
        for k in range(n0, n):
            if timing:
                ctx.timing_reset()
            t1 = time.perf_counter()
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            ctx.synchronize()
            lat.append((time.perf_counter() - t1) * 1e3)
            cls.append(int(ctx.get(0, "flags")[0]))
            if timing:
                ker.append(ctx.timing_read())
    finally:
        ctx.close()
    return lat, cls, ker


def main():
    cfg = slo_amd.preset("hdl64_1800")
    pid = slo_amd.PRESETS["hdl64_1800"]
    n0, n = 215, 215 + int(os.environ.get("SCANS", "120"))
    buf = torch.empty((n, 1, cfg.max_points, 4), dtype=torch.float32, device="cuda:0")
    gen = slo_amd.DeviceGenerator(pid, 3, 0, 1, 0)
    gen.scans(0, n, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), cfg.max_points, dtype=torch.int32, device="cuda:0")
    out = {}
    lat, cls, _ = run(True, False, n0, n, buf, cnt, cfg, pid)
    out["graph"] = {"lat_ms": [round(x, 3) for x in lat], "flags": cls}
    lat2, cls2, ker = run(False, True, n0, n, buf, cnt, cfg, pid) if os.environ.get("EAGER", "1") == "1" else ([], [], [])
    out["eager"] = {"lat_ms": [round(x, 3) for x in lat2], "flags": cls2}
    by = {}
    for f, kt in zip(cls2, ker):
        d = by.setdefault(f, {"scans": 0, "k": {}})
        d["scans"] += 1
        for nm, (ms, c) in kt.items():
            e = d["k"].setdefault(nm, [0.0, 0])
            e[0] += ms
            e[1] += c
    out["kernels_by_flags"] = {str(f): {"scans": d["scans"], "k": {nm: [round(v[0] / d["scans"], 4), v[1] / d["scans"]]
                                                                  for nm, v in sorted(d["k"].items(), key=lambda x: -x[1][0])}}
                               for f, d in by.items()}
    for f in sorted(set(cls)):
        l = np.array([x for x, c in zip(lat, cls) if c == f])
        print(f"flags {f}: {len(l)} scans, graph ms mean {l.mean():.3f} p50 {np.median(l):.3f} max {l.max():.3f}", flush=True)
    l = np.array(lat)
    print(f"all: mean {l.mean():.3f} p50 {np.median(l):.3f} p99 {np.percentile(l, 99):.3f}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.environ.get("TRACE_OUT") or os.path.join(ROOT, "gpurun_out", "single_trace.json"), "w"))


if __name__ == "__main__":
    main()
