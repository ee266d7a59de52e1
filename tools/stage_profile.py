"""Per-kernel times of one C3 stream's three Mode S stages (front | odometry |
mapping contexts, run one after the other), from the contexts' launch
timing: where a stage's per-scan time goes.  GPU.
python tools/stage_profile.py [scans]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sc-lego-loam_amd"))
import torch  # noqa: E402

import slo_amd  # noqa: E402
from slo_amd import modes  # noqa: E402


def main():
    scans = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    cfg = slo_amd.preset(6)
    P = cfg.max_points
    gen = slo_amd.DeviceGenerator(6, 3, 0, 1)
    buf = torch.empty((scans, 1, P, 4), dtype=torch.float32, device="cuda")
    gen.scans(0, scans, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device="cuda")
    eng = modes.SloEngine(cfg, fronts=1, split_back=True)
    ptr = [buf[k].data_ptr() for k in range(scans)]
    tim = [0.1 * k for k in range(scans)]
    warm = 20
    modes.run_local_slo(eng, 1, ptr[:warm], cnt.data_ptr(), tim[:warm])
    ctxs = {"front": eng.fronts[0], "odometry": eng.odo, "mapping": eng.owner}
    for c in ctxs.values():
        c.synchronize()
        c.timing(True)
        c.timing_reset()
    modes.run_local_slo(eng, 1, ptr[warm:], cnt.data_ptr(), tim[warm:])
    m = scans - warm
    for name, c in ctxs.items():
        t = c.timing_read()
        tot = sum(v[0] for v in t.values())
        print(f"== {name}: {tot / m * 1e3:.1f} us/scan over {sum(v[1] for v in t.values()) / m:.1f} launches/scan")
        for k, (ms, n) in sorted(t.items(), key=lambda kv: -kv[1][0])[:24]:
            print(f"   {k:28s} {ms / m * 1e3:8.1f} us/scan  {n / m:5.2f}/scan  {ms / max(n, 1) * 1e3:7.1f} us/launch")
    eng.close()


if __name__ == "__main__":
    main()
