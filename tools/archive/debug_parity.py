"""Print only the mismatching entries of a parity run (GPU box helper).
python tools/debug_parity.py os1_64 | ragged"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sc-lego-loam_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import oracle_py as O  # noqa: E402
import parity_report  # noqa: E402
import slo_amd  # noqa: E402


def show(rep, worst, counts):
    for r in rep:
        bad = {k: v for k, v in r.items() if isinstance(v, int) and v != 0 and k not in
               ("scan", "stream", "flags_cpu", "flags_gpu")}
        extra = {k: r[k] for k in r if k in ("flags_cpu", "flags_gpu", "odom", "mapped", "mo_iters", "n_kf")
                 or k.endswith("_len")}
        if bad or r["flags_cpu"] != r["flags_gpu"] or r.get("mapped", 0) or r.get("odom", 0):
            print(r["scan"], r["stream"], bad, extra, flush=True)
    print("SUMMARY", worst, counts, flush=True)


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "os1_64":
        show(*parity_report.run(4, 2, 2, 10, verbose=False))
    elif what == "ragged":
        cfg = slo_amd.preset(0)
        P = cfg.max_points
        nan = np.full((P, 4), np.nan, np.float32)
        show(*parity_report.run(0, 1, 5, 8, verbose=False,
                                n_points=lambda k, s: [P, P // 2, 0 if k == 3 else P, 1000, P][s],
                                scan_fn=lambda k, s: nan if (s == 4 and k == 2) else O.gen_scan(0, 1, s, k)))
