"""Cut a rocprofv3 kernel trace to bench.py's timed window and summarise it.

bench.py --trace-marker launches a torch spin kernel just before and just
after its timed steps; everything between the last two of them is the timed
window.  Prints per-kernel launches / total / average duration inside the
window, the window's wall time, the time at least one kernel was running
(busy) and the idle gaps — where host round trips and launch latency show up.

    python tools/trace_window.py gpurun_out/<tag>/kt [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def load(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not f:
        raise SystemExit(f"no *kernel_trace.csv under {d}")
    rows = []
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows, f[0]


def short(name):
    m = re.search(r"\b(k_\w+|spin\w*|sleep\w*)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows, src = load(a.dir)
    marks = [i for i, r in enumerate(rows) if re.search(r"spin|sleep", r[2], re.I)]
    if len(marks) < 2:
        raise SystemExit(f"{len(marks)} marker kernels found (bench.py --trace-marker)")
    i0, i1 = marks[-2], marks[-1]
    t0, t1 = rows[i0][1], rows[i1][0]
    win = [r for r in rows[i0 + 1:i1]]
    per = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        k = per[short(n)]
        k[0] += 1
        k[1] += e - s
    # busy = union of kernel intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    wall = t1 - t0
    tot = sum(v[1] for v in per.values())
    out = {"source": os.path.relpath(src), "window_ms": wall / 1e6, "busy_ms": busy / 1e6,
           "busy_frac": busy / wall if wall else None, "kernel_sum_ms": tot / 1e6, "launches": len(win),
           "kernels": {k: {"launches": v[0], "total_ms": round(v[1] / 1e6, 3), "avg_us": round(v[1] / v[0] / 1e3, 2)}
                       for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])}}
    print(f"window {wall / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({out['busy_frac']:.1%}), "
          f"kernel sum {tot / 1e6:.2f} ms over {len(win)} launches")
    for k, v in list(out["kernels"].items())[:30]:
        print(f"  {k:28s} {v['launches']:6d} {v['total_ms']:9.3f} ms {v['avg_us']:9.2f} us")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
