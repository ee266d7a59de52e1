"""Summarise a tools/profile_round.sh run into profiles/<tag>/summary.json.

Per kernel (named as in libslo's timing table, i.e. the SLO_LAUNCH names in
sc-lego-loam_amd/csrc): calls and average duration from the
`rocprofv3 --kernel-trace --stats` pass, and HBM traffic per launch from the
separate FETCH_SIZE and WRITE_SIZE passes.  gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half the bytes of wide
coalesced reads, so read bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE is exact
(bytes = 1024 x WRITE_SIZE).

python tools/pmc_summary.py gpurun_out/r01 profiles/r01
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def launch_names():
    """kernel symbol (as in the trace) -> timing name"""
    m = {}
    for f in glob.glob(os.path.join(ROOT, "sc-lego-loam_amd", "csrc", "*.hip")):
        for name, kern in re.findall(r'SLO_LAUNCH\(ctx,\s*"([^"]+)",\s*([\w:<>]+)', open(f).read()):
            m[kern.split("::")[-1]] = name
    return m


# launches whose kernel is a template instance named through macros
# (SLO_LAUNCH(ctx, "pc_finish_b", (k_pc_finish<PC_T, PC_FW>), ...)): instance -> timing name
TEMPLATED = {"k_pc_finish32<4096, 4>": "pc_finish_b", "k_pc_finish32<2048, 4>": "pc_finish_s",
             "k_pc_finish32<4096, 16>": "pc_finish_b", "k_pc_finish32<2048, 8>": "pc_finish_s",
             "k_pc_finish<4096, 4>": "pc_finish_bx", "k_pc_finish<2048, 4>": "pc_finish_s",
             "k_pc_finish<512, 1>": "pc_finish_w", "k_fa_ring_ds_pcl<2048, 4>": "fa_ring_ds",
             "k_fa_ring_ds_pcl<2048, 16>": "fa_ring_ds", "k_fa_ring_ds_pcl<4096, 4>": "fa_ring_ds",
             "k_fa_ring_ds_pcl<2048, 1>": "fa_ring_ds",
             "k_pc_finish<4096, 16>": "pc_finish_bx", "k_pc_finish<2048, 8>": "pc_finish_s",
             "k_fa_ring_ds_pcl<4096>": "fa_ring_ds",
             "k_pc_tail<512, 4096, 3>": "pc_tail"}


def short(kname, names):
    k = re.sub(r"\(.*$", "", kname).replace("void ", "").split("::")[-1].strip()
    if k in TEMPLATED:
        return TEMPLATED[k]
    if k in names:
        return names[k]
    if "rocprim" in kname or "hipcub" in kname:
        return "rocprim_sort_scan"
    if kname.startswith("__amd_rocclr"):
        return k
    return k


def window(rows):
    """rows between the last two bench.py --trace-marker spin kernels (by
    Dispatch_Id), i.e. the timed steps; all rows when there are no markers"""
    marks = sorted({int(r["Dispatch_Id"]) for r in rows if re.search(r"spin|sleep", r["Kernel_Name"], re.I)})
    if len(marks) < 2:
        return rows
    lo, hi = marks[-2], marks[-1]
    return [r for r in rows if lo < int(r["Dispatch_Id"]) < hi]


def main(src, dst):
    names = launch_names()
    out = defaultdict(lambda: {"calls": 0, "total_ns": 0.0, "fetch_kib": 0.0, "write_kib": 0.0,
                               "pmc_calls_fetch": 0, "pmc_calls_write": 0})
    kt = glob.glob(os.path.join(src, "kt", "**", "*kernel_trace.csv"), recursive=True)
    for r in window(list(csv.DictReader(open(kt[0])))):
        n = short(r["Kernel_Name"], names)
        out[n]["calls"] += 1
        out[n]["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for which, key in (("pmc_fetch", "fetch_kib"), ("pmc_write", "write_kib")):
        ps = glob.glob(os.path.join(src, which, "**", "*counter_collection.csv"), recursive=True)
        if not ps:
            continue
        for r in window(list(csv.DictReader(open(ps[0])))):
            n = short(r["Kernel_Name"], names)
            out[n][key] += float(r["Counter_Value"])
            out[n]["pmc_calls_" + key.split("_")[0]] += 1
    res = {}
    for n, d in out.items():
        if d["calls"] == 0:
            continue
        rb = 2 * 1024 * d["fetch_kib"] / max(1, d["pmc_calls_fetch"])
        wb = 1024 * d["write_kib"] / max(1, d["pmc_calls_write"])
        res[n] = {"calls": d["calls"], "avg_us": round(d["total_ns"] / d["calls"] / 1e3, 2),
                  "total_ms": round(d["total_ns"] / 1e6, 3),
                  "hbm_read_bytes_per_launch": int(rb), "hbm_write_bytes_per_launch": int(wb),
                  "hbm_bytes_per_launch": int(rb + wb)}
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]["total_ms"]))
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump({"source": src, "note": "read bytes = 2*1024*FETCH_SIZE (gfx950), write = 1024*WRITE_SIZE",
                   "kernels": res}, f, indent=1)
    for n, d in list(res.items())[:15]:
        print(f"{n:28s} calls={d['calls']:5d} avg_us={d['avg_us']:9.1f} total_ms={d['total_ms']:8.1f} "
              f"hbm_MB/launch={d['hbm_bytes_per_launch'] / 1e6:8.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
