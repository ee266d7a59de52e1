"""Timeline of one scan from a rocprofv3 --kernel-trace CSV (tools/single_trace.py
under rocprofv3): per kernel the queue, start offset and duration in us, and the
gaps on the critical stream.  usage: trace_timeline.py kt_kernel_trace.csv [nth-last mapping scan]"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1]


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), short(r["Kernel_Name"])))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[3] == "k_ip_init"]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
maps = [k for k in range(len(starts) - 1) if any(rows[j][3] == "k_mo_finish" for j in range(starts[k], starts[k + 1]))]
k = maps[-which]
seg = rows[starts[k]:starts[k + 1]]
t0 = seg[0][0]
tend = max(r[1] for r in seg)
print(f"scan {k}: {len(seg)} kernels, {(tend - t0) / 1e3:.1f} us first start to last end")
agg = {}
for s, e, q, n in seg:
    print(f"q{q:<3d} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")
