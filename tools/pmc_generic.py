"""Per-kernel averages of every counter in a rocprofv3 --pmc output dir.

python tools/pmc_generic.py gpurun_out/<dir> [name-filter]
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main(d, filt=""):
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pmc_summary import window   # the timed steps when bench.py ran with --trace-marker
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in window(list(csv.DictReader(open(f)))):
            k = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").split("::")[-1][:40]
            if filt and filt not in k:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k][r["Counter_Name"]] += 1
    for k in sorted(acc):
        vals = {c: acc[k][c] / calls[k][c] for c in acc[k]}
        print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
