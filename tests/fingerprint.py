"""Per-scan stage fingerprints shared by the golden generator
(tests/golden/make_golden.py), the oracle regression test and the GPU
fixture test: counts, SHA-256 prefixes of the bit patterns and exact poses."""
import hashlib

import numpy as np

HASHED = ["range", "ground", "seg_pts", "seg_col", "ring_start", "ring_end", "sharp", "flat", "corner_last",
          "surf_last"]
COUNTED = {"n_seg": "seg_pts", "n_outlier": "outlier", "n_sharp": "sharp", "n_flat": "flat",
           "n_corner_last": "corner_last", "n_surf_last": "surf_last"}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def row(k, flags, get):
    """flags: 2 = mapping ran, 4 = keyframe saved (the oracle_step bits);
    get(name) -> numpy array with the dtypes of slo_get / oracle_get."""
    r = {"scan": k, "flags": int(flags & 6)}
    for key, name in COUNTED.items():
        r[key] = len(get(name))
    for name in HASHED:
        r[name] = sha(get(name))
    r["transform_sum"] = [float(x) for x in get("transform_sum")]
    r["fa_iters"] = [int(x) for x in get("fa_iters")]
    if flags & 2:
        r["mapped"] = [float(x) for x in get("mapped")]
        r["mo_iters"] = int(get("mo_iters")[0])
        r["n_keyframes"] = int(get("n_keyframes")[0])
    if flags & 4:
        r["sc_desc"] = sha(get("sc_desc"))
        r["ring_key"] = sha(get("ring_key"))
    return r


def oracle_rows(O, pid, config, n_scans, stream=0):
    st = O.OracleStream(O.preset(pid), stable_voxel=False)
    rows = []
    for k in range(n_scans):
        flags = st.step(O.gen_scan(pid, config, stream, k), 0.1 * k)
        rows.append(row(k, flags, st.get))
    return rows
