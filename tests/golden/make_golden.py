"""Generate the committed golden fixtures under tests/golden/ (run in the
build container, where /root/reference exists):

  python tests/golden/make_golden.py

1. sc_loop_hdl64.npz — Scan Context loop-detection fixture pinned by the
   reference's own ring-key tree.  A synthetic hdl64_1800 stream (config 3,
   stream 0) is sampled every 3rd scan for 240 keyframes (> one 606 m lap,
   so loops close).  Each keyframe goes through the oracle's
   VoxelGrid(0.5) + makeAndSaveScancontextAndKeys + detectLoopClosureID
   (PCL's std::sort in-voxel order, the reference's, which the GPU VoxelGrid
   reproduces by default).  For every
   detect the tree snapshot and query are also fed to oracle/_ref/nanoflann_pin
   — the reference's KDTreeVectorOfVectorsAdaptor + nanoflann.hpp, compiled
   from /root/reference by `make -C oracle ref` — for K = 10 (C3) and K = 50
   (C5).  Stored: the float ring keys, per-detect snapshot size, nanoflann
   indices/distances, and the oracle's loop id / candidates / yaw / min dist.

2. front_vlp16.json, front_hdl64.json — per-scan stage fingerprints of the
   oracle (restatement) on short synthetic streams: segmented / feature counts,
   SHA-256 prefixes of the range image, labels and feature clouds, odometry
   and mapped poses, keyframe counts.  These pin the oracle against silent
   regressions (parity of the restatement itself is unpinned beyond
   nanoflann: SURVEY §8(c)) and are what the GPU path is checked against.
"""
import json
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_py as O  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
import fingerprint as F  # noqa: E402

PIN = os.path.join(ROOT, "oracle", "_ref", "nanoflann_pin")

SC_PRESET, SC_CONFIG, SC_STREAM, SC_STEP, SC_N = 6, 3, 0, 3, 240
FRONT = {"vlp16": (0, 1, 12), "hdl64": (6, 3, 10)}   # preset, config, scans


def nanoflann(queries, dim, K):
    """queries: list of (snapshot float32 [n][dim], key float32 [dim])."""
    buf = [struct.pack("<iii", dim, K, len(queries))]
    for snap, key in queries:
        buf.append(struct.pack("<i", len(snap)))
        buf.append(np.ascontiguousarray(snap, np.float32).tobytes())
        buf.append(np.ascontiguousarray(key, np.float32).tobytes())
    out = subprocess.run([PIN], input=b"".join(buf), stdout=subprocess.PIPE, check=True).stdout
    idx, dist = [], []
    rec = 8 * K + 4 * K
    for q in range(len(queries)):
        r = out[q * rec:(q + 1) * rec]
        idx.append(np.frombuffer(r[:8 * K], np.uint64).astype(np.int64))
        dist.append(np.frombuffer(r[8 * K:], np.float32))
    return np.array(idx), np.array(dist)


def make_sc():
    cfg = O.preset(SC_PRESET)
    NR, EXC, PER = cfg.sc_num_ring, cfg.sc_num_exclude_recent, cfg.sc_tree_making_period
    ses = O.SCSession(cfg, stable_voxel=False)
    keys, n_ds, det = [], [], []
    snaps, counter = None, 0
    queries = []
    for j in range(SC_N):
        pts = O.gen_scan(SC_PRESET, SC_CONFIG, SC_STREAM, j * SC_STEP)
        n, key = ses.add(pts)
        keys.append(key)
        n_ds.append(n)
        d = ses.detect()
        if len(keys) >= EXC + 1:
            if counter % PER == 0:
                snaps = len(keys) - EXC
            counter += 1
            queries.append((j, snaps))
        det.append(d)
    keys = np.array(keys, np.float32)
    q = [(keys[:s], keys[j]) for j, s in queries]
    i10, d10 = nanoflann(q, NR, 10)
    i50, d50 = nanoflann(q, NR, 50)
    qj = np.array([j for j, _ in queries], np.int32)
    cand = np.array([det[j]["cand"] for j in qj], np.int32)
    out = dict(
        preset=np.int32(SC_PRESET), config=np.int32(SC_CONFIG), stream=np.int32(SC_STREAM), step=np.int32(SC_STEP),
        ring_keys=keys, n_ds=np.array(n_ds, np.int32), query_frame=qj,
        snapshot=np.array([s for _, s in queries], np.int32),
        nf_idx10=i10, nf_dist10=d10, nf_idx50=i50, nf_dist50=d50,
        loop_id=np.array([det[j]["loop_id"] for j in range(SC_N)], np.int32),
        nn_idx=np.array([det[j]["nn_idx"] for j in range(SC_N)], np.int32),
        yaw=np.array([det[j]["yaw"] for j in range(SC_N)], np.float64),
        min_dist=np.array([det[j]["min_dist"] for j in range(SC_N)], np.float64),
        cand10=cand,
    )
    np.savez_compressed(os.path.join(HERE, "sc_loop_hdl64.npz"), **out)
    loops = int((out["loop_id"] >= 0).sum())
    print(f"sc_loop_hdl64: {SC_N} keyframes, {len(qj)} detects, {loops} loops")


def make_front(name, pid, config, n_scans):
    rows = F.oracle_rows(O, pid, config, n_scans)
    with open(os.path.join(HERE, f"front_{name}.json"), "w") as f:
        json.dump({"preset": pid, "config": config, "stream": 0, "stable_voxel": False, "scans": rows}, f, indent=1)
    print(f"front_{name}: {n_scans} scans")


if __name__ == "__main__":
    if not os.path.exists(PIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    for name, (pid, config, n) in FRONT.items():
        make_front(name, pid, config, n)
    make_sc()
