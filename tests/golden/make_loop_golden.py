"""Generate tests/golden/loop_vlp16.npz — the loop-closure verification
fixture (oracle/oracle_lc.h):

  python tests/golden/make_loop_golden.py

A synthetic VLP-16 stream (preset 0, config 1, stream 0) sampled every 2nd
scan (2 m per scan, so one 606 m lap takes ~303 scans) runs through the
oracle's whole pipeline with cfg.loop_verify = 1 (stable in-voxel VoxelGrid
order, the order the GPU produces) for LOOP_SCANS scans at t = 0.1 s * k.
Every SC detect that finds a candidate records the two LoopResult records
(radius-search and Scan Context ICP verification).  The first lap yields
false SC candidates that ICP rejects (fitness > 1.5); the second lap closes
true loops that it accepts.  Parity of the restatement with PCL / Eigen
themselves is unpinned (they are absent here); this fixture pins the
restatement against regressions and is what the GPU path is checked against.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_py as O  # noqa: E402

LOOP_PRESET, LOOP_CONFIG, LOOP_STREAM, LOOP_STRIDE, LOOP_SCANS = 0, 1, 0, 2, 360
LOOP_ARCHIVE = 1 << 22


def loop_config(pid=LOOP_PRESET):
    cfg = O.preset(pid)
    cfg.loop_verify = 1
    cfg.loop_archive_points = LOOP_ARCHIVE
    return cfg


def run_oracle(n_scans=LOOP_SCANS):
    cfg = loop_config()
    st = O.OracleStream(cfg, stable_voxel=False)
    scans, nkf, det, loops = [], [], [], []
    for k in range(n_scans):
        pts = O.gen_scan(LOOP_PRESET, LOOP_CONFIG, LOOP_STREAM, k * LOOP_STRIDE)
        f = st.step(pts, k * 0.1)
        if f & 8:
            d = st.get("detect")
            lp = st.get("loop")
            if d[0] >= 0 or lp[0]["id"] >= 0:
                scans.append(k)
                nkf.append(int(st.get("n_keyframes")[0]))
                det.append(int(d[0]))
                loops.append(lp.copy())
    return (np.array(scans, np.int32), np.array(nkf, np.int32), np.array(det, np.int32),
            np.stack(loops) if loops else np.zeros((0, 2), O.LOOP_DTYPE))


def main():
    scans, nkf, det, loops = run_oracle()
    path = os.path.join(HERE, "loop_vlp16.npz")
    np.savez_compressed(path, scans=scans, n_keyframes=nkf, sc_id=det,
                        loop_bytes=np.frombuffer(loops.tobytes(), np.uint8).reshape(len(scans), -1))
    acc = loops["accepted"]
    print(f"{path}: {len(scans)} detects with a candidate, RS ran {int(loops['ran'][:, 0].sum())}, "
          f"SC accepted {int(acc[:, 1].sum())} / rejected {int((1 - acc[:, 1]).sum())}")


if __name__ == "__main__":
    main()
