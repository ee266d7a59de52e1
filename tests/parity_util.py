"""Shared helpers for parity tests: run the same synthetic scans through the
oracle (CPU restatement) and libslo (GPU) and compare."""
import numpy as np


def bits(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.float32:
        return a.view(np.uint32)
    if a.dtype == np.float64:
        return a.view(np.uint64)
    return a


def same_bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    return bool(np.array_equal(bits(a), bits(b)))


def mismatch(a, b):
    """count of differing elements (bitwise; NaN==NaN by bits)"""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return -1
    d = bits(a) != bits(b)
    if d.ndim > 1:
        d = d.any(axis=tuple(range(1, d.ndim)))
    return int(d.sum())


def seg_class(label):
    """segmentation classes that matter downstream: -1 (ground/none), 0,
    999999 (rejected), positive feasible segment"""
    out = np.where(label > 0, 1, label)
    out = np.where(label == 999999, 2, out)
    return out.astype(np.int32)


def make_scans(preset_id, config_id, n_streams, n_scans, oracle_mod):
    return [[oracle_mod.gen_scan(preset_id, config_id, s, k) for k in range(n_scans)] for s in range(n_streams)]


def canon_smooth(smooth_ind, curv, seg_ground, ring_start, ring_end, edge_th, surf_th):
    """cloudSmoothness indices with the one freedom the pipeline cannot observe
    removed: inside a group of equal curvatures of a sector, only the order of
    the pick candidates is read (FA:704-705, 737-738: one list per curvature
    value), so non-candidates are put last in index order and candidates keep
    their relative order.  Positions below 5 (the stale entry 4 that the next
    scan reads, Q5) and every position outside the sorted ranges are compared
    as they are."""
    out = np.array(smooth_ind, np.int64, copy=True)
    S = len(seg_ground)
    for r in range(len(ring_start)):
        a, b = int(ring_start[r]), int(ring_end[r])
        for j in range(6):
            sp, ep = (a * (6 - j) + b * j) // 6, (a * (5 - j) + b * (j + 1)) // 6 - 1
            sp = max(sp, 5)
            if sp >= ep:
                continue
            inds = out[sp:ep]
            ok = inds < S
            if not ok.all():
                continue
            c = curv[inds]
            g = seg_ground[inds]
            cand = ((c > edge_th) & (g == 0)) | ((c < surf_th) & (g == 1))
            cb = c.view(np.uint32).astype(np.int64)
            key2 = np.where(cand, np.arange(len(inds)), len(inds) + inds)
            order = np.lexsort((key2, ~cand, cb))
            out[sp:ep] = inds[order]
    return out.astype(np.int32)
