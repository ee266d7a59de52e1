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
