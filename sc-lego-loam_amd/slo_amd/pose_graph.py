"""Pose-graph back end through the C ABI (include/slo_abi.h, csrc/slo_pg.hip).

Mirrors how mapOptimization drives GTSAM iSAM2 (SC-LeGO-LOAM
LeGO-LOAM/src/mapOptmization.cpp): ``add_keyframe`` is the graph half of
saveKeyFramesAndFactor (MO:1541-1611), ``add_loop`` + ``optimize`` the loop
factor and the ``isam->update`` calls after it (MO:1038-1046, 1083-1091), and
``key_poses`` is correctPoses (MO:1642-1664).
"""
import ctypes

import numpy as np

from . import _abi

_BOUND = False


def _lib():
    global _BOUND
    L = _abi.lib()
    if not _BOUND:
        P, F6 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)
        L.slo_pg_create.argtypes = [ctypes.POINTER(P)]
        L.slo_pg_destroy.argtypes = [P]
        L.slo_pg_destroy.restype = None
        L.slo_pg_last_error.argtypes = [P]
        L.slo_pg_last_error.restype = ctypes.c_char_p
        L.slo_pg_size.argtypes = [P]
        L.slo_pg_add_keyframe.argtypes = [P, F6, F6, F6]
        L.slo_pg_add_loop.argtypes = [P, ctypes.c_int, ctypes.c_int, F6, F6]
        L.slo_pg_optimize.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
        L.slo_pg_get_key_poses.argtypes = [P, F6, ctypes.c_int]
        L.slo_pg_last_transform.argtypes = [P, F6]
        _BOUND = True
    return L


def _f6(v):
    a = np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(6))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class PoseGraph:
    """The key-pose factor graph of one map (one stream)."""

    def __init__(self):
        self._L = _lib()
        self._g = ctypes.c_void_p()
        rc = self._L.slo_pg_create(ctypes.byref(self._g))
        if rc != 0:
            raise RuntimeError(f"slo_pg_create failed ({rc})")

    def _check(self, rc):
        if rc < 0:
            raise RuntimeError(self._L.slo_pg_last_error(self._g).decode())
        return rc

    def __del__(self):
        if getattr(self, "_g", None):
            self._L.slo_pg_destroy(self._g)
            self._g = None

    def __len__(self):
        return self._L.slo_pg_size(self._g)

    def add_keyframe(self, transform):
        """transformAftMapped (LeGO order) → (updated transform, cloudKeyPoses6D entry)."""
        t, tp = _f6(transform)
        out, op = _f6(np.zeros(6))
        kp, kpp = _f6(np.zeros(6))
        self._check(self._L.slo_pg_add_keyframe(self._g, tp, op, kpp))
        return out.copy(), kp.copy()

    def add_loop(self, from_id, to_id, pose_from, pose_to):
        a, ap = _f6(pose_from)
        b, bp = _f6(pose_to)
        self._check(self._L.slo_pg_add_loop(self._g, int(from_id), int(to_id), ap, bp))

    def optimize(self, max_iters=100):
        """(iterations, final cost); ``self.converged`` is False when max_iters ran out first"""
        it, cost = ctypes.c_int(), ctypes.c_double()
        rc = self._L.slo_pg_optimize(self._g, int(max_iters), ctypes.byref(it), ctypes.byref(cost))
        self._check(rc)
        self.converged = rc == 0
        return it.value, cost.value

    def key_poses(self):
        n = len(self)
        out = np.zeros((max(n, 1), 6), np.float32)
        self._check(self._L.slo_pg_get_key_poses(self._g, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n))
        return out[:n]
