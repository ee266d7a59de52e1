"""Cross-stream Scan Context candidates over the all-gathered records
(csrc/slo_xsc.hip).

Every rank all-gathers one record per stream per step (Context.pack_records,
slo_amd.dist.gather_records).  A CrossSession on each rank ingests the whole
gathered table — the descriptors of the streams that saved a keyframe — and
answers, for the rank's own streams, SCManager::detectLoopClosureID
(Scancontext.cpp:247-338) against every other stream's history.
"""
import ctypes

import numpy as np

from . import _abi

MATCH_DTYPE = np.dtype([("valid", np.int32), ("n_cand", np.int32), ("nn_stream", np.int32),
                        ("nn_keyframe", np.int32), ("loop", np.int32), ("yaw", np.float32),
                        ("min_dist", np.float64)])
assert MATCH_DTYPE.itemsize == ctypes.sizeof(_abi.XscMatch)


class CrossSession:
    """Descriptor history of `n_streams` global streams, `cap` keyframes each, on HIP device `device`."""

    def __init__(self, cfg, n_streams, cap=64, device=0):
        self.L = _abi.lib()
        self.h = ctypes.c_void_p()
        self.n_streams = n_streams
        rc = self.L.slo_xsc_create(ctypes.byref(cfg), int(device), int(n_streams), int(cap), ctypes.byref(self.h))
        if rc != 0:
            raise RuntimeError(f"slo_xsc_create failed ({rc})")

    def ingest(self, d_records, hip_stream=None):
        """d_records: device pointer to the gathered [n_streams][RECORD_FLOATS] table"""
        rc = self.L.slo_xsc_ingest(self.h, ctypes.c_void_p(int(d_records)), self.n_streams, hip_stream)
        if rc != 0:
            raise RuntimeError(f"slo_xsc_ingest failed ({rc})")

    def query(self, d_records, n_query, global0, d_out, hip_stream=None):
        """detect for records [global0, global0 + n_query) (device pointer to their rows) into d_out
        (device memory, n_query x slo_xsc_match)"""
        rc = self.L.slo_xsc_query(self.h, ctypes.c_void_p(int(d_records)), int(n_query), int(global0),
                                  ctypes.c_void_p(int(d_out)), hip_stream)
        if rc != 0:
            raise RuntimeError(f"slo_xsc_query failed ({rc})")

    def close(self):
        if self.h:
            self.L.slo_xsc_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
