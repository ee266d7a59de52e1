"""slo_amd — MI355X-native SC-LeGO-LOAM per-scan hot path (host mirror).

Python view of libslo.so (include/slo_abi.h).  The classes mirror the
reference's node interfaces for the hot path:

  ImageProjection.cloudHandler        imageProjection.cpp:181
  FeatureAssociation.runFeatureAssociation  featureAssociation.cpp:1817
  MapOptimization.run                 mapOptmization.cpp:1673
  SCManager.detectLoopClosureID       Scancontext.h:73

and `Pipeline` drives the batched path (one scan per stream per call) that
bench.py measures.  Device memory for batched inputs is owned by torch
(plumbing only); all compute is the HIP kernels in csrc/.
"""
import ctypes

import numpy as np

from . import _abi
from ._abi import SloConfig, SegView, FaView, MapView, IMU_DTYPE
from . import wire

PRESETS = {
    "vlp16": 0, "hdl32": 1, "vls128": 2, "os1_16": 3, "os1_64": 4,
    "os64_1800": 5, "hdl64_1800": 6, "dense128": 7,
}

_CLOUD_OUT = {"full_cloud", "seg_pts", "outlier", "fa_seg_pts", "sharp", "less_sharp", "flat", "less_flat",
              "corner_last", "surf_last", "raw_ds", "corner_ds", "surf_total_ds", "map_corner_ds", "map_surf_ds"}
_DT = {"map_ids": np.int32, "map_raw_n": np.int32, "range": np.float32, "label": np.int32, "ground": np.int8, "seg_ground": np.uint8,
       "seg_col": np.uint32, "seg_range": np.float32, "ring_start": np.int32, "ring_end": np.int32,
       "orient": np.float32, "curvature": np.float32, "picked": np.int32, "cloud_label": np.int32,
       "smooth_ind": np.int32, "transform_sum": np.float32, "transform_cur": np.float32, "integrated": np.float32,
       "fa_iters": np.int32, "mapped": np.float32, "n_keyframes": np.int32, "flags": np.int32,
       "keyposes": np.float32, "sc_desc": np.float64, "ring_key": np.float64, "sector_key": np.float64,
       "detect": np.int32, "detect_f": np.float64, "mo_iters": np.int32, "tobe_mapped": np.float32,
       "err": np.int32, "dbg": np.uint64, "key_times": np.float64}
# slo_loop_result (include/slo_abi.h), one per candidate: [RS, SC]
LOOP_DTYPE = np.dtype([("id", "<i4"), ("ran", "<i4"), ("converged", "<i4"), ("accepted", "<i4"), ("iters", "<i4"),
                       ("n_src", "<i4"), ("n_tgt", "<i4"), ("pad", "<i4"), ("fitness", "<f8"),
                       ("T", "<f4", (16,)), ("xyzrpy", "<f4", (6,))])
assert LOOP_DTYPE.itemsize == 128
_DT["loop"] = LOOP_DTYPE
_DT["imu"] = np.float64
_DT["vg_in"] = np.int32
_DT["vg_stats"] = np.int32
_DT["pcl_work"] = np.uint64
_DT["work"] = np.uint64      # DevView::wctr: [0] Scan Context pairs whose distance was evaluated, [1] / [2] long-voxel
                             # points / voxels (k_vg_long)
_DT["counts"] = np.int32     # the stream's cloud sizes in one read (slo_get "counts", csrc/slo_ctx.hip)


class SloError(RuntimeError):
    pass


def preset(name_or_id):
    pid = PRESETS.get(name_or_id, name_or_id)
    c = SloConfig()
    if _abi.lib().slo_config_preset(int(pid), ctypes.byref(c)) != 0:
        raise ValueError(f"unknown preset {name_or_id}")
    return c


def gen_batch(preset_id, config_id, stream0, n_streams, scan0, n_scans, n_points, n_threads=8, out=None):
    """[n_scans][n_streams][n_points][4] float32 synthetic scans (host threads)."""
    if out is None:
        out = np.empty((n_scans, n_streams, n_points, 4), np.float32)
    rc = _abi.lib().slo_gen_batch(int(preset_id), int(config_id), int(stream0), int(n_streams), int(scan0),
                                  int(n_scans), out.ctypes.data, int(n_threads))
    if rc != 0:
        raise SloError("slo_gen_batch failed")
    return out


class DeviceGenerator:
    """slo_gen on the device (csrc/slo_gendev.hip): the scans gen_batch makes,
    bit for bit, written straight into device memory."""

    def __init__(self, preset_id, config_id, stream0, n_streams, device=0):
        preset_id = PRESETS.get(preset_id, preset_id)
        self.L = _abi.lib()
        self.h = ctypes.c_void_p()
        self.n_streams = n_streams
        self.max_points = preset(preset_id).max_points
        rc = self.L.slo_gen_device_create(int(preset_id), int(config_id), int(stream0), int(n_streams), int(device),
                                          ctypes.byref(self.h))
        if rc != 0:
            raise SloError(f"slo_gen_device_create failed ({rc})")

    def scans(self, scan0, n_scans, d_out, hip_stream=None):
        """write scans scan0 .. scan0+n_scans-1 of every stream to the device
        pointer d_out ([n_scans][n_streams][max_points][4] float32)"""
        per_scan = self.n_streams * self.max_points * 16
        step = max(1, 65535 // self.n_streams)
        for k in range(0, n_scans, step):
            nk = min(step, n_scans - k)
            rc = self.L.slo_gen_device_scans(self.h, int(scan0 + k), int(nk), ctypes.c_void_p(int(d_out) + k * per_scan),
                                             hip_stream)
            if rc != 0:
                raise SloError(f"slo_gen_device_scans failed ({rc})")

    def close(self):
        if self.h:
            self.L.slo_gen_device_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gen_scan(preset_id, config_id, stream_id, k, n_points):
    out = np.empty((n_points, 4), np.float32)
    n = _abi.lib().slo_gen_scan(int(preset_id), int(config_id), int(stream_id), int(k), out.ctypes.data)
    if n < 0:
        raise SloError("slo_gen_scan failed")
    return out[:n]


class Context:
    """One libslo context: `n_streams` independent streams on HIP device `device`."""

    def __init__(self, cfg, device=0, n_streams=1):
        self.L = _abi.lib()
        self.cfg = cfg
        self.n_streams = n_streams
        h = ctypes.c_void_p()
        rc = self.L.slo_create(ctypes.byref(cfg), int(device), int(n_streams), ctypes.byref(h))
        if rc != 0:
            raise SloError(f"slo_create failed ({rc})")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.slo_destroy(self.h)
            self.h = None

    __del__ = close

    def _ok(self, rc, what):
        if rc != 0:
            raise SloError(f"{what}: {rc} {self.L.slo_last_error(self.h).decode()}")

    @property
    def stream_handle(self):
        return self.L.slo_stream(self.h)

    def synchronize(self):
        self._ok(self.L.slo_synchronize(self.h), "slo_synchronize")

    def pipeline(self, depth=6):
        """slo_pipeline: the front end, the odometry and the mapping stage of
        every scan on three HIP streams of this one context (depth: the
        buffer rings; 0 = off), bit-identical to the context without it"""
        self._ok(self.L.slo_pipeline(self.h, int(depth)), "slo_pipeline")

    def prepare_mapping(self):
        """slo_prepare_mapping: the mapping step's workspaces now (a caller
        budgeting HBM measures free memory after this)"""
        self._ok(self.L.slo_prepare_mapping(self.h), "slo_prepare_mapping")

    # batched, device pointers (int addresses)
    def batch_image_projection(self, d_pts, d_cnt):
        self._ok(self.L.slo_batch_image_projection(self.h, d_pts, d_cnt), "slo_batch_image_projection")

    def batch_pc2_unpack(self, d_bytes, msg_stride, d_dims, layout, d_pts, d_cnt, d_rings=None):
        """slo_batch_pc2_unpack: one raw PointCloud2 payload per stream (device
        bytes, message s at s * msg_stride, d_dims int32 [S][3] = width,
        height, row_step) -> the d_pts / d_cnt of batch_image_projection
        (and, if given, each point's uint16 ring into d_rings)."""
        self._ok(self.L.slo_batch_pc2_unpack(self.h, d_bytes, msg_stride, d_dims, ctypes.byref(layout), d_pts,
                                             d_cnt, d_rings), "slo_batch_pc2_unpack")

    def batch_set_rings(self, d_rings):
        """slo_batch_set_rings (cfg.use_cloud_ring): device uint16 [S][max_points]"""
        self._ok(self.L.slo_batch_set_rings(self.h, d_rings), "slo_batch_set_rings")

    def batch_feature_association(self):
        self._ok(self.L.slo_batch_feature_association(self.h), "slo_batch_feature_association")

    def batch_process(self, d_pts, d_cnt, t_scan):
        self._ok(self.L.slo_batch_process(self.h, d_pts, d_cnt, float(t_scan)), "slo_batch_process")

    def batch_imu(self, d_msgs, msgs_per_stream, d_counts):
        """slo_batch_imu: device IMU_DTYPE [S][msgs_per_stream], device int32 counts [S] -> each stream's imuHandler"""
        self._ok(self.L.slo_batch_imu(self.h, d_msgs, int(msgs_per_stream), d_counts), "slo_batch_imu")

    def scan_time(self, t_scan):
        """slo_batch_scan_time: the stamp the next feature step deskews against the IMU ring"""
        self._ok(self.L.slo_batch_scan_time(self.h, float(t_scan)), "slo_batch_scan_time")

    def imu_handler(self, msg):
        """slo_imu_handler (one-stream context): msg = one IMU_DTYPE record"""
        m = np.ascontiguousarray(np.asarray(msg, _abi.IMU_DTYPE).reshape(1))
        self._ok(self.L.slo_imu_handler(self.h, m.ctypes.data), "slo_imu_handler")

    def graph_mode(self, on=True):
        """slo_graph_mode: replay captured HIP graphs in batch_process (default) or launch eagerly"""
        self._ok(self.L.slo_graph_mode(self.h, 1 if on else 0), "slo_graph_mode")

    def batch_sc_make(self, d_pts, d_cnt):
        self._ok(self.L.slo_batch_sc_make(self.h, d_pts, d_cnt), "slo_batch_sc_make")

    def batch_voxel_grid(self, d_in, in_stride, d_n, leaf, d_out, out_stride, d_nout, out_cap):
        """pcl::VoxelGrid filter of every stream's device cloud (slo_batch_voxel_grid); asynchronous"""
        self._ok(self.L.slo_batch_voxel_grid(self.h, d_in, int(in_stride), d_n, float(leaf), d_out, int(out_stride),
                                             d_nout, int(out_cap)), "slo_batch_voxel_grid")

    def batch_loop_closure(self):
        """RS + SC loop verification (MO:841-1110) for every stream whose SC detect ran."""
        self._ok(self.L.slo_batch_loop_closure(self.h), "slo_batch_loop_closure")

    def loop_closure(self):
        """stream 0: -> LOOP_DTYPE[2] (RS, SC)"""
        out = np.zeros(2, LOOP_DTYPE)
        self._ok(self.L.slo_loop_closure(self.h, out.ctypes.data), "slo_loop_closure")
        return out

    def icp_align_batch(self, d_src, src_stride, d_nsrc, d_tgt, tgt_stride, d_ntgt):
        """pcl::IterativeClosestPoint::align + getFitnessScore per stream on
        device clouds -> LOOP_DTYPE[n_streams]"""
        out = np.zeros(self.n_streams, LOOP_DTYPE)
        self._ok(self.L.slo_icp_align_batch(self.h, d_src, int(src_stride), d_nsrc, d_tgt, int(tgt_stride), d_ntgt,
                                            out.ctypes.data), "slo_icp_align_batch")
        return out

    def pack_records(self, d_out):
        self._ok(self.L.slo_pack_records(self.h, d_out), "slo_pack_records")

    def sc_make_and_save(self, pts_xyzi):
        pts = np.ascontiguousarray(pts_xyzi, np.float32)
        self._ok(self.L.slo_sc_make_and_save(self.h, pts.ctypes.data, len(pts), 16, 0, 12), "slo_sc_make_and_save")

    def sc_detect(self):
        lid, yaw, md = ctypes.c_int32(), ctypes.c_float(), ctypes.c_double()
        self._ok(self.L.slo_sc_detect(self.h, ctypes.byref(lid), ctypes.byref(yaw), ctypes.byref(md)), "slo_sc_detect")
        return int(lid.value), float(yaw.value), float(md.value)

    def get(self, stream, name):
        n = self.L.slo_get(self.h, int(stream), name.encode(), None, 0)
        if n < 0:
            raise SloError(f"slo_get({name}) -> {n}")
        out = np.empty((n, 4), np.float32) if name in _CLOUD_OUT else np.empty(n, _DT[name])
        if n:
            rc = self.L.slo_get(self.h, int(stream), name.encode(), out.ctypes.data, out.nbytes)
            if rc < 0:
                raise SloError(f"slo_get({name}) -> {rc}")
        return out

    # per-kernel timing (HIP events)
    def timing(self, enable=True):
        self._ok(self.L.slo_timing_enable(self.h, int(enable)), "slo_timing_enable")

    def timing_filter(self, name=None):
        """time only launches named `name` (None: all)"""
        self._ok(self.L.slo_timing_filter(self.h, name.encode() if name else None), "slo_timing_filter")

    def timing_reset(self):
        self._ok(self.L.slo_timing_reset(self.h), "slo_timing_reset")

    def timing_read(self):
        cap = 256
        buf = ctypes.create_string_buffer(32768)
        ms = (ctypes.c_double * cap)()
        cnt = (ctypes.c_int64 * cap)()
        n = self.L.slo_timing_read(self.h, buf, 32768, ms, cnt, cap)
        names = buf.raw.split(b"\0")[:n]
        return {names[i].decode(): (ms[i], cnt[i]) for i in range(n)}


def _arr(ptr, n, dtype, cols=None):
    """Copy a view array (context-owned host memory) into numpy."""
    shape = (n, cols) if cols else (n,)
    if not n or not ptr:
        return np.empty(shape, dtype)
    nbytes = n * (cols or 1) * np.dtype(dtype).itemsize
    return np.frombuffer(ctypes.string_at(ptr, nbytes), dtype).reshape(shape).copy()


class _Node:
    """Single-scan node mirrors share one one-stream Context (the reference
    runs the nodes as separate processes joined by topics; here the topics are
    the context's device buffers)."""

    def __init__(self, ctx):
        if ctx.n_streams != 1:
            raise SloError("node mirrors need a Context with n_streams == 1 (use the batch_* calls otherwise)")
        self.ctx = ctx


class ImageProjection(_Node):
    """Mirror of ImageProjection::cloudHandler (imageProjection.cpp:181-196).

    Returns the /segmented_cloud, /segmented_cloud_info and /outlier_cloud
    contents as numpy arrays."""

    def cloudHandler(self, points_xyzi, rings=None):
        """points_xyzi: (n, 4) float32 array, or a wire.PointCloud2 message
        (converted by pcl::fromROSMsg rules inside libslo, IP:167).  rings:
        uint16 per point for cfg.use_cloud_ring with an array input (a
        message brings its own "ring" field)."""
        v = SegView()
        if isinstance(points_xyzi, wire.PointCloud2):
            m = wire._CMsg(points_xyzi)
            self.ctx._ok(self.ctx.L.slo_image_projection_pc2(self.ctx.h, ctypes.byref(m.c), ctypes.byref(v)),
                         "slo_image_projection_pc2")
        else:
            pts = np.ascontiguousarray(points_xyzi, np.float32)
            r = None if rings is None else np.ascontiguousarray(rings, np.uint16)
            self.ctx._ok(self.ctx.L.slo_image_projection_ring(self.ctx.h, pts.ctypes.data, len(pts), 16, 0, 12,
                                                              None if r is None else r.ctypes.data,
                                                              ctypes.byref(v)), "slo_image_projection_ring")
        R = self.ctx.cfg.n_scan
        return {
            "seg_pts": _arr(v.segmented, v.n_segmented, np.float32, 4),
            "seg_ground": _arr(v.ground_flag, v.n_segmented, np.uint8),
            "seg_col": _arr(v.col_ind, v.n_segmented, np.uint32),
            "seg_range": _arr(v.range, v.n_segmented, np.float32),
            "ring_start": _arr(v.start_ring_index, R, np.int32),
            "ring_end": _arr(v.end_ring_index, R, np.int32),
            "orient": np.array([v.start_orientation, v.end_orientation, v.orientation_diff], np.float32),
            "outlier": _arr(v.outlier, v.n_outlier, np.float32, 4),
        }


class FeatureAssociation(_Node):
    """Mirror of FeatureAssociation::runFeatureAssociation (featureAssociation.cpp:1817-1859)
    and its imuHandler (FA:459-486)."""

    def imuHandler(self, msg):
        """one sensor_msgs/Imu as a slo_amd.IMU_DTYPE record or an 11-sequence
        (stamp, qx, qy, qz, qw, ax, ay, az, wx, wy, wz)"""
        m = np.asarray(msg)
        if m.dtype != _abi.IMU_DTYPE:
            m = np.ascontiguousarray(m, np.float64).reshape(-1, 11)[0].view(_abi.IMU_DTYPE)
        self.ctx.imu_handler(m)

    def runFeatureAssociation(self, t_scan=0.0):
        v = FaView()
        self.ctx._ok(self.ctx.L.slo_feature_association(self.ctx.h, float(t_scan), ctypes.byref(v)),
                     "slo_feature_association")
        return {"transform_sum": np.array(v.transform_sum[:], np.float32), "published": bool(v.published),
                "sharp": _arr(v.sharp, v.n_sharp, np.float32, 4), "flat": _arr(v.flat, v.n_flat, np.float32, 4),
                "corner_last": _arr(v.less_sharp, v.n_less_sharp, np.float32, 4),
                "surf_last": _arr(v.less_flat, v.n_less_flat, np.float32, 4)}


class TransformFusion(_Node):
    """Mirror of TransformFusion (transformFusion.cpp): no callbacks to drive,
    the device computes /integrated_to_init inside every odometry step."""

    def integrated(self, stream=0):
        """transformMapped (rx, ry, rz, tx, ty, tz) of the last scan (TF:186-219)"""
        return self.ctx.get(stream, "integrated")


class MapOptimization(_Node):
    """Mirror of mapOptimization::run (mapOptmization.cpp:1673-1706) minus
    GTSAM and publishing; `raw_xyzi` is the scan's raw cloud (/os1_points)."""

    def run(self, raw_xyzi, t_scan):
        pts = np.ascontiguousarray(raw_xyzi, np.float32)
        v = MapView()
        self.ctx._ok(self.ctx.L.slo_map_optimization(self.ctx.h, pts.ctypes.data, len(pts), 16, 0, 12,
                                                     float(t_scan), ctypes.byref(v)), "slo_map_optimization")
        return {"ran": bool(v.ran), "keyframe_saved": bool(v.keyframe_saved), "n_keyframes": v.n_keyframes,
                "transform_aft_mapped": np.array(v.transform_aft_mapped[:], np.float32)}

    def performLoopClosure(self):
        """detectLoopClosure + performLoopClosure (MO:841-1110) minus the GTSAM
        factors, after this keyframe's SCManager.detectLoopClosureID (context
        created with cfg.loop_verify = 1).  -> {"RS": record, "SC": record}
        with the LOOP_DTYPE fields (id, converged, accepted, fitness, T, ...)."""
        r = self.ctx.loop_closure()
        return {"RS": r[0], "SC": r[1]}


class SCManager:
    """Mirror of the public SCManager API (Scancontext.h:63-73) on stream 0 of
    a Context: makeAndSaveScancontextAndKeys / detectLoopClosureID, and the
    public helpers makeScancontext, makeRingkeyFromScancontext,
    makeSectorkeyFromScancontext, fastAlignUsingVkey, distDirectSC,
    distanceBtnScanContext (slo_sc_* in include/slo_abi.h).  Descriptors are
    (NR, NS) float64 arrays (ring, sector), as the reference's MatrixXd."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.NR, self.NS = ctx.cfg.sc_num_ring, ctx.cfg.sc_num_sector

    def _desc(self, d):
        d = np.ascontiguousarray(d, np.float64)
        if d.shape != (self.NR, self.NS):
            raise SloError(f"a descriptor is ({self.NR}, {self.NS}), got {d.shape}")
        return d

    def makeScancontext(self, scan_down_xyzi):
        p = np.ascontiguousarray(scan_down_xyzi, np.float32).reshape(-1, 4)
        d = np.zeros((self.NR, self.NS), np.float64)
        self.ctx._ok(self.ctx.L.slo_sc_make_scancontext(self.ctx.h, p.ctypes.data, len(p), 16, 0, d.ctypes.data),
                     "slo_sc_make_scancontext")
        return d

    def makeRingkeyFromScancontext(self, desc):
        d, k = self._desc(desc), np.zeros(self.NR, np.float64)
        self.ctx._ok(self.ctx.L.slo_sc_ring_key(self.ctx.h, d.ctypes.data, k.ctypes.data), "slo_sc_ring_key")
        return k

    def makeSectorkeyFromScancontext(self, desc):
        d, k = self._desc(desc), np.zeros(self.NS, np.float64)
        self.ctx._ok(self.ctx.L.slo_sc_sector_key(self.ctx.h, d.ctypes.data, k.ctypes.data), "slo_sc_sector_key")
        return k

    def fastAlignUsingVkey(self, vkey1, vkey2):
        a, b = (np.ascontiguousarray(v, np.float64).reshape(self.NS) for v in (vkey1, vkey2))
        sh = ctypes.c_int32(0)
        self.ctx._ok(self.ctx.L.slo_sc_fast_align(self.ctx.h, a.ctypes.data, b.ctypes.data, ctypes.byref(sh)),
                     "slo_sc_fast_align")
        return sh.value

    def distDirectSC(self, sc1, sc2):
        a, b = self._desc(sc1), self._desc(sc2)
        d = ctypes.c_double(0)
        self.ctx._ok(self.ctx.L.slo_sc_dist_direct(self.ctx.h, a.ctypes.data, b.ctypes.data, ctypes.byref(d)),
                     "slo_sc_dist_direct")
        return d.value

    def distanceBtnScanContext(self, sc1, sc2):
        """-> (min distance, shift) like the reference's std::pair<double, int>"""
        a, b = self._desc(sc1), self._desc(sc2)
        d, sh = ctypes.c_double(0), ctypes.c_int32(0)
        self.ctx._ok(self.ctx.L.slo_sc_distance(self.ctx.h, a.ctypes.data, b.ctypes.data, ctypes.byref(d),
                                                ctypes.byref(sh)), "slo_sc_distance")
        return d.value, sh.value

    def makeAndSaveScancontextAndKeys(self, scan_down_xyzi):
        self.ctx.sc_make_and_save(scan_down_xyzi)

    def detectLoopClosureID(self):
        """-> (loop_id, yaw_rad) like the reference's std::pair<int, float>."""
        lid, yaw, _ = self.ctx.sc_detect()
        return lid, yaw
