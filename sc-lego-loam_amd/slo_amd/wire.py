"""sensor_msgs/PointCloud2 on the host side.

`PointField` / `PointCloud2` mirror the ROS message classes field for field
(header left out: the scan time is passed separately, as everywhere in
slo_amd).  `fromROSMsg` is pcl::fromROSMsg into PointXYZI as
ImageProjection::copyPointCloud calls it (imageProjection.cpp:167); the
conversion itself runs in libslo (slo_pc2_to_xyzi, csrc/slo_wire.hip), so
this module only marshals.  `pack` builds messages in the layouts LiDAR
drivers publish, for tests and for feeding recorded xyzi arrays through the
message path.
"""
import ctypes
from dataclasses import dataclass
from typing import List

import numpy as np

from . import _abi
from ._abi import Pc2, Pc2Field, Pc2Layout

INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 = range(1, 9)
_NP = {INT8: np.int8, UINT8: np.uint8, INT16: np.int16, UINT16: np.uint16, INT32: np.int32, UINT32: np.uint32,
       FLOAT32: np.float32, FLOAT64: np.float64}


@dataclass
class PointField:
    name: str
    offset: int
    datatype: int
    count: int = 1


@dataclass
class PointCloud2:
    height: int
    width: int
    fields: List[PointField]
    is_bigendian: bool
    point_step: int
    row_step: int
    data: bytes
    is_dense: bool = False


class _CMsg:
    """slo_pc2 view of a PointCloud2; keeps the buffers it points into alive."""

    def __init__(self, msg: PointCloud2):
        self._names = [f.name.encode() for f in msg.fields]
        self._fields = (Pc2Field * max(1, len(msg.fields)))()
        for k, f in enumerate(msg.fields):
            self._fields[k] = Pc2Field(self._names[k], f.offset, f.datatype, f.count)
        self._data = np.frombuffer(msg.data, np.uint8) if len(msg.data) else np.zeros(1, np.uint8)
        self.c = Pc2(msg.height, msg.width, self._fields, len(msg.fields), int(msg.is_bigendian), msg.point_step,
                     msg.row_step, self._data.ctypes.data, len(msg.data), int(msg.is_dense))


def _check(rc, what):
    if rc != 0:
        raise ValueError(f"{what}: {rc}")


def layout_of(msg: PointCloud2) -> Pc2Layout:
    """PCL's field mapping for PointXYZI (slo_pc2_layout_of)."""
    L = _abi.lib()
    out = Pc2Layout()
    _check(L.slo_pc2_layout_of(ctypes.byref(_CMsg(msg).c), ctypes.byref(out)), "slo_pc2_layout_of")
    return out


def fromROSMsg(msg: PointCloud2) -> np.ndarray:
    """pcl::fromROSMsg(msg, PointCloud<PointXYZI>) -> float32 (width*height, 4)."""
    L = _abi.lib()
    n = msg.width * msg.height
    out = np.zeros((max(n, 1), 4), np.float32)
    got = ctypes.c_size_t()
    _check(L.slo_pc2_to_xyzi(ctypes.byref(_CMsg(msg).c), out.ctypes.data, n, ctypes.byref(got)),
           "slo_pc2_to_xyzi")
    return out[:got.value]


# (name, offset, datatype) per driver layout; point_step last
LAYOUTS = {
    # pcl::PointXYZI as published by pcl_conversions (x y z, pad, intensity, pad to 32)
    "xyzi": ([("x", 0, FLOAT32), ("y", 4, FLOAT32), ("z", 8, FLOAT32), ("intensity", 16, FLOAT32)], 32),
    # velodyne_pointcloud PointXYZIR(+time)
    "velodyne": ([("x", 0, FLOAT32), ("y", 4, FLOAT32), ("z", 8, FLOAT32), ("intensity", 16, FLOAT32),
                  ("ring", 20, UINT16), ("time", 24, FLOAT32)], 32),
    # ouster_ros PointOS1 (the reference's default topic /os1_points, utility.h:57)
    "ouster": ([("x", 0, FLOAT32), ("y", 4, FLOAT32), ("z", 8, FLOAT32), ("intensity", 16, FLOAT32),
                ("t", 20, UINT32), ("reflectivity", 24, UINT16), ("ring", 26, UINT8), ("noise", 28, UINT16),
                ("range", 32, UINT32)], 48),
}


def pack(points_xyzi, layout="ouster", height=1, row_pad=0, intensity_type=FLOAT32, ring=None) -> PointCloud2:
    """A PointCloud2 holding `points_xyzi` (n, 4) in a driver layout, organised
    as `height` rows (n must divide) with `row_pad` bytes after every row.
    `intensity_type` other than FLOAT32 stores intensity as that integer type
    (the message PCL maps to 0)."""
    pts = np.ascontiguousarray(points_xyzi, np.float32).reshape(-1, 4)
    n = len(pts)
    assert height >= 1 and n % height == 0
    width = n // height
    spec, step = LAYOUTS[layout]
    row_step = width * step + row_pad
    buf = np.zeros(height * row_step, np.uint8)
    fields = []
    for name, off, dt in spec:
        if name == "intensity" and intensity_type != FLOAT32:
            dt = intensity_type
        fields.append(PointField(name, off, dt, 1))
        if n == 0:
            continue
        if name in ("x", "y", "z", "intensity"):
            src = pts[:, "xyz".index(name) if name != "intensity" else 3]
        elif name == "ring" and ring is not None:
            src = np.asarray(ring)
        elif name == "range":
            src = np.sqrt((pts[:, :3].astype(np.float64) ** 2).sum(1)) * 1000.0
        else:
            src = np.arange(n)
        vals = np.nan_to_num(src.astype(np.float64), nan=0.0) if dt != FLOAT32 and dt != FLOAT64 else src
        vals = np.asarray(vals).astype(_NP[dt])
        raw = vals.view(np.uint8).reshape(n, -1)
        for r in range(height):
            rows = buf[r * row_step: r * row_step + width * step].reshape(width, step)
            rows[:, off:off + raw.shape[1]] = raw[r * width:(r + 1) * width]
    return PointCloud2(height, width, fields, False, step, row_step, buf.tobytes(),
                       bool(np.isfinite(pts[:, :3]).all()))
