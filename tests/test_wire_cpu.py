"""PointCloud2 -> PointXYZI: slo_pc2_to_xyzi, host code
in libslo, against the driver layouts LiDARs publish and against an
independent numpy restatement of pcl::fromROSMsg's field mapping
(pcl/conversions.h FieldMapper / FieldMatches) on random messages.  PCL is
not in this image, so the restatement is the pin ("parity unpinned" beyond
the rules written down in csrc/slo_wire.hip)."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import oracle_py as O
from slo_amd import wire

SCAN = O.gen_scan(0, 1, 0, 0)   # VLP-16 scan with no-return NaNs


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32).tobytes()


@pytest.mark.parametrize("layout", ["xyzi", "velodyne", "ouster"])
@pytest.mark.parametrize("height,row_pad", [(1, 0), (16, 0), (16, 12), (1800, 4)])
def test_driver_layouts_round_trip(layout, height, row_pad):
    msg = wire.pack(SCAN, layout, height=height, row_pad=row_pad)
    assert msg.width * msg.height == len(SCAN)
    got = wire.fromROSMsg(msg)
    assert bits(got) == bits(SCAN)   # NaNs travel bit for bit: removal is the projection's job


def test_integer_intensity_maps_to_zero():
    # FieldMatches needs datatype FLOAT32: a UINT16 intensity is not matched
    # and PointXYZI keeps its constructed 0 (PCL only warns)
    msg = wire.pack(SCAN, "ouster", intensity_type=wire.UINT16)
    assert wire.layout_of(msg).off_intensity == -1
    got = wire.fromROSMsg(msg)
    assert (got[:, 3] == 0).all()
    assert bits(got[:, :3]) == bits(SCAN[:, :3])


def test_missing_fields_are_zero_and_first_match_wins():
    pts = SCAN[:64]
    msg = wire.pack(pts, "xyzi")
    # drop y, add a decoy intensity of the wrong count before the real one,
    # then a duplicate x pointing at z's bytes after the real x
    msg.fields = [wire.PointField("x", 0, wire.FLOAT32, 1), wire.PointField("intensity", 12, wire.FLOAT32, 2),
                  wire.PointField("z", 8, wire.FLOAT32, 0), wire.PointField("intensity", 16, wire.FLOAT32, 1),
                  wire.PointField("x", 8, wire.FLOAT32, 1)]
    got = wire.fromROSMsg(msg)
    want = pts.copy()
    want[:, 1] = 0
    assert bits(got) == bits(want)


def test_empty_and_malformed_messages():
    msg = wire.pack(SCAN[:0], "ouster")
    assert wire.fromROSMsg(msg).shape == (0, 4)
    msg = wire.pack(SCAN[:10], "ouster")
    msg.data = msg.data[:-1]   # last point cut short
    with pytest.raises(ValueError):
        wire.fromROSMsg(msg)
    msg = wire.pack(SCAN[:10], "ouster")
    msg.fields = [wire.PointField("x", 46, wire.FLOAT32, 1)]   # reaches past point_step
    with pytest.raises(ValueError):
        wire.fromROSMsg(msg)


def from_ros_msg_numpy(msg):
    """pcl::fromROSMsg into PointXYZI restated in numpy (independent of libslo)."""
    offs = []
    for name in ("x", "y", "z", "intensity"):
        off = -1
        for f in msg.fields:
            if f.name == name and f.datatype == wire.FLOAT32 and f.count in (0, 1):
                off = f.offset
                break
        offs.append(off)
    data = np.frombuffer(msg.data, np.uint8)
    out = np.zeros((msg.width * msg.height, 4), np.float32)
    for r in range(msg.height):
        for c in range(msg.width):
            base = r * msg.row_step + c * msg.point_step
            for k, off in enumerate(offs):
                if off >= 0:
                    out[r * msg.width + c, k] = data[base + off: base + off + 4].copy().view(np.float32)[0]
    return out


NAMES = ["x", "y", "z", "intensity", "ring", "t", "X"]


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**31 - 1), width=st.integers(0, 12), height=st.integers(1, 4),
       step=st.integers(4, 40), pad=st.integers(0, 9), nf=st.integers(0, 8))
def test_field_mapping_matches_restatement(seed, width, height, step, pad, nf):
    rng = np.random.default_rng(seed)
    fields = []
    for _ in range(nf):
        fields.append(wire.PointField(str(rng.choice(NAMES)), int(rng.integers(0, step - 3)),
                                      int(rng.choice([wire.FLOAT32, wire.FLOAT32, wire.UINT16, wire.FLOAT64])),
                                      int(rng.choice([0, 1, 1, 3]))))
    row_step = width * step + pad
    data = rng.integers(0, 256, size=height * row_step, dtype=np.uint8).tobytes()
    msg = wire.PointCloud2(height, width, fields, False, step, row_step, data)
    got = wire.fromROSMsg(msg)
    want = from_ros_msg_numpy(msg)
    assert bits(got) == bits(want)


def test_oracle_cloud_ring_rows():
    # useCloudRing (IP:225-226): every point's row is its ring; rings >= N_SCAN
    # are dropped (IP:232); the ring is read at the index after NaN removal
    cfg = O.preset(0)
    cfg.use_cloud_ring = 1
    R, C = cfg.n_scan, cfg.horizon_scan
    orc = O.OracleStream(cfg, stable_voxel=False)
    n_fin = int(np.isfinite(SCAN[:, :3]).all(axis=1).sum())
    rings = np.full(len(SCAN), 3, np.uint16)
    rings[n_fin // 2:] = R + 1   # the second half of the finite points: out of range
    orc.set_rings(rings)
    orc.image_projection(SCAN)
    rng = orc.get("range").reshape(R, C)
    empty = rng[0, 0]
    assert (rng[np.arange(R) != 3] == empty).all()
    filled = int((rng[3] != empty).sum())
    assert 0 < filled <= n_fin // 2
