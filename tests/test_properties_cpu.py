"""Property tests (hypothesis) of the CPU restatement — SURVEY §4's extra
pins for a reference that ships no tests: Scan Context shift identities,
VoxelGrid invariants against an independent numpy restatement, and rigid
motions for Umeyama / ICP.  Every case is generated from a seed, so a
failure reproduces from hypothesis' printed example."""
import ctypes

import numpy as np
import pytest
from hypothesis import HealthCheck, example, given, settings, strategies as st

import oracle_py as O

CFG = O.preset(6)
NR, NS = CFG.sc_num_ring, CFG.sc_num_sector
FAST = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def sc_distance(a, b):
    """SCManager::distanceBtnScanContext (Scancontext.cpp:116-148) -> (distance, shift)"""
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    shift = ctypes.c_int()
    d = O.lib().oracle_sc_distance(ctypes.byref(CFG), a.ctypes.data, b.ctypes.data, ctypes.byref(shift))
    return d, shift.value


@FAST
@given(seed=st.integers(0, 2**31 - 1), k=st.integers(0, NS - 1), empty=st.integers(0, 20))
def test_sc_distance_recovers_a_column_shift(seed, k, empty):
    # sc2 = sc1 rotated by k sectors: distDirectSC compares column j of sc1
    # with column j - shift of sc2 (SCc:69-90), so the match is shift = -k
    rng = np.random.default_rng(seed)
    a = rng.uniform(0.5, 30.0, size=(NR, NS))
    a[:, rng.choice(NS, empty, replace=False)] = 0.0   # empty sectors: zero-norm columns are skipped
    d, sh = sc_distance(a, np.roll(a, k, axis=1))
    assert sh == (NS - k) % NS
    assert abs(d) < 1e-12


@FAST
@given(seed=st.integers(0, 2**31 - 1), scale=st.floats(0.1, 10.0))
def test_sc_distance_is_scale_invariant_and_bounded(seed, scale):
    # cosine similarity per column: scaling one descriptor changes nothing;
    # 1 - mean(cos) of non-negative columns lies in [0, 1]
    rng = np.random.default_rng(seed)
    a = rng.uniform(0.0, 20.0, size=(NR, NS))
    b = rng.uniform(0.0, 20.0, size=(NR, NS))
    d1, s1 = sc_distance(a, b)
    d2, s2 = sc_distance(a, b * scale)
    assert s1 == s2 and abs(d1 - d2) < 1e-12
    assert -1e-12 <= d1 <= 1.0 + 1e-12


def voxel_grid_numpy(pts, leaf):
    """PCL VoxelGrid (stable in-voxel order) restated independently in numpy float32."""
    p = pts.astype(np.float32)
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = p[:, :3].min(axis=0), p[:, :3].max(axis=0)
    # PCL's int32 guard (voxel_grid.cpp applyFilter): when the cell count of
    # the bounding box overflows int32 the filter warns and returns the input
    cells = [int(np.float32((mx[a] - mn[a]) * inv)) + 1 for a in range(3)]
    if cells[0] * cells[1] * cells[2] > 2**31 - 1:
        return p.copy()
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    div = maxb - minb + 1
    ijk = (np.floor(p[:, :3] * inv) - minb.astype(np.float32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(idx, kind="stable")
    out = []
    for v in np.unique(idx):
        members = order[idx[order] == v]
        acc = np.zeros(4, np.float32)
        for m in members:   # one float chain per field, in input order
            acc = (acc + p[m]).astype(np.float32)
        out.append(acc / np.float32(len(members)))
    return np.array(out, np.float32).reshape(-1, 4)


@FAST
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(1, 400), leaf=st.sampled_from([0.2, 0.3, 0.4, 0.5]),
       spread=st.floats(0.5, 40.0))
@example(seed=0, n=365, leaf=0.2, spread=40.0)   # 1368*1355*1165 cells > 2^31-1: the input comes back
@example(seed=1, n=50, leaf=0.5, spread=1.0)     # far below the guard: a real filter
def test_voxel_grid_matches_independent_restatement(seed, n, leaf, spread):
    rng = np.random.default_rng(seed)
    pts = np.zeros((n, 4), np.float32)
    pts[:, :3] = rng.normal(scale=spread, size=(n, 3)) + rng.uniform(-100, 100, size=3)
    pts[:, 3] = rng.uniform(0, 64, size=n)
    got = O.voxel_grid(pts, leaf, stable=True)
    want = voxel_grid_numpy(pts, leaf)
    if (seed, n, leaf, spread) == (0, 365, 0.2, 40.0):
        assert want.tobytes() == pts.tobytes()   # the pinned example does take the overflow branch
    assert got.shape == want.shape and len(got) <= n
    assert got.view(np.uint32).tobytes() == want.view(np.uint32).tobytes()


def _rot(rx, ry, rz):
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    return (np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]]) @
            np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]]))


@FAST
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(4, 300), angle=st.floats(0.0, 3.0))
def test_umeyama_recovers_any_rigid_motion(seed, n, angle):
    rng = np.random.default_rng(seed)
    src = np.zeros((n, 4), np.float32)
    src[:, :3] = rng.uniform(-20, 20, size=(n, 3))
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    R = np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * K @ K   # Rodrigues
    t = rng.uniform(-10, 10, size=3)
    dst = src.copy()
    dst[:, :3] = (src[:, :3].astype(np.float64) @ R.T + t).astype(np.float32)
    T = O.umeyama(src, dst)
    assert T is not None
    assert abs(np.linalg.det(T[:3, :3].astype(np.float64)) - 1.0) < 1e-5   # a rotation, never a reflection
    np.testing.assert_allclose(T[:3, :3], R, atol=1e-4)
    np.testing.assert_allclose(T[:3, 3], t, atol=1e-3)


@FAST
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(10, 300))
def test_icp_of_a_cloud_onto_itself_is_the_identity(seed, n):
    rng = np.random.default_rng(seed)
    pts = np.zeros((n, 4), np.float32)
    pts[:, :3] = rng.uniform(-30, 30, size=(n, 3))
    r = O.icp_align(CFG, pts, pts)
    assert r["converged"] == 1 and r["accepted"] == 1 and r["iters"] == 1
    np.testing.assert_allclose(r["T"].reshape(4, 4), np.eye(4), atol=1e-5)
    assert r["fitness"] < 1e-8


@pytest.mark.parametrize("leaf", [0.3, 0.5])
def test_voxel_grid_single_point_voxels_are_fixed_points(leaf):
    # a cloud with one point per voxel comes back unchanged (centroid of one point = itself)
    g = np.stack(np.meshgrid(np.arange(5), np.arange(4), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    pts = np.zeros((len(g), 4), np.float32)
    pts[:, :3] = (g * 3 + 1).astype(np.float32) * np.float32(leaf) + np.float32(leaf * 0.5)
    pts[:, 3] = np.arange(len(g), dtype=np.float32)
    out = O.voxel_grid(pts, leaf, stable=True)
    assert len(out) == len(pts)
    assert sorted(map(tuple, out.tolist())) == sorted(map(tuple, pts.tolist()))


def _cam_rot(t):
    """rotation of a camera-frame pose (rx, ry, rz) as the mapping node builds
    it: Rot3::RzRyRx(rz, rx, ry) in the GTSAM axes (MO:1545)"""
    return _rot(float(t[2]), float(t[0]), float(t[1]))


@FAST
@given(rx=st.floats(-1.5, 1.5), ry=st.floats(-12.0, 12.0), rz=st.floats(-3.1, 3.1),
       which=st.sampled_from(["odom", "keyframe"]))
def test_pose_round_trips_wrap_but_keep_the_rotation(rx, ry, rz, which):
    # the tf hand-off (FA:1728 -> MO:658) and the Rot3 read-back
    # of a keyframe (MO:1588-1601) keep the float angles inside (-pi, pi]
    # (to the last bit, except that a zero or tiny angle picks up the
    # ~1e-16..1e-15 rad residue of the f64 trig — larger near rx = +-pi/2 —
    # as in the reference), and
    # elsewhere wrap them to an equal rotation
    t = np.array([rx, ry, rz, 1.5, -2.0, 7.25], np.float32)
    out = O.pose_roundtrip(t, which)
    assert out[3:].tobytes() == t[3:].tobytes()
    assert -np.pi <= out[1] <= np.pi and -np.pi / 2 <= out[0] <= np.pi / 2
    np.testing.assert_allclose(_cam_rot(out), _cam_rot(t), atol=2e-6)
    if abs(float(t[1])) < 3.14159:
        np.testing.assert_allclose(out, t, rtol=2.0 ** -23, atol=1e-14)
    else:
        k = np.round((float(t[1]) - float(out[1])) / (2 * np.pi))
        assert k != 0 and abs(float(out[1]) - (float(t[1]) - 2 * np.pi * k)) < 1e-5
