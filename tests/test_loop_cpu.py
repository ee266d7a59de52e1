"""Loop-closure verification, CPU side: the oracle's
restatement of Eigen's JacobiSVD / pcl::umeyama / pcl::IterativeClosestPoint
(oracle/oracle_lc.h) against numpy's SVD and known rigid transforms, and the
whole detectLoopClosure + performLoopClosure path against the committed
fixture tests/golden/loop_vlp16.npz (tests/golden/make_loop_golden.py).
PCL and Eigen are absent here, so parity with them is unpinned: these
tests pin the restatement to the mathematics (tolerances stated inline) and
against regressions (bit for bit)."""
import os

import numpy as np
import pytest

import oracle_py as O

HERE = os.path.dirname(os.path.abspath(__file__))


def _rot(rx, ry, rz):
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def test_svd3_matches_numpy():
    rng = np.random.default_rng(7)
    mats = [rng.normal(size=(3, 3)) for _ in range(50)]
    mats += [np.diag([3.0, 2.0, 0.0]), np.zeros((3, 3)), np.outer([1.0, 2, 3], [4.0, 5, 6]), -np.eye(3)]
    for A in mats:
        U, S, V = O.svd3(A)
        assert np.all(np.diff(S) <= 0), S                              # descending
        np.testing.assert_allclose(S, np.linalg.svd(A)[1], atol=1e-12)  # singular values
        np.testing.assert_allclose(U @ np.diag(S) @ V.T, A, atol=1e-12)
        np.testing.assert_allclose(U.T @ U, np.eye(3), atol=1e-12)
        np.testing.assert_allclose(V.T @ V, np.eye(3), atol=1e-12)


def test_umeyama_recovers_rigid_transform():
    rng = np.random.default_rng(3)
    for trial in range(20):
        n = int(rng.integers(3, 400))
        src = np.zeros((n, 4), np.float32)
        src[:, :3] = rng.uniform(-50, 50, size=(n, 3)) + rng.uniform(-200, 200, size=3)
        R = _rot(*rng.uniform(-0.3, 0.3, size=3))
        t = rng.uniform(-5, 5, size=3)
        dst = src.copy()
        dst[:, :3] = (src[:, :3].astype(np.float64) @ R.T + t).astype(np.float32)
        T = O.umeyama(src, dst)
        # float inputs (~1e-5 relative rounding) bound the recovered transform
        np.testing.assert_allclose(T[:3, :3], R, atol=2e-5)
        np.testing.assert_allclose(T[:3, 3], t, atol=2e-3)
        np.testing.assert_array_equal(T[3], [0, 0, 0, 1])


def _scene_pair(shift=(0.4, -0.3, 0.1), yaw=0.03):
    cfg = O.preset(0)
    tgt = O.voxel_grid(O.gen_scan(0, 1, 0, 20), 0.3, stable=True)
    src = O.voxel_grid(O.gen_scan(0, 1, 0, 20), 0.5, stable=True)
    R = _rot(0.0, 0.0, yaw)
    moved = src.copy()
    moved[:, :3] = (src[:, :3].astype(np.float64) @ R.T + np.array(shift)).astype(np.float32)
    return cfg, moved, tgt, R


def test_icp_recovers_known_offset():
    cfg, src, tgt, R = _scene_pair()
    r = O.icp_align(cfg, src, tgt)
    T = r["T"].reshape(4, 4).astype(np.float64)
    assert r["ran"] == 1 and r["converged"] == 1 and r["accepted"] == 1
    assert 1 <= r["iters"] <= cfg.icp_max_iterations
    # ICP undoes the offset: T * (R p + s) ~= p, to a few cm on a 0.3 m voxelised target
    np.testing.assert_allclose(T[:3, :3] @ R, np.eye(3), atol=5e-3)
    assert r["fitness"] < 0.05
    assert r["n_src"] == len(src) and r["n_tgt"] == len(tgt)
    assert np.isclose(r["xyzrpy"][5], np.arctan2(T[1, 0], T[0, 0]), atol=1e-6)


def test_icp_degenerate_inputs():
    cfg, src, tgt, _ = _scene_pair()
    e = np.zeros((0, 4), np.float32)
    for a, b in ((e, tgt), (src, e), (e, e)):
        r = O.icp_align(cfg, a, b)
        assert r["ran"] == 1 and r["converged"] == 0 and r["accepted"] == 0 and r["iters"] == 0
        assert r["fitness"] == np.finfo(np.float64).max
        np.testing.assert_array_equal(r["T"], np.eye(4, dtype=np.float32).ravel())
    far = src.copy()
    far[:, 0] += 1000.0   # every neighbour beyond icp_max_corr_dist (100 m): < 3 correspondences
    r = O.icp_align(cfg, far, tgt)
    assert r["converged"] == 0 and r["iters"] == 0 and r["fitness"] > 1e5


def _fixture():
    z = np.load(os.path.join(HERE, "golden", "loop_vlp16.npz"))
    loops = np.frombuffer(z["loop_bytes"].tobytes(), O.LOOP_DTYPE).reshape(len(z["scans"]), 2)
    return z["scans"], z["n_keyframes"], z["sc_id"], loops


def test_loop_fixture_shape():
    scans, nkf, sc, loops = _fixture()
    assert len(scans) >= 10
    assert (loops["id"][:, 1] == sc).all()
    assert (loops["ran"][:, 1] == 1).all()                       # an SC candidate always runs ICP
    assert ((loops["ran"][:, 0] == 1) == (loops["id"][:, 0] >= 0)).all()
    acc = loops["accepted"][:, 1]
    assert acc.sum() >= 5 and (1 - acc).sum() >= 3             # true loops accepted, false ones rejected
    assert (loops["fitness"][acc == 1, 1] <= 1.5).all() and (loops["fitness"][acc == 0, 1] > 1.5).all()


@pytest.mark.timeout(600)
def test_loop_fixture_oracle_regression():
    """The oracle reproduces the committed fixture bit for bit (~1 min)."""
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_loop_golden as G
    scans, nkf, sc, loops = _fixture()
    s2, n2, d2, l2 = G.run_oracle()
    np.testing.assert_array_equal(s2, scans)
    np.testing.assert_array_equal(n2, nkf)
    np.testing.assert_array_equal(d2, sc)
    assert l2.tobytes() == loops.tobytes()
