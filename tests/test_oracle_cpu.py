"""CPU tests of the oracle (test infrastructure) and of the product's host-side
restatements: the restated glibc libm and libstdc++ introsort against the
host's, the Scan Context K-NN against the
reference's own nanoflann tree (committed fixture), and the oracle against
its committed stage fingerprints (tests/golden/make_golden.py)."""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def libm_check(tmp_path_factory):
    """tests/cpp/libm_check.cpp: the product's libm restatements (slo_libm.h,
    slo_libm_d.h), compiled with the product's -ffp-contract=off rule"""
    import ctypes
    so = tmp_path_factory.mktemp("libm") / "libm_check.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(so),
                    os.path.join(HERE, "cpp", "libm_check.cpp")], check=True)
    L = ctypes.CDLL(str(so))
    L.libm_selftest.restype = ctypes.c_long
    L.libm_selftest.argtypes = [ctypes.c_long, ctypes.c_ulong]
    L.libm_d.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return L


def test_libm_restatement_matches_glibc(libm_check):
    # atan2f, sinf, cosf, atanf, asinf bit-for-bit vs the host glibc
    for seed in (1, 7, 12345):
        assert libm_check.libm_selftest(300000, seed) == 0


def _libm_d(L, which, a, b=None):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    out = np.zeros_like(a)
    L.libm_d(which, a.ctypes.data, b.ctypes.data, out.ctypes.data, len(a))
    return out


def test_double_libm_within_one_ulp_of_glibc(libm_check):
    # slo_libm_d.h (fdlibm sin/cos/atan2/asin, the
    # device for the Q18 round trips) against the host glibc via Python's math
    import math
    rng = np.random.default_rng(3)
    n = 40000
    ang = np.concatenate([rng.uniform(-20, 20, n), rng.uniform(-1e-3, 1e-3, n),
                          rng.uniform(-7, 7, n).astype(np.float32).astype(np.float64)])
    cases = [(0, ang, None, math.sin), (1, ang, None, math.cos),
             (3, np.concatenate([rng.uniform(-1, 1, n), rng.uniform(-1e-4, 1e-4, n)]), None, math.asin),
             (2, rng.normal(size=n) * 10.0 ** rng.integers(-8, 3, n), rng.normal(size=n), math.atan2)]
    for which, a, b, f in cases:
        got = _libm_d(libm_check, which, a, b)
        want = np.array([f(*v) for v in (zip(a, b) if b is not None else ((x,) for x in a))])
        ulp = np.abs(got.view(np.int64) - want.view(np.int64))
        assert ulp.max() <= 1, (which, int(ulp.max()))
        assert (ulp == 0).mean() > 0.7, which


def test_introsort_restatement_matches_libstdcxx(tmp_path):
    exe = tmp_path / "introsort_check"
    src = os.path.join(HERE, "cpp", "introsort_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src], check=True)
    bad, cases = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert cases > 900 and bad == 0


@pytest.fixture(scope="module")
def sc_gold():
    with np.load(os.path.join(GOLD, "sc_loop_hdl64.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("K", [10, 50])
def test_sc_knn_matches_reference_nanoflann(sc_gold, K):
    """Exact K-NN of the restatement == the reference's nanoflann tree
    (oracle/_ref/nanoflann_pin built from /root/reference's headers)."""
    cfg = O.preset(int(sc_gold["preset"]))
    keys = sc_gold["ring_keys"]
    nf_i, nf_d = sc_gold[f"nf_idx{K}"], sc_gold[f"nf_dist{K}"]
    checked = 0
    for q, (j, snap) in enumerate(zip(sc_gold["query_frame"], sc_gold["snapshot"])):
        idx, dist = O.sc_knn(cfg, keys[:snap], keys[j], K)
        m = min(K, int(snap))
        assert np.array_equal(dist[:m].view(np.uint32), nf_d[q][:m].view(np.uint32)), q
        # same neighbours; order only free inside equal-distance groups
        for d in np.unique(dist[:m]):
            assert set(idx[:m][dist[:m] == d]) == set(nf_i[q][:m][nf_d[q][:m] == d])
        # unfilled slots keep the zero-initialised index (Scancontext.cpp:282)
        assert (nf_i[q][m:] == 0).all() and (idx[m:] == 0).all()
        checked += 1
    assert checked == len(sc_gold["query_frame"]) > 100


def test_sc_session_reproduces_fixture_prefix(sc_gold):
    """First 60 keyframes: ring keys and detect results are bit-identical."""
    pid, cid, sid, step = (int(sc_gold[k]) for k in ("preset", "config", "stream", "step"))
    cfg = O.preset(pid)
    ses = O.SCSession(cfg, stable_voxel=False)
    for j in range(60):
        n, key = ses.add(O.gen_scan(pid, cid, sid, j * step))
        assert n == sc_gold["n_ds"][j]
        assert np.array_equal(key.view(np.uint32), sc_gold["ring_keys"][j].view(np.uint32))
        d = ses.detect()
        assert d["loop_id"] == sc_gold["loop_id"][j] and d["nn_idx"] == sc_gold["nn_idx"][j]
        assert np.float64(d["min_dist"]).view(np.uint64) == sc_gold["min_dist"][j].view(np.uint64)


def test_sc_fixture_has_true_and_early_loops(sc_gold):
    lid = sc_gold["loop_id"]
    assert (lid[:50] == -1).all()                 # < 51 contexts: early return (SCc:257-261)
    assert sc_gold["snapshot"][0] == 1            # first tree: 51 - NUM_EXCLUDE_RECENT rows
    assert (lid[205:] >= 0).sum() > 20            # the second lap closes loops


@pytest.mark.parametrize("name", ["vlp16", "hdl64"])
def test_oracle_front_fingerprints(name):
    with open(os.path.join(GOLD, f"front_{name}.json")) as f:
        gold = json.load(f)
    import fingerprint as F
    rows = F.oracle_rows(O, gold["preset"], gold["config"], len(gold["scans"]))
    for got, want in zip(rows, gold["scans"]):
        assert got == want, (name, want["scan"])


def test_voxel_grid_stable_and_sorted_orders_agree_as_sets():
    """The GPU VoxelGrid keeps input order inside a voxel ("stable"); PCL's
    std::sort does not.  Same voxels, same counts, centroids within rounding."""
    pts = O.gen_scan(6, 3, 0, 5)
    pts = pts[np.isfinite(pts[:, :3]).all(1)]
    outs = []
    for stable in (0, 1):
        out = np.empty_like(pts)
        n = O.lib().oracle_voxel_grid(pts.ctypes.data, len(pts), 0.5, stable, out.ctypes.data, len(out))
        outs.append(out[:n])
    a, b = outs
    assert len(a) == len(b) > 1000
    np.testing.assert_allclose(a, b, rtol=0, atol=2e-5)


def test_gpu_sincos_matches_sinf_cosf(tmp_path):
    # the fused sin/cos of the GPU pose transforms == its sinf/cosf == glibc
    exe = tmp_path / "sincos_check"
    src = os.path.join(HERE, "cpp", "sincos_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-o", str(exe), src], check=True)
    bad, cases = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert cases > 700000 and bad == 0


def test_atan2_bracket_contains_glibc_atan2f(tmp_path):
    # the image projection's fast path (slo_fastatan.h) decides bins at both
    # ends of a polynomial bracket; it must contain glibc's atan2f everywhere
    exe = tmp_path / "atan_bracket_check"
    src = os.path.join(HERE, "cpp", "atan_bracket_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src], check=True)
    bad, cases, worst = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert int(cases) > 40_000_000 and int(bad) == 0
    assert float(worst) < 1e-6   # 2.5e-6 half-width: > 2x margin


def test_radius_branch_keeps_the_keyframes_near_the_robot():
    """loopClosureEnableFlag = false (MO:1167-1222): the local map's keyframes
    are the key poses within 50 m of the last mapped position, downsampled at
    1 m; the list is updated in place, so it holds no duplicates, and
    keyframes that fell out of range leave it."""
    cfg = O.preset(0)
    cfg.loop_closure_enable = 0
    o = O.OracleStream(cfg, stable_voxel=False)
    last = None
    dropped = False
    for k in range(120):
        fl = o.step(O.gen_scan(0, 1, 0, k), 0.1 * k)
        if fl & 2:
            ids = o.get("map_ids")
            kp = o.get("keyposes").reshape(-1, 6)
            assert len(set(ids.tolist())) == len(ids)
            if last is not None and len(ids):
                # every listed keyframe was within radius + a voxel diagonal of the robot
                d = np.linalg.norm(kp[ids, :3] - last, axis=1)
                assert (d < 50.0 + np.sqrt(3.0)).all()
                dropped |= ids.min() > 0
            last = o.get("mapped")[3:6].astype(np.float64)
            assert not (fl & 8)                          # no loop detection without loop closure
    assert dropped
