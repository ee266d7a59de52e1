"""The VoxelGrid in PCL's own order (cfg.voxel_order = SLO_VOXEL_PCL, the
default; csrc/slo_vgpcl.hip + csrc/slo_pclsort.h) against the oracle's
reference-faithful restatement — PCL's applyFilter with the host libstdc++
std::sort (oracle_common.h voxel_grid, stable=False; FA:779-780,
MO:1224-1262) — bit for bit, through slo_batch_voxel_grid.

The clouds cover the sort's regimes: a 570 k-point map-like cloud (global
introsort levels, then the LDS finish), a raw scan with NaNs (compaction),
McIlroy's killer sequences (introsort's depth limit and heapsort, in the LDS
finish and past the global levels), one voxel holding 20 000 points, tiny,
single-point and empty clouds.  Points inside a voxel are jittered, so a
wrong in-voxel order changes the centroid's float sums."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O
import slo_amd
from parity_util import mismatch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _torch():
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    return torch


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    exe = tmp_path_factory.mktemp("pclsort") / "pcl_sort_model"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "cpp", "pcl_sort_model.cpp")],
                   check=True)
    return exe


def killer_keys(model, n, tmp, div=1):
    out = tmp / f"killer{n}_{div}.u32"
    r = subprocess.run([str(model), "--killer", str(n), str(out)] + ([str(div)] if div > 1 else []),
                       capture_output=True, text=True)
    assert r.returncode == 0 and "heapsorts=1" in r.stdout and "OK" in r.stdout, r.stdout
    return np.fromfile(out, np.uint32)


def cloud_from_keys(keys, rng):
    """points whose voxel index at leaf 1 is the key (x voxel = key, y = z = 0),
    jittered inside the voxel, random intensities"""
    n = len(keys)
    p = np.empty((n, 4), np.float32)
    p[:, 0] = keys.astype(np.float32) + rng.uniform(0.05, 0.95, n).astype(np.float32)
    p[:, 1] = rng.uniform(0.05, 0.95, n).astype(np.float32)
    p[:, 2] = rng.uniform(0.05, 0.95, n).astype(np.float32)
    p[:, 3] = rng.uniform(0, 1, n).astype(np.float32)
    return p


def run_batch(clouds, leaf, voxel_order=0):
    torch = _torch()
    cfg = slo_amd.preset(0)
    cfg.voxel_order = voxel_order
    S = len(clouds)
    stride = max(1, max(len(c) for c in clouds))
    host = np.zeros((S, stride, 4), np.float32)
    for s, c in enumerate(clouds):
        host[s, :len(c)] = c
    ctx = slo_amd.Context(cfg, 0, S)
    try:
        d_in = torch.from_numpy(host).cuda()
        d_n = torch.tensor([len(c) for c in clouds], dtype=torch.int32, device="cuda")
        d_out = torch.zeros((S, stride, 4), dtype=torch.float32, device="cuda")
        d_nout = torch.zeros(S, dtype=torch.int32, device="cuda")
        ctx.batch_voxel_grid(d_in.data_ptr(), stride, d_n.data_ptr(), leaf, d_out.data_ptr(), stride,
                             d_nout.data_ptr(), stride)
        ctx.synchronize()
        nout = d_nout.cpu().numpy()
        out = d_out.cpu().numpy()
        stats = ctx.get(0, "vg_stats")
        return [out[s, :nout[s]] for s in range(S)], stats
    finally:
        ctx.close()


def test_pcl_order_map_and_raw_clouds():
    rng = np.random.default_rng(11)
    parts = []
    for k in range(5):
        p = O.gen_scan(6, 3, 0, 4 * k)
        p = p[np.isfinite(p[:, :3]).all(1)].copy()
        p[:, 0] += np.float32(2.0 * k)
        parts.append(p)
    big = np.concatenate(parts)                       # ~570 k points, 0.3 m voxels
    raw = O.gen_scan(6, 3, 1, 7)                      # with NaNs (dropouts)
    small = big[rng.choice(len(big), 3000, replace=False)]
    clouds = [big, raw, small, big[:1], big[:0], raw[:20000]]
    for leaf in (0.3, 0.5):
        got, stats = run_batch(clouds, leaf)
        for s, c in enumerate(clouds):
            want = O.voxel_grid(c[np.isfinite(c[:, :3]).all(1)], leaf, stable=False)
            assert len(got[s]) == len(want) and mismatch(got[s], want) == 0, (leaf, s)
        assert stats[0] == 0   # no range needed the one-lane fallback
        assert stats[2] == 0 and stats[3] == 0 and stats[4] == 0   # no inconsistent wave-sort / tail step
    # the test has teeth: the stable order gives different centroids on the big cloud
    stable = O.voxel_grid(big, 0.3, stable=True)
    assert mismatch(stable, O.voxel_grid(big, 0.3, stable=False)) != 0


def test_pcl_order_many_map_streams():
    """twelve map-like streams at once (the bench's batched regime, more than
    PC_FEW streams: global levels down to 64 Ki-item ranges, the workgroup
    tail, four waves per finish entry), each shifted and thinned differently,
    against the oracle one by one; test_pcl_order_map_and_raw_clouds (six
    streams) covers the few-streams shape (16 Ki tail ranges, 16 / 8 waves)"""
    rng = np.random.default_rng(13)
    parts = []
    for k in range(5):
        p = O.gen_scan(6, 3, 0, 4 * k)
        p = p[np.isfinite(p[:, :3]).all(1)].copy()
        p[:, 0] += np.float32(2.0 * k)
        parts.append(p)
    big = np.concatenate(parts)
    clouds = []
    for s in range(12):
        c = big[rng.random(len(big)) < 0.4 + 0.05 * s].copy()
        c[:, 1] += np.float32(0.37 * s)
        clouds.append(c)
    got, stats = run_batch(clouds, 0.3)
    for s, c in enumerate(clouds):
        want = O.voxel_grid(c, 0.3, stable=False)
        assert len(got[s]) == len(want) and mismatch(got[s], want) == 0, s
    assert stats[0] == 0 and stats[2] == 0 and stats[3] == 0 and stats[4] == 0


def _map_like_clouds(n_distinct, seed):
    """map-like clouds (five hdl64 scans side by side, ~570 k points), each
    thinned, shifted and cut differently"""
    rng = np.random.default_rng(seed)
    parts = []
    for k in range(5):
        p = O.gen_scan(6, 3, 0, 4 * k)
        p = p[np.isfinite(p[:, :3]).all(1)].copy()
        p[:, 0] += np.float32(2.0 * k)
        parts.append(p)
    big = np.concatenate(parts)
    out = []
    for d in range(n_distinct):
        c = big[rng.random(len(big)) < 0.25 + 0.7 * d / max(1, n_distinct - 1)].copy()
        c[:, 1] += np.float32(0.37 * d)
        c[:, 2] -= np.float32(0.11 * d)
        out.append(c[: len(c) - int(rng.integers(0, 5000))])
    return out


def test_pcl_order_bench_shape_171_streams():
    """The bench's per-context shape (bench.py: 512 streams in 3 contexts ->
    171 streams; the local-map surf VoxelGrid's input stride at C3 with
    keyframe_cloud_cap 32768, MO:1224-1230) — the shape at which round 3's
    vg_bench runs faulted before the tail kernel's barrier fix — at leaf 0.3:
    every stream bit for bit against the oracle's std::sort VoxelGrid, every
    guard counter 0 and no stream's error word set."""
    torch = _torch()
    cfg = slo_amd.preset(6)
    S = 171
    stride = 50 * (32768 + cfg.n_scan * ((cfg.horizon_scan + 4) // 5))   # v.cap_ms (slo_ctx.hip)
    distinct = _map_like_clouds(19, 21)
    clouds = [distinct[s % len(distinct)] for s in range(S)]
    cap = max(len(c) for c in clouds)
    ctx = slo_amd.Context(cfg, 0, S)
    try:
        d_in = torch.empty((S, stride, 4), dtype=torch.float32, device="cuda")
        for s, c in enumerate(clouds):
            d_in[s, :len(c)] = torch.from_numpy(c).cuda()
        d_n = torch.tensor([len(c) for c in clouds], dtype=torch.int32, device="cuda")
        d_out = torch.zeros((S, cap, 4), dtype=torch.float32, device="cuda")
        d_nout = torch.zeros(S, dtype=torch.int32, device="cuda")
        for rep in range(2):   # twice: the second call reuses every workspace and list counter
            ctx.batch_voxel_grid(d_in.data_ptr(), stride, d_n.data_ptr(), 0.3, d_out.data_ptr(), cap,
                                 d_nout.data_ptr(), cap)
            ctx.synchronize()
            nout, out = d_nout.cpu().numpy(), d_out.cpu().numpy()
            want = [O.voxel_grid(c, 0.3, stable=False) for c in distinct]
            for s in range(S):
                w = want[s % len(distinct)]
                assert nout[s] == len(w) and mismatch(out[s, :nout[s]], w) == 0, (rep, s)
        stats = ctx.get(0, "vg_stats")
        assert stats[0] == 0 and stats[2] == 0 and stats[3] == 0 and stats[4] == 0, stats.tolist()
        assert all(int(ctx.get(s, "err")[0]) == 0 for s in range(S))
        work = ctx.get(0, "pcl_work")
        print(f"171 streams x {stride} stride: {int(work[5])} points, {int(work[6])} finish entries, "
              f"tail items {int(work[7])}, vg_stats {stats.tolist()}")
    finally:
        ctx.close()


def test_voxel_grid_argument_checks():
    """out_cap beyond out_stride would let a stream write into the next one's
    row: refused (SLO_E_ARG) before any launch; so are a zero stride and a
    non-positive leaf"""
    torch = _torch()
    cfg = slo_amd.preset(0)
    ctx = slo_amd.Context(cfg, 0, 2)
    try:
        d_in = torch.zeros((2, 100, 4), dtype=torch.float32, device="cuda")
        d_n = torch.full((2,), 100, dtype=torch.int32, device="cuda")
        d_out = torch.zeros((2, 50, 4), dtype=torch.float32, device="cuda")
        d_nout = torch.zeros(2, dtype=torch.int32, device="cuda")
        for args in ((100, 0.3, 50, 51), (0, 0.3, 50, 50), (100, 0.0, 50, 50)):
            st, leaf, ost, cap = args
            with pytest.raises(slo_amd.SloError):
                ctx.batch_voxel_grid(d_in.data_ptr(), st, d_n.data_ptr(), leaf, d_out.data_ptr(), ost,
                                     d_nout.data_ptr(), cap)
        ctx.batch_voxel_grid(d_in.data_ptr(), 100, d_n.data_ptr(), 0.3, d_out.data_ptr(), 50, d_nout.data_ptr(), 50)
        ctx.synchronize()
        assert d_nout.cpu().tolist() == [1, 1]   # 100 points at the origin: one voxel each
    finally:
        ctx.close()


@pytest.mark.parametrize("copies", [1, 2])
def test_pcl_order_killer_sequences_and_one_voxel(model, tmp_path, copies):
    """median-of-three killers (std::sort's heapsort fallback, taken by the
    wave: slo_pclsort.h wave_heap_sort), one voxel, few voxels, organ pipes;
    copies=2 runs ten streams (the batched finish shape: four waves per entry)
    instead of five (the few-stream shape: sixteen)"""
    rng = np.random.default_rng(12)
    k5 = killer_keys(model, 5000, tmp_path)           # heapsort inside the LDS finish
    k100 = killer_keys(model, 100000, tmp_path)       # depth limit past the global levels
    one = np.zeros(20000, np.uint32)                  # every point in one voxel
    few = rng.integers(0, 50, 3000).astype(np.uint32)
    runs = np.concatenate([np.arange(4000, dtype=np.uint32) // 7, (np.arange(4000, dtype=np.uint32) // 5)[::-1]])
    small = [killer_keys(model, n, tmp_path) for n in (70, 129, 300, 1000, 2047, 4096)]   # one heapsort each
    clouds = [cloud_from_keys(k, rng) for k in (k5, k100, one, few, runs)] * copies
    clouds += [cloud_from_keys(k, rng) for k in small]
    got, stats = run_batch(clouds, 1.0)
    for s, c in enumerate(clouds):
        want = O.voxel_grid(c, 1.0, stable=False)
        assert len(got[s]) == len(want) and mismatch(got[s], want) == 0, s
    print("finish ranges over the LDS capacity:", int(stats[0]))


def test_stable_order_switch():
    """cfg.voxel_order = SLO_VOXEL_STABLE keeps the radix sort: input order in a voxel"""
    big = O.gen_scan(6, 3, 0, 3)
    big = big[np.isfinite(big[:, :3]).all(1)]
    got, _ = run_batch([big], 0.3, voxel_order=1)
    assert mismatch(got[0], O.voxel_grid(big, 0.3, stable=True)) == 0


def test_spent_depth_heapsort_paths(model, tmp_path):
    """pc_fallback_entry (slo_vgpcl.hip, inside k_pc_finish32<4 Ki>): spent-depth ranges over 4 Ki items,
    heapsorted by one wave in global memory — a 12 000-item killer, a
    7 000-item killer with its keys spread x97 (a key span over 2^18) and the
    100 000-item killer, several ranges in one call (each workgroup's scratch
    slots must stay its own range's) — each bit for bit against std::sort's
    order.  Every killer key is halved, so the heaps hold pairs of equal keys
    (two points of one voxel) whose order the heapsort decides."""
    rng = np.random.default_rng(14)
    k12 = killer_keys(model, 12000, tmp_path, 2)
    k7 = killer_keys(model, 7000, tmp_path, 2) * np.uint32(97)
    k100 = killer_keys(model, 100000, tmp_path, 2)
    assert int(k7.max() - k7.min()) >= (1 << 18) and int(k12.max() - k12.min()) < (1 << 18)
    clouds = [cloud_from_keys(k, rng) for k in (k12, k7, k100)]
    got, stats = run_batch(clouds, 1.0)
    for s, c in enumerate(clouds):
        want = O.voxel_grid(c, 1.0, stable=False)
        assert len(got[s]) == len(want) and mismatch(got[s], want) == 0, s
    assert stats[0] >= 3, stats.tolist()   # each stream sent its spent range to the fallback
    assert stats[2] == 0 and stats[3] == 0 and stats[4] == 0, stats.tolist()
