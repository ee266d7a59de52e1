"""The public SCManager helpers (Scancontext.h:63-69) at the C ABI
(slo_sc_make_scancontext, slo_sc_ring_key, slo_sc_sector_key,
slo_sc_fast_align, slo_sc_dist_direct, slo_sc_distance, batched
slo_batch_sc_distance) and their Python mirrors (slo_amd.SCManager), bit for
bit against the oracle's restatement of Scancontext.cpp:39-227 on the
descriptors of the committed loop stream's keyframes (hdl64_1800, the scans
tests/golden/sc_loop_hdl64.npz is built from)."""
import os

import numpy as np
import pytest

import oracle_py as O
import slo_amd

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def scans():
    with np.load(os.path.join(GOLD, "sc_loop_hdl64.npz"), allow_pickle=False) as z:
        pid, cid, sid, step = (int(z[k]) for k in ("preset", "config", "stream", "step"))
    cfg = O.preset(pid)
    out = []
    for j in (0, 1, 2, 40, 200, 201, 239):   # neighbours, and keyframes a lap apart (a loop)
        p = O.gen_scan(pid, cid, sid, j * step)
        p = p[np.isfinite(p[:, :3]).all(1)]
        out.append(O.voxel_grid(p, cfg.leaf_sc))
    return pid, out


def bits(x):
    return np.ascontiguousarray(x, np.float64).view(np.uint64)


def test_sc_helpers_match_oracle(scans):
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    pid, clouds = scans
    ocfg = O.preset(pid)
    ctx = slo_amd.Context(slo_amd.preset(pid), 0, 1)
    try:
        sc = slo_amd.SCManager(ctx)
        descs = []
        for c in clouds:
            d = sc.makeScancontext(c)
            od, orr, osk = O.sc_make(ocfg, c)
            assert np.array_equal(bits(d), bits(od))
            assert np.array_equal(bits(sc.makeRingkeyFromScancontext(d)), bits(orr))
            assert np.array_equal(bits(sc.makeSectorkeyFromScancontext(d)), bits(osk))
            descs.append(d)
        empty = np.zeros_like(descs[0])
        pairs = [(a, b) for a in range(len(descs)) for b in range(len(descs))]
        for a, b in pairs:
            A, B = descs[a], descs[b]
            va, vb = sc.makeSectorkeyFromScancontext(A), sc.makeSectorkeyFromScancontext(B)
            assert sc.fastAlignUsingVkey(va, vb) == O.sc_fast_align(ocfg, va, vb)
            assert bits(sc.distDirectSC(A, B)) == bits(O.sc_dist_direct(ocfg, A, B))
            d, sh = sc.distanceBtnScanContext(A, B)
            od, osh = O.sc_distance(ocfg, A, B)
            assert bits(d) == bits(od) and sh == osh, (a, b)
        # a descriptor with empty sectors only: every column skipped, 1 - 0/0 (NaN), as Eigen gives
        assert np.isnan(sc.distDirectSC(empty, descs[0])) and np.isnan(O.sc_dist_direct(ocfg, empty, descs[0]))
        # batched on the device: every pair in one launch
        d1 = torch.from_numpy(np.stack([descs[a] for a, _ in pairs])).cuda()
        d2 = torch.from_numpy(np.stack([descs[b] for _, b in pairs])).cuda()
        dist = torch.zeros(len(pairs), dtype=torch.float64, device="cuda")
        shift = torch.zeros(len(pairs), dtype=torch.int32, device="cuda")
        ctx._ok(ctx.L.slo_batch_sc_distance(ctx.h, d1.data_ptr(), d2.data_ptr(), len(pairs), dist.data_ptr(),
                                            shift.data_ptr()), "slo_batch_sc_distance")
        ctx.synchronize()
        for i, (a, b) in enumerate(pairs):
            od, osh = O.sc_distance(ocfg, descs[a], descs[b])
            assert bits(dist[i].item()) == bits(od) and int(shift[i]) == osh
    finally:
        ctx.close()


def test_sc_distance_mfma_adversarial():
    """distanceBtnScanContext over 3000 random pairs of descriptors built to
    expose any slip in the matrix-core Gram (slo_scdist.h sc_gram_mfma): float
    cells of mixed magnitudes (2^-12 .. 2^8) and both signs (points below the
    sensor height), empty cells and empty columns, so that a wrong tile
    layout, a wrong ring order in any of Eigen's four accumulators or a
    different combine would change the doubles; batched on the device against
    the oracle's Eigen-order restatement, bit for bit, distance and shift."""
    import torch
    assert torch.cuda.is_available(), "no HIP device"
    pid = 6
    ocfg = O.preset(pid)
    NR, NS = ocfg.sc_num_ring, ocfg.sc_num_sector
    rng = np.random.default_rng(17)
    n = 3000

    def desc():
        mag = np.exp2(rng.integers(-12, 9, (NR, NS))).astype(np.float32)
        d = (rng.uniform(-0.3, 1.0, (NR, NS)).astype(np.float32) * mag).astype(np.float32)
        d[rng.random((NR, NS)) < 0.3] = 0.0                      # empty cells
        d[:, rng.random(NS) < 0.1] = 0.0                         # empty sectors
        return d.astype(np.float64)

    A = [desc() for _ in range(n)]
    B = [desc() if k % 3 else np.roll(A[k], int(rng.integers(0, NS)), axis=1) for k in range(n)]
    ctx = slo_amd.Context(slo_amd.preset(pid), 0, 1)
    try:
        d1 = torch.from_numpy(np.stack(A)).cuda()
        d2 = torch.from_numpy(np.stack(B)).cuda()
        dist = torch.zeros(n, dtype=torch.float64, device="cuda")
        shift = torch.zeros(n, dtype=torch.int32, device="cuda")
        ctx._ok(ctx.L.slo_batch_sc_distance(ctx.h, d1.data_ptr(), d2.data_ptr(), n, dist.data_ptr(),
                                            shift.data_ptr()), "slo_batch_sc_distance")
        ctx.synchronize()
        got_d, got_s = dist.cpu().numpy(), shift.cpu().numpy()
        bad = 0
        for k in range(n):
            od, osh = O.sc_distance(ocfg, A[k], B[k])
            bad += int(bits(got_d[k]) != bits(od) or int(got_s[k]) != osh)
        assert bad == 0, f"{bad} of {n} pairs differ"
    finally:
        ctx.close()
