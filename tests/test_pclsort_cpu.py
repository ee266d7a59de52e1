"""The data-parallel formulation of libstdc++'s std::sort that the GPU
VoxelGrid uses for PCL's in-voxel order (csrc/slo_pclsort.h,
csrc/slo_vgpcl.hip), checked against the host std::sort by
tests/cpp/pcl_sort_model.cpp: random keys with many ties, sorted / reversed
runs, all-equal keys, and McIlroy's killer sequences (introsort's depth limit
and heapsort); plus the lane restatement of a sub-range
(slo_sort::introsort_range) it finishes small ranges with."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    exe = tmp_path_factory.mktemp("pclsort") / "pcl_sort_model"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "cpp", "pcl_sort_model.cpp")],
                   check=True)
    return exe


@pytest.mark.parametrize("seed,n,nkeys", [(1, 100000, 5000), (2, 1000, 3), (3, 50000, 50), (4, 17, 2), (5, 9000, 9000)])
def test_formulation_matches_std_sort(model, seed, n, nkeys):
    r = subprocess.run([str(model), "--random", str(seed), str(n), str(nkeys)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count("OK") == 5


@pytest.mark.parametrize("n", [100, 5000, 60000])
def test_killer_sequences_reach_heapsort(model, tmp_path, n):
    r = subprocess.run([str(model), "--killer", str(n), str(tmp_path / "k.u32")], capture_output=True, text=True)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout
    assert "heapsorts=0" not in r.stdout


def test_wave_tier_emulation_matches_std_sort(model, tmp_path):
    """The wave tier's lane-level steps (ballots, prefix / select, m by
    binary search, cuts, swap partners, child tables, leaf ranks), emulated in
    Python (tests/pclsort_emul.py), give std::sort's order — random ties,
    runs, all-equal keys, and a killer sequence (depth limit, heapsort)."""
    import random
    import sys
    import numpy as np
    sys.path.insert(0, HERE)
    import pclsort_emul as P
    rng = random.Random(5)
    cases = []
    for n in (2, 16, 17, 40, 64, 65, 200, 511, 512):
        for nk in (1, 3, 50, 1000):
            cases.append([(rng.randrange(nk), i) for i in range(n)])
    cases.append([(i // 3, i) for i in range(300)])
    cases.append([(300 - i, i) for i in range(300)])
    subprocess.run([str(model), "--killer", "500", str(tmp_path / "k.u32")], check=True, capture_output=True)
    cases.append([(int(k), i) for i, k in enumerate(np.fromfile(tmp_path / "k.u32", np.uint32))])
    for keys in cases:
        n = len(keys)
        want = P.std_sort(keys)
        buf = [(7, -1)] * 3 + list(keys) + [(7, -1)] * 2
        P.wave_sort(buf, 3, n, 2 * (n.bit_length() - 1))
        assert buf[3:3 + n] == want, n
