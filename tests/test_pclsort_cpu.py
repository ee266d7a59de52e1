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

