"""CPU checks of the drop-in boundary: libslo.so (built for gfx950) loads and
exports exactly the functions include/slo_abi.h declares, the struct mirrors
match the C layout, and the host-side pieces that need no GPU agree with the
oracle (presets, the synthetic stream generator)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "slo_abi.h")
LIB = os.path.join(ROOT, "sc-lego-loam_amd", "libslo.so")


def header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(slo_\w+)\s*\(", txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sc-lego-loam_amd")], check=True)
    from slo_amd import _abi
    return _abi.lib()


def test_header_declares_the_reference_entry_points():
    fns = header_functions()
    for f in ("slo_create", "slo_destroy", "slo_image_projection", "slo_feature_association",
              "slo_map_optimization", "slo_sc_make_and_save", "slo_sc_detect", "slo_batch_process"):
        assert f in fns


def test_every_declared_symbol_is_exported(lib):
    from slo_amd import _abi
    fns = header_functions()
    assert sorted(_abi.EXPORTS) == fns
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT\s+(slo_\w+)$", nm, flags=re.M))
    missing = [f for f in fns if f not in exported]
    assert not missing, missing
    for f in fns:
        assert hasattr(lib, f)


def test_library_carries_gfx950_code_objects(lib):
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob      # offload bundle entry of the fat binary
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_config_struct_mirrors_agree(lib):
    import oracle_py as O
    from slo_amd import _abi
    assert ctypes.sizeof(_abi.SloConfig) == ctypes.sizeof(O.SloConfig)
    for pid in range(8):
        a, b = _abi.SloConfig(), O.SloConfig()
        assert lib.slo_config_preset(pid, ctypes.byref(a)) == 0
        assert O.lib().oracle_config_preset(pid, ctypes.byref(b)) == 0
        assert bytes(a) == bytes(b)
    assert lib.slo_config_preset(99, ctypes.byref(_abi.SloConfig())) != 0


def test_generator_matches_oracle(lib):
    import oracle_py as O
    import slo_amd
    for pid, cid, sid, k in [(0, 1, 0, 0), (6, 3, 2, 7), (5, 2, 1, -3)]:
        cfg = slo_amd.preset(pid)
        a = slo_amd.gen_scan(pid, cid, sid, k, cfg.max_points)
        b = O.gen_scan(pid, cid, sid, k)
        assert a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
        assert np.isnan(a[:, 0]).mean() > 0.01        # dropouts kept as NaN (exercise removeNaN)
    batch = slo_amd.gen_batch(6, 3, 4, 2, 10, 2, slo_amd.preset(6).max_points, 2)
    assert np.array_equal(batch[1, 1].view(np.uint32), O.gen_scan(6, 3, 5, 11).view(np.uint32))


def test_bad_arguments_are_rejected_without_a_device(lib):
    from slo_amd import _abi
    h = ctypes.c_void_p()
    cfg = _abi.SloConfig()
    lib.slo_config_preset(6, ctypes.byref(cfg))
    assert lib.slo_create(None, 0, 1, ctypes.byref(h)) == -1
    assert lib.slo_create(ctypes.byref(cfg), 0, 0, ctypes.byref(h)) == -1
    bad = _abi.SloConfig.from_buffer_copy(bytes(cfg))
    bad.sc_num_candidates = 65
    assert lib.slo_create(ctypes.byref(bad), 0, 1, ctypes.byref(h)) == -1
    assert lib.slo_record_floats() == _abi.RECORD_FLOATS == 1240
    assert lib.slo_batch_process(None, None, None, 0.0) == -1
    assert lib.slo_get(None, 0, b"range", None, 0) == -1


def test_c_caller_compiles_and_runs_against_the_public_header(lib, tmp_path):
    """a C99 program that includes only include/slo_abi.h links against
    libslo.so and runs the host-side entry points (no GPU needed)"""
    exe = tmp_path / "abi_caller"
    libdir = os.path.dirname(LIB)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "abi_caller.c"), "-o", str(exe), f"-L{libdir}", "-lslo",
                    f"-Wl,-rpath,{libdir}", "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "abi_caller ok" in r.stdout
