"""slo_ddsum.h against exact arithmetic.

Every normal-equation sum in both builds (FA:1324-1326, 1425-1427;
MO:1445-1447; the ICP sums of MO:1006-1016) goes through slo_ddsum.h: exact
float products accumulated in double-double and rounded once to float.  The
GPU reduces in a tree, the oracle sequentially, and the two agree only
because the result is the correctly rounded float of the exact sum.  A bug
there would cancel out of every GPU-vs-oracle parity check, so it is pinned
here against Python's exact rationals (fractions.Fraction), in all three
summation orders, on random data and on cancellation cases built to land on
or next to float rounding boundaries."""
import ctypes
from fractions import Fraction

import numpy as np
import pytest

import oracle_py as O


def exact_float32(q):
    """float32 nearest to the rational q, ties to even significand"""
    f = np.float32(float(q))          # within one float ulp of q
    best = None
    for c in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
        if not np.isfinite(c):
            continue
        err = abs(Fraction(float(c)) - q)
        key = (err, int(np.array(c, np.float32).view(np.uint32)) & 1)
        if best is None or key < best[0]:
            best = (key, c)
    return np.float32(best[1])


def dd(a, b, mode):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return np.float32(O.lib().oracle_ddsum(a.ctypes.data, b.ctypes.data, len(a), mode))


def exact(a, b):
    return sum((Fraction(float(x)) * Fraction(float(y)) for x, y in zip(a, b)), Fraction(0))


def check(a, b):
    want = exact_float32(exact(a, b))
    for mode in (0, 1, 2):
        got = dd(a, b, mode)
        assert got.view(np.uint32) == want.view(np.uint32), (mode, got, want)


@pytest.mark.parametrize("seed", range(40))
def test_random_normal_equation_sums_are_correctly_rounded(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 3000))
    scale = 10.0 ** rng.uniform(-6, 4, size=n)      # mixed magnitudes, as Jacobian rows have
    a = (rng.normal(size=n) * scale).astype(np.float32)
    b = (rng.normal(size=n) * 10.0 ** rng.uniform(-3, 3)).astype(np.float32)
    check(a, b)


@pytest.mark.parametrize("seed", range(40))
def test_cancellation_leaves_a_tiny_exact_residue(seed):
    # large terms that cancel to the last bit, plus a residue far below the
    # rounding error of a plain double sum of the large terms
    rng = np.random.default_rng(1000 + seed)
    big = (rng.normal(size=200) * 1e6).astype(np.float32)
    tiny = (rng.normal(size=7) * 1e-9).astype(np.float32)
    a = np.concatenate([big, -big, tiny])
    b = np.concatenate([big, big, np.ones(7, np.float32)])
    perm = rng.permutation(len(a))
    a, b = a[perm], b[perm]
    check(a, b)
    assert dd(a, b, 0) == exact_float32(Fraction(0) + sum(Fraction(float(t)) for t in tiny))


@pytest.mark.parametrize("seed", range(20))
def test_sums_on_and_next_to_float_midpoints(seed):
    # x + (half an ulp of x) is a tie: it must round to the even neighbour;
    # nudged by 2^-60 relative either way it must round away from the tie
    rng = np.random.default_rng(2000 + seed)
    x = np.float32(rng.uniform(1, 2) * 2.0 ** int(rng.integers(-20, 20)))
    ulp = np.float64(np.nextafter(x, np.float32(np.inf))) - np.float64(x)
    half = ulp / 2                           # a power of two: exact as a float product 1 * half
    nudge = float(x) * 2.0 ** -60
    for extra in (0.0, nudge, -nudge):
        parts = [x, np.float32(half)] + ([np.float32(extra)] if extra else [])
        a = np.array(parts, np.float32)
        b = np.ones(len(a), np.float32)
        check(a, b)
    tie = dd(np.array([x, half], np.float32), np.ones(2, np.float32), 0)
    assert int(tie.view(np.uint32)) & 1 == 0


def test_empty_and_single_term():
    assert dd(np.zeros(0, np.float32), np.zeros(0, np.float32), 0) == 0.0
    for mode in (0, 1, 2):
        assert dd(np.array([3.0], np.float32), np.array([np.float32(1.1)], np.float32), mode) == \
            exact_float32(Fraction(3) * Fraction(float(np.float32(1.1))))
