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


# ---- the oracle's second accumulation mode: OpenCV 3.x's own GEMM order (Q11)
def _opencv_order(A, B):
    """GEMMSingleMul<float, double> as oracle_common.h restates it, in Python
    doubles: matAtA one accumulator per entry in k order; matAtB four
    accumulators over k mod 4, the tail into the first, summed left to right"""
    A = np.asarray(A, np.float32).astype(np.float64)
    B = np.asarray(B, np.float32).astype(np.float64)
    n, m = A.shape
    ata = np.zeros((m, m), np.float32)
    atb = np.zeros(m, np.float32)
    for i in range(m):
        for j in range(m):
            s = 0.0
            for k in range(n):
                s += float(A[k, i]) * float(A[k, j])
            ata[i, j] = np.float32(s)
        s = [0.0, 0.0, 0.0, 0.0]
        k = 0
        while k <= n - 4:
            for u in range(4):
                s[u] += float(A[k + u, i]) * float(B[k + u])
            k += 4
        while k < n:
            s[0] += float(A[k, i]) * float(B[k])
            k += 1
        atb[i] = np.float32(((s[0] + s[1]) + s[2]) + s[3])
    return ata, atb


def test_gemm_modes_restated():
    """mode 1 equals the Python restatement of OpenCV's order bit for bit on
    random mixed-magnitude data; mode 0 is the correctly rounded float of the
    exact sums (Fraction)"""
    rng = np.random.default_rng(3)
    for n, m in ((1, 3), (7, 3), (64, 6), (203, 6)):
        A = (rng.standard_normal((n, m)) * np.exp2(rng.integers(-20, 20, (n, m)))).astype(np.float32)
        B = (rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n))).astype(np.float32)
        ata1, atb1 = O.gemm_at(A, B, 1)
        want = _opencv_order(A, B)
        assert np.array_equal(ata1.view(np.uint32), want[0].view(np.uint32)), (n, m)
        assert np.array_equal(atb1.view(np.uint32), want[1].view(np.uint32)), (n, m)
        ata0, atb0 = O.gemm_at(A, B, 0)
        for i in range(m):
            q = sum(Fraction(float(A[k, i])) * Fraction(float(B[k])) for k in range(n))
            assert atb0[i] == exact_float32(q)


def test_gemm_modes_differ_where_expected():
    """products 1, 2^-24, 2^-60: a sequential double sum stops at 1 + 2^-24,
    the float midpoint, which rounds to even (1.0); the exact sum lies above
    it (1 + 2^-23).  The two modes differ only in such ~2^-29-wide windows
    around float rounding boundaries, and tools/faithful_drift.py --gemm
    measures that no C1-C5 stream reaches one."""
    A = np.array([[1.0], [2.0 ** -12], [2.0 ** -30]], np.float32)
    ata0, atb0 = O.gemm_at(A, A[:, 0], 0)
    ata1, atb1 = O.gemm_at(A, A[:, 0], 1)
    assert ata1[0, 0] == np.float32(1.0) and atb1[0] == np.float32(1.0)
    assert ata0[0, 0] == np.float32(1.0 + 2.0 ** -23) and atb0[0] == np.float32(1.0 + 2.0 ** -23)
