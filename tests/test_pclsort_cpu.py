"""CPU model of the PCL-order sort's register tier (slo_pclsort.h
wave_small_sort): one item per lane, every segment over 16 items stepped at
once through the flag formulation (left / right stoppers, m = max over
boundaries of min(Lb, Rb), pairs swapped by rank, cut = min(i_{m+1}, j_m)),
the leaves placed by their rank by (key, lane).  The lane arithmetic (masks,
prefix counts, the partner table, the permutes) is restated here line for
line and checked against a sequential restatement of libstdc++'s introsort
(median-of-three to first, unguarded Hoare partition, threshold 16, final
insertion sort) — the algorithm tests/cpp/introsort_check.cpp pins to the
host std::sort.  Ties are the point: the keys are drawn from a few values so
that the in-voxel order of equal keys is what gets checked."""
import random

import pytest


def median3(a, b, c):
    if a < b:
        if b < c:
            return 1
        return 2 if a < c else 0
    if a < c:
        return 0
    return 2 if b < c else 1


def introsort(items, depth):
    """libstdc++ std::sort restated on (key, payload) pairs, keys compared only"""
    a = list(items)
    n = len(a)
    stack = [(0, n, depth)]
    while stack:
        lo, hi, d = stack.pop()
        while hi - lo > 16:
            if d == 0:
                raise OverflowError("heapsort")   # not modelled: the device hands these to a lane
            d -= 1
            f, l, mid = lo, hi, lo + (hi - lo) // 2
            A, B, C = f + 1, mid, l - 1
            k = lambda x: a[x][0]  # noqa: E731
            if k(A) < k(B):
                m = B if k(B) < k(C) else (C if k(A) < k(C) else A)
            else:
                m = A if k(A) < k(C) else (C if k(B) < k(C) else B)
            a[f], a[m] = a[m], a[f]
            first, last, p = f + 1, l, a[f][0]
            while True:
                while a[first][0] < p:
                    first += 1
                last -= 1
                while p < a[last][0]:
                    last -= 1
                if not first < last:
                    break
                a[first], a[last] = a[last], a[first]
                first += 1
            stack.append((first, hi, d))
            hi = first
    for i in range(1, n):   # the final insertion sort (stable)
        v, j = a[i], i
        while j > 0 and v[0] < a[j - 1][0]:
            a[j] = a[j - 1]
            j -= 1
        a[j] = v
    return a


def popc(x):
    return bin(x).count("1")


def ctz(x):
    return (x & -x).bit_length() - 1


def below(k):
    return (1 << 64) - 1 if k >= 64 else (1 << k) - 1


def ballot(flags):
    return sum(1 << i for i, f in enumerate(flags) if f)


def wave_small_sort(items, depth, segs=None):
    """slo_pclsort.h wave_small_sort, lane by lane (64 lanes, n <= 64 items);
    segs: adjacent ranges [(lo, hi, depth), ...] covering the items, sorted in
    one call (wave_sort_range merges a small range with the stack's next ones)"""
    n, L = len(items), 64
    it = [items[min(i, n - 1)] for i in range(L)]
    lo, hi, dd = [0] * L, [n] * L, [depth] * L
    for a, b, d in segs or []:
        for i in range(a, b):
            lo[i], hi[i], dd[i] = a, b, d
    live = [i < n for i in range(L)]
    while True:
        act = [live[i] and hi[i] - lo[i] > 16 and dd[i] > 0 for i in range(L)]
        if not any(act):
            break
        key0 = [x[0] for x in it]
        mid = [lo[i] + (hi[i] - lo[i]) // 2 for i in range(L)]
        ka = [key0[lo[i] + 1 if act[i] else i] for i in range(L)]
        kb = [key0[mid[i] if act[i] else i] for i in range(L)]
        kc = [key0[hi[i] - 1 if act[i] else i] for i in range(L)]
        w = [median3(ka[i], kb[i], kc[i]) for i in range(L)]
        med = [(lo[i] + 1, mid[i], hi[i] - 1)[w[i]] for i in range(L)]
        p = [(ka[i], kb[i], kc[i])[w[i]] for i in range(L)]
        src = [(med[i] if i == lo[i] else (lo[i] if i == med[i] else i)) if act[i] else i for i in range(L)]
        it = [it[src[i]] for i in range(L)]                       # the median swap (a lane permute)
        k = [x[0] for x in it]
        inr = [act[i] and i > lo[i] for i in range(L)]
        iL = [inr[i] and not k[i] < p[i] for i in range(L)]
        iR = [inr[i] and not p[i] < k[i] for i in range(L)]
        BL, BR = ballot(iL), ballot(iR)
        seg = [below(hi[i]) & ~below(lo[i] + 1) for i in range(L)]
        pl = [popc(BL & below(i) & seg[i]) for i in range(L)]
        pr = [popc(BR & below(i) & seg[i]) for i in range(L)]
        TL = [popc(BL & seg[i]) for i in range(L)]
        TR = [popc(BR & seg[i]) for i in range(L)]
        Q = ballot([inr[i] and pl[i] >= TR[i] - pr[i] for i in range(L)])
        X = [ctz(Q & seg[i]) if Q & seg[i] else hi[i] for i in range(L)]
        prX = [pr[X[i] if act[i] and X[i] < hi[i] else i] for i in range(L)]
        plX1 = [pl[X[i] - 1 if act[i] and X[i] - 1 > lo[i] else i] for i in range(L)]
        m = [max(TR[i] - prX[i] if X[i] < hi[i] else 0, plX1[i] if X[i] - 1 > lo[i] else 0) for i in range(L)]
        A = ballot([iL[i] and pl[i] == m[i] for i in range(L)])
        B = ballot([iR[i] and TR[i] - 1 - pr[i] == m[i] - 1 for i in range(L)])
        cut = [min(ctz(A & seg[i]) if m[i] < TL[i] and A & seg[i] else 64,
                   ctz(B & seg[i]) if m[i] > 0 and B & seg[i] else 64) for i in range(L)]
        sL = [iL[i] and pl[i] < m[i] for i in range(L)]
        sR = [iR[i] and TR[i] - 1 - pr[i] < m[i] for i in range(L)]
        tw = [None] * 128                                          # the partner tables (LDS)
        for i in range(L):
            if sL[i]:
                tw[lo[i] + pl[i]] = i
            if sR[i]:
                tw[64 + lo[i] + TR[i] - 1 - pr[i]] = i
        src = list(range(L))
        for i in range(L):
            if sL[i]:
                src[i] = tw[64 + lo[i] + pl[i]]
            if sR[i]:
                src[i] = tw[lo[i] + TR[i] - 1 - pr[i]]
        it = [it[src[i]] for i in range(L)]                       # the pair swaps (a lane permute)
        for i in range(L):
            if act[i]:
                if i < cut[i]:
                    hi[i] = cut[i]
                else:
                    lo[i] = cut[i]
                dd[i] -= 1
    k = [x[0] for x in it]
    out = [None] * n
    for i in range(n):   # leaves: rank by (key, lane)
        rank = sum((lo[i] + t < hi[i]) and (k[min(lo[i] + t, 63)] < k[i] or
                                             (k[min(lo[i] + t, 63)] == k[i] and lo[i] + t < i)) for t in range(16))
        out[lo[i] + rank] = it[i]
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_small_sort_is_std_sort_order(seed):
    rng = random.Random(seed)
    checked = 0
    for trial in range(600):
        n = rng.randint(2, 64)
        if trial % 4 == 0:
            items = [(i // rng.randint(1, 5), i) for i in range(n)]            # runs of equal keys
        elif trial % 4 == 1:
            items = [((n - i) // rng.randint(1, 4), i) for i in range(n)]      # reversed runs
        else:
            items = [(rng.randrange(rng.choice([1, 2, 3, 5, 10, 40])), i) for i in range(n)]
        depth = 2 * (n.bit_length() - 1)
        try:
            want = introsort(items, depth)
        except OverflowError:
            continue
        assert wave_small_sort(items, depth) == want, items
        checked += 1
    assert checked > 500


@pytest.mark.parametrize("seed", [4, 5])
def test_small_sort_merged_ranges(seed):
    """several adjacent small ranges (each with its own depth budget) sorted in
    one register call equal each range sorted alone"""
    rng = random.Random(seed)
    checked = 0
    for trial in range(400):
        segs, a = [], 0
        while a < 64:
            n = rng.choice([1, 2, 3, 7, 12, 16, 17, 25, 33, 40])
            if a + n > 64:
                break
            d = rng.randint(1, 12)
            segs.append((a, a + n, d))
            a += n
        if not segs:
            continue
        items = [(rng.randrange(rng.choice([1, 2, 4, 9])), i) for i in range(a)]
        try:
            want = []
            for lo, hi, d in segs:
                want += introsort(items[lo:hi], d)
        except OverflowError:
            continue
        assert wave_small_sort(items, 0, segs) == want, (segs, items)
        checked += 1
    assert checked > 300
