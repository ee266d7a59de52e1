"""TEST INFRASTRUCTURE.  A lane-level Python emulation of the wave tier of
the PCL-order VoxelGrid sort (csrc/slo_pclsort.h pcl_wave_sort): the same
rows of 64 lanes, ballots, prefix / select from the ballots, binary search
for m, cut, swap partners, child tables and leaf ranks, step for step — and
a plain restatement of libstdc++'s std::sort (slo_introsort.h) to check it
against.  Used by tests/test_pclsort_cpu.py."""
KWT, ROWS, KDONE, KHEAP = 512, 8, 0xff, 0xff


def std_sort(keys):
    """libstdc++ std::sort of [(key, idx)] by key only (slo_introsort.h)."""
    a = list(keys)
    n = len(a)
    if n <= 1:
        return a

    def lt(x, y):
        return x[0] < y[0]

    def median_to_first(r, i, j, k):
        if lt(a[i], a[j]):
            if lt(a[j], a[k]):
                a[r], a[j] = a[j], a[r]
            elif lt(a[i], a[k]):
                a[r], a[k] = a[k], a[r]
            else:
                a[r], a[i] = a[i], a[r]
        elif lt(a[i], a[k]):
            a[r], a[i] = a[i], a[r]
        elif lt(a[j], a[k]):
            a[r], a[k] = a[k], a[r]
        else:
            a[r], a[j] = a[j], a[r]

    def partition(first, last, piv):
        while True:
            while lt(a[first], a[piv]):
                first += 1
            last -= 1
            while lt(a[piv], a[last]):
                last -= 1
            if not first < last:
                return first
            a[first], a[last] = a[last], a[first]
            first += 1

    def heapsort(lo, hi):
        sub = sorted(range(lo, hi), key=lambda i: 0)  # placeholder, replaced below
        del sub
        b = a[lo:hi]
        # libstdc++ make_heap + sort_heap
        L = len(b)

        def push(hole, top, v):
            parent = (hole - 1) // 2
            while hole > top and lt(b[parent], v):
                b[hole] = b[parent]
                hole = parent
                parent = (hole - 1) // 2
            b[hole] = v

        def adjust(hole, ln, v):
            top = hole
            second = hole
            while second < (ln - 1) // 2:
                second = 2 * (second + 1)
                if lt(b[second], b[second - 1]):
                    second -= 1
                b[hole] = b[second]
                hole = second
            if (ln & 1) == 0 and second == (ln - 2) // 2:
                second = 2 * (second + 1)
                b[hole] = b[second - 1]
                hole = second - 1
            push(hole, top, v)
        if L >= 2:
            parent = (L - 2) // 2
            while True:
                adjust(parent, L, b[parent])
                if parent == 0:
                    break
                parent -= 1
        ln = L
        while ln > 1:
            ln -= 1
            v = b[ln]
            b[ln] = b[0]
            adjust(0, ln, v)
        a[lo:hi] = b

    lg = n.bit_length() - 1
    stack = [(0, n, 2 * lg)]
    while stack:
        lo, hi, d = stack.pop()
        while hi - lo > 16:
            if d == 0:
                heapsort(lo, hi)
                break
            d -= 1
            median_to_first(lo, lo + 1, lo + (hi - lo) // 2, hi - 1)
            c = partition(lo + 1, hi, lo)
            stack.append((c, hi, d))
            hi = c
    # final insertion sort (stable)
    for i in range(1, n):
        v = a[i]
        j = i - 1
        while j >= 0 and lt(v, a[j]):
            a[j + 1] = a[j]
            j -= 1
        a[j + 1] = v
    return a


def popc(x):
    return bin(x).count("1")


def wave_sort(items, F, n, depth):
    """Emulates pcl_wave_sort on items[F:F+n] (list of (key, idx)), in place."""
    E = F + n
    ln = range(64)
    st = [[0] * 64 for _ in range(ROWS)]
    act0 = n > 16 and depth > 0
    for j in range(ROWS):
        for t in ln:
            x = F + 64 * j + t
            st[j][t] = ((0 if (act0 and x < E) else KDONE) | ((n if n <= 16 else KHEAP) << 8) | (F << 16))
    ns = 1 if act0 else 0
    nheap = 1 if (not act0 and n > 16) else 0
    tab = [(F, E, depth)]                     # lane s < ns: (tf, tl, td)
    heaps = [(F, E)] if nheap else []

    def prefix(b, cum, r):
        row = r >> 6
        if row >= ROWS:
            return cum[ROWS]
        return cum[row] + popc(b[row] & ((1 << (r & 63)) - 1))

    def select(b, cum, k):
        row = sum(1 for j in range(1, ROWS) if k >= cum[j])
        x, kk, p = b[row], k - cum[row], 0
        w = 32
        while w >= 1:
            c = popc(x & ((1 << w) - 1))
            if kk >= c:
                kk -= c
                x >>= w
                p += w
            w >>= 1
        return row * 64 + p

    while ns > 0:
        # (1) medians
        piv = []
        for s in range(ns):
            tf, tl, _ = tab[s]
            i, j, k = tf + 1, tf + (tl - tf) // 2, tl - 1
            a = items
            lt = lambda u, v: a[u][0] < a[v][0]  # noqa
            if lt(i, j):
                m = j if lt(j, k) else (k if lt(i, k) else i)
            elif lt(i, k):
                m = i
            elif lt(j, k):
                m = k
            else:
                m = j
            a[tf], a[m] = a[m], a[tf]
            piv.append(a[tf][0])
        # (2) ballots
        bL, bR = [0] * ROWS, [0] * ROWS
        for j in range(ROWS):
            for t in ln:
                x = F + 64 * j + t
                s = st[j][t] & 0xff
                if s == KDONE or x >= E:
                    continue
                if x == tab[s][0]:
                    continue
                k = items[x][0]
                if not k < piv[s]:
                    bL[j] |= 1 << t
                if not piv[s] < k:
                    bR[j] |= 1 << t
        cL, cR = [0] * (ROWS + 1), [0] * (ROWS + 1)
        for j in range(ROWS):
            cL[j + 1] = cL[j] + popc(bL[j])
            cR[j + 1] = cR[j] + popc(bR[j])
        # (3)
        res = []
        for s in range(ns):
            tf, tl, td = tab[s]
            r0, r1 = tf + 1 - F, tl - F
            tsL, teR = prefix(bL, cL, r0), prefix(bR, cR, r1)
            key = tsL + teR
            lo, hi = r0, r1
            for _ in range(10):
                mid = (lo + hi) >> 1
                ge = prefix(bL, cL, mid) + prefix(bR, cR, mid) >= key
                if lo < hi:
                    if ge:
                        hi = mid
                    else:
                        lo = mid + 1
            tm = teR - prefix(bR, cR, lo) if lo < r1 else 0
            if lo > r0:
                tm = max(tm, prefix(bL, cL, lo - 1) - tsL)
            tL = prefix(bL, cL, r1)
            INF = 0x7fffffff
            cutA = F + select(bL, cL, tsL + tm) if tsL + tm < tL else INF
            cutB = F + select(bR, cR, teR - tm) if tm > 0 else INF
            res.append((tsL, teR, tm, min(cutA, cutB)))
        # (4) swaps (reads first, then writes)
        swaps = []
        for j in range(ROWS):
            for t in ln:
                if not (bL[j] >> t) & 1:
                    continue
                s = st[j][t] & 0xff
                sL, eR, m, _ = res[s]
                k = cL[j] + popc(bL[j] & ((1 << t) - 1)) - sL
                if k < m:
                    swaps.append((F + 64 * j + t, F + select(bR, cR, eR - 1 - k)))
        old = list(items)
        for x, y in swaps:
            items[x], items[y] = old[y], old[x]
        # (5) children
        nt, nh = [], []
        nid = []
        for s in range(ns):
            tf, tl, td = tab[s]
            cut, D = res[s][3], td - 1
            assert tf < cut < tl, (tf, cut, tl)
            idl = idr = -1
            if cut - tf > 16 and D > 0:
                idl = len(nt)
                nt.append((tf, cut, D))
            if tl - cut > 16 and D > 0:
                idr = len(nt)
                nt.append((cut, tl, D))
            if cut - tf > 16 and D == 0:
                nh.append((tf, cut))
            if tl - cut > 16 and D == 0:
                nh.append((cut, tl))
            nid.append((idl, idr))
        heaps += nh
        for j in range(ROWS):
            for t in ln:
                s = st[j][t] & 0xff
                if s == KDONE:
                    continue
                x = F + 64 * j + t
                tf, tl, _ = tab[s]
                cut = res[s][3]
                left = x < cut
                i = nid[s][0 if left else 1]
                if i >= 0:
                    st[j][t] = (st[j][t] & ~0xff) | i
                else:
                    lo, hi = (tf, cut) if left else (cut, tl)
                    st[j][t] = KDONE | ((hi - lo if hi - lo <= 16 else KHEAP) << 8) | (lo << 16)
        tab = nt
        ns = len(nt)
    # heaps
    for lo, hi in heaps:
        items[lo:hi] = std_sort_heap(items[lo:hi])
    # leaves
    out = list(items)
    for j in range(ROWS):
        for t in ln:
            x = F + 64 * j + t
            lo, sz = st[j][t] >> 16, (st[j][t] >> 8) & 0xff
            if x >= E or sz == KHEAP:
                continue
            k = items[x][0]
            r = sum(1 for y in range(lo, lo + sz) if items[y][0] < k or (items[y][0] == k and y < x))
            out[lo + r] = items[x]
    items[:] = out


def std_sort_heap(b):
    """libstdc++ heapsort (make_heap + sort_heap) of a list of (key, idx)."""
    tmp = [(k, i) for k, i in b]
    srt = std_sort.__wrapped__(tmp) if hasattr(std_sort, "__wrapped__") else None
    del srt
    a = list(b)
    L = len(a)

    def lt(x, y):
        return x[0] < y[0]

    def push(hole, top, v):
        parent = (hole - 1) // 2
        while hole > top and lt(a[parent], v):
            a[hole] = a[parent]
            hole = parent
            parent = (hole - 1) // 2
        a[hole] = v

    def adjust(hole, ln, v):
        top = hole
        second = hole
        while second < (ln - 1) // 2:
            second = 2 * (second + 1)
            if lt(a[second], a[second - 1]):
                second -= 1
            a[hole] = a[second]
            hole = second
        if (ln & 1) == 0 and second == (ln - 2) // 2:
            second = 2 * (second + 1)
            a[hole] = a[second - 1]
            hole = second - 1
        push(hole, top, v)
    if L >= 2:
        parent = (L - 2) // 2
        while True:
            adjust(parent, L, a[parent])
            if parent == 0:
                break
            parent -= 1
    ln = L
    while ln > 1:
        ln -= 1
        v = a[ln]
        a[ln] = a[0]
        adjust(0, ln, v)
    return a
