"""HBM budget of a bench rank (bench.py): contexts, the resident input
window, the cross-stream Scan Context store, and what is left.

A rank holds, per GPU:
- its contexts (slo_create: every stream's persistent state, measured with
  mem_get_info around their creation);
- the cross-stream store when records are gathered (slo_xsc_create,
  csrc/slo_xsc.hip:199-202: per global stream and keyframe slot a 20 x 60
  f64 descriptor, a 60 f64 sector key, a 20 f32 ring key and an index);
- the resident input window: `scans` whole steps of every stream's points
  (S x P x 16 B per step), generated on the device before a timed segment.

The window is sized from what is free after the contexts and the store, less
a reserve for the runtime's scratch (kernel scratch, graph instantiation,
the legs after the timed region).  When the steps asked for do not fit at
once, bench.py times them in segments: each segment's scans are generated
untimed, then the segment is timed between barriers like the whole run.
"""

GIB = 1 << 30


def point_bytes():
    """one input point on the device: x, y, z, intensity f32"""
    return 16


def step_bytes(streams, max_points):
    """one step of the window: every stream's scan"""
    return int(streams) * int(max_points) * point_bytes()


def xsc_bytes(n_streams, cap, nr=20, ns=60):
    """bytes slo_xsc_create allocates (csrc/slo_xsc.hip:199-203)"""
    e = int(n_streams) * int(cap)
    return e * (nr * ns * 8 + ns * 8 + nr * 4 + 4) + int(n_streams) * 4


def window_scans(free_bytes, step_b, need_scans, lag_scans=0, store_b=0, reserve_b=8 * GIB, cap_scans=0):
    """scans of every stream resident at once: as many as fit in
    free - store - reserve (at most need_scans + lag_scans, at most cap_scans
    when given), and at least lag_scans + 1 (one step of every context);
    raises MemoryError with the arithmetic when even that does not fit"""
    avail = int(free_bytes) - int(store_b) - int(reserve_b)
    fit = avail // int(step_b) if avail > 0 else 0
    want = int(need_scans) + int(lag_scans)
    if cap_scans:
        want = min(want, int(cap_scans) + int(lag_scans))
    if fit < lag_scans + 1:
        raise MemoryError(
            f"HBM budget: {free_bytes / GIB:.2f} GiB free after the contexts, cross-stream store "
            f"{store_b / GIB:.2f} GiB, reserve {reserve_b / GIB:.2f} GiB: room for {fit} scan(s) of "
            f"{step_b / GIB:.3f} GiB each, {lag_scans + 1} needed (fewer --streams, or a smaller --hbm-reserve-gb)")
    return int(min(fit, want))


def segments(k0, k1, seg_len):
    """[k0, k1) in consecutive pieces of at most seg_len"""
    if seg_len <= 0:
        raise ValueError("seg_len")
    out, k = [], k0
    while k < k1:
        n = min(seg_len, k1 - k)
        out.append((k, n))
        k += n
    return out
