"""Mode S: one vehicle's stream over several contexts or ranks.

The reference deploys one stream as a pipeline of processes
(imageProjection | featureAssociation | mapOptimization,
launch/run.launch:14-17).  Mode S deals the scans' front ends round-robin
over `world` ranks — scan k's imageProjection and featureAssociation feature
extraction (FA:1833-1841) on rank k % world — and runs every scan's back end
(odometry FA:1843-1858, mapOptimization, Scan Context) on the owner, rank 0.
Per scan two buffers travel (include/slo_abi.h "Mode S"):
- the carry, from scan k's front rank to scan k+1's: the stale state a front
  end inherits from the previous scan;
- the features, from scan k's front rank to the owner.
`run_rank3` splits the back end once more, the reference's third process
boundary: odometry on rank 1, mapping + transformFusion + Scan Context on
rank 0, a third buffer (the odometry hand-off) between them.

The rank drivers (`run_rank`, `run_rank3`) are written against an engine
interface that both engines implement:
- `rank_front(scan, t, carry_in, need_carry)` -> (carry or None, features);
  carry_in None = the previous scan's front end ran on this engine;
- `rank_back(features, scan, t)` -> flags; `rank_odometry(features, scan, t)`
  -> the odometry buffer; `rank_mapping(odom, scan, t)` -> flags;
- `recv_buffer(tag)` -> a buffer to receive that tag into (None: the
  transport allocates);
`SloEngine` here (libslo contexts, device buffers: RCCL moves them between
GPUs with `DistTransport`, `LocalTransport` between threads of one process)
and the oracle engine of the CPU rehearsal (tests/mode_engines.py, gloo).
The owner's poses, keyframes and loop ids are bit-identical to a one-context
run (tests/test_modes_gloo.py, tests/test_gpu_modes.py).

What it can buy is bounded by the owner (Amdahl): the front ends leave the
owner, the back ends do not, and the carry chain serialises the feature
extraction of consecutive scans (each waits for the previous scan's carry);
only imageProjection runs fully in parallel.  DESIGN.md §8 gives the bound
from the measured stage split and the bytes per scan.
"""
import numpy as np


class SloEngine:
    """libslo on one GPU: `fronts` front contexts, an owner context and (with
    split_back) an odometry context, each one stream (or n_streams vehicles
    split the same way); buffers are torch uint8 device tensors.  owner=False
    leaves the owner out (a front-only rank of run_rank3)."""

    def __init__(self, cfg, fronts=1, device=0, n_streams=1, split_back=False, owner=True, read_flags=True):
        import torch
        import slo_amd
        self.torch = torch
        self.L = slo_amd._abi.lib()
        self.fronts = [slo_amd.Context(cfg, device, n_streams) for _ in range(fronts)]
        self.owner = slo_amd.Context(cfg, device, n_streams) if owner else None
        if self.owner is not None:   # the one context here that maps: its workspaces up front
            self.owner.prepare_mapping()
        # split_back: the back end on two contexts, odometry (self.odo) and
        # mapping (self.owner, which then holds the results)
        self.odo = slo_amd.Context(cfg, device, n_streams) if split_back else None
        any_ctx = next(c for c in self.fronts + [self.owner, self.odo] if c is not None)
        self.cbytes = int(self.L.slo_modes_carry_bytes(any_ctx.h))
        self.fbytes = int(self.L.slo_modes_features_bytes(any_ctx.h))
        self.obytes = int(self.L.slo_modes_odom_bytes(any_ctx.h))
        self.dev = torch.device("cuda", device)
        self.read_flags = read_flags
        self._ring = {}

    @classmethod
    def for_rank(cls, cfg, rank, world, split_back=False, device=0, n_streams=1, read_flags=True):
        """the contexts rank `rank` of run_rank (split_back False) or
        run_rank3 (True) needs: every rank of run_rank runs front ends, rank 0
        also the owner; in run_rank3 rank 0 maps, rank 1 runs the odometry,
        the others the front ends"""
        if not split_back:
            return cls(cfg, fronts=1, device=device, n_streams=n_streams, owner=rank == 0, read_flags=read_flags)
        return cls(cfg, fronts=1 if rank >= 2 else 0, device=device, n_streams=n_streams, split_back=rank == 1,
                   owner=rank == 0, read_flags=read_flags)

    def buffers(self):
        t = self.torch
        return (t.empty(self.cbytes, dtype=t.uint8, device=self.dev),
                t.empty(self.fbytes, dtype=t.uint8, device=self.dev))

    def front(self, slot, d_points, d_counts, t, carry_in, carry_out, features_out):
        ctx = self.fronts[slot]
        ctx._ok(self.L.slo_front_process(ctx.h, d_points, d_counts, float(t),
                                         None if carry_in is None else carry_in.data_ptr(),
                                         None if carry_out is None else carry_out.data_ptr(),
                                         features_out.data_ptr()), "slo_front_process")
        ctx.synchronize()   # the buffers are complete before they travel

    def odom_buffer(self):
        return self.torch.empty(self.obytes, dtype=self.torch.uint8, device=self.dev)

    def back(self, features, d_points, d_counts, t):
        if self.odo is not None:   # the two back-end stages one after the other
            o = self.odom_buffer()
            self.odometry(features, d_points, d_counts, t, o)
            self.mapping(o, d_points, d_counts, t)
            return
        self.owner._ok(self.L.slo_back_process(self.owner.h, features.data_ptr(), d_points, d_counts, float(t)),
                       "slo_back_process")

    def odometry(self, features, d_points, d_counts, t, odom_out):
        self.odo._ok(self.L.slo_odom_process(self.odo.h, features.data_ptr(), d_points, d_counts, float(t),
                                             odom_out.data_ptr()), "slo_odom_process")
        self.odo.synchronize()   # the odometry buffer is complete, the features slot read

    def mapping(self, odom, d_points, d_counts, t):
        self.owner._ok(self.L.slo_map_process(self.owner.h, odom.data_ptr(), d_points, d_counts, float(t)),
                       "slo_map_process")

    # ---- the rank interface (run_rank / run_rank3); scan = (device points, device counts)
    def _buf(self, name, nbytes):
        """two alternating buffers per kind: a buffer handed out for scan k is
        not written again before scan k + 2 (the drivers drain the sends of
        each scan before the next)"""
        pair = self._ring.get(name)
        if pair is None:
            pair = self._ring[name] = [[self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.dev) for _ in
                                        range(2)], 0]
        b = pair[0][pair[1]]
        pair[1] ^= 1
        return b

    def recv_buffer(self, tag):
        return self._buf(("recv", tag), {TAG_CARRY: self.cbytes, TAG_FEATURES: self.fbytes, TAG_ODOM: self.obytes}[tag])

    def _flags(self):
        return int(self.owner.get(0, "flags")[0]) if self.read_flags else None

    def rank_front(self, scan, t, carry_in, need_carry):
        cout = self._buf("carry", self.cbytes) if need_carry else None
        feat = self._buf("features", self.fbytes)
        self.front(0, scan[0], scan[1], t, carry_in, cout, feat)
        return cout, feat

    def rank_back(self, features, scan, t):
        self.back(features, scan[0], scan[1], t)
        self.owner.synchronize()   # the features buffer is read before the next recv reuses it
        return self._flags()

    def rank_odometry(self, features, scan, t):
        o = self._buf("odom", self.obytes)
        self.odometry(features, scan[0], scan[1], t, o)
        return o

    def rank_mapping(self, odom, scan, t):
        self.mapping(odom, scan[0], scan[1], t)
        self.owner.synchronize()
        return self._flags()

    def close(self):
        for c in self.fronts + [self.owner, self.odo]:
            if c is not None:
                c.close()


def front_rank(k, world):
    """the rank that runs scan k's front end"""
    return k % world


TAG_CARRY, TAG_FEATURES, TAG_ODOM = 1, 2, 3


class DistTransport:
    """torch.distributed point-to-point (gloo on CPU tensors, RCCL on device
    tensors); variable-size blobs go as (length, bytes).  RCCL ignores tags:
    the drivers order each pair of ranks' messages the same way on both sides."""

    def __init__(self):
        import torch
        import torch.distributed as dist
        self.t, self.d = torch, dist
        self.pending, self.keep = [], []

    def send(self, x, dst, tag):
        t = self.t
        x = t.as_tensor(np.ascontiguousarray(x)) if isinstance(x, np.ndarray) else x
        n = t.tensor([x.numel()], dtype=t.int64, device=x.device)
        self.pending += [self.d.isend(n, dst, tag=tag), self.d.isend(x, dst, tag=tag)]
        self.keep += [n, x]   # alive until drain()

    def recv(self, src, tag, like=None):
        t = self.t
        dev = like.device if like is not None else "cpu"
        n = t.zeros(1, dtype=t.int64, device=dev)
        self.d.recv(n, src, tag=tag)
        x = t.empty(int(n.item()), dtype=t.uint8, device=dev) if like is None else like[:int(n.item())]
        self.d.recv(x, src, tag=tag)
        if like is None:
            return x.numpy()
        if x.is_cuda:   # the engine's own HIP stream reads it next
            t.cuda.current_stream(x.device).synchronize()
        return x

    def drain(self):
        """every send of this scan complete before its buffers are handed out
        again: Work.wait() on an RCCL send only orders the current stream
        after it, so for device tensors the host then waits on that stream too
        (libslo's own HIP stream, which writes the buffers next, is not
        ordered against RCCL's)"""
        for r in self.pending:
            r.wait()
        cuda = sorted({x.device.index for x in self.keep if x.is_cuda})
        for d in cuda:
            self.t.cuda.current_stream(d).synchronize()
        self.pending, self.keep = [], []


class HostTransport(DistTransport):
    """DistTransport for a group whose backend moves host tensors only
    (gloo): a device buffer is staged through pinned host memory on both
    sides — the fallback of bench.py's Mode S leg when RCCL point-to-point is
    not available; the drivers and their message order are the same"""

    def send(self, x, dst, tag):
        if not isinstance(x, np.ndarray) and x.is_cuda:
            x = x.to("cpu")   # synchronous: the buffer is complete before it travels
        super().send(x, dst, tag)

    def recv(self, src, tag, like=None):
        if like is None or not like.is_cuda:
            return super().recv(src, tag, like)
        host = super().recv(src, tag, None)   # a numpy array of the message's bytes
        x = like[:host.size]
        x.copy_(self.t.from_numpy(host))
        self.t.cuda.current_stream(x.device).synchronize()
        return x


class LocalTransport:
    """the ranks as threads of one process (one GPU, or CPU engines): one
    mailbox per (source, destination, tag); a sent buffer is copied, so the
    sender may reuse it at once.  `boxes` is shared by every rank's transport
    (LocalTransport.group(world))."""

    def __init__(self, rank, boxes, timeout=300.0):
        self.rank, self.boxes, self.timeout = rank, boxes, timeout

    @staticmethod
    def group(world):
        import queue
        boxes = {(a, b, g): queue.Queue() for a in range(world) for b in range(world)
                 for g in (TAG_CARRY, TAG_FEATURES, TAG_ODOM)}
        return [LocalTransport(r, boxes) for r in range(world)]

    def send(self, x, dst, tag):
        if isinstance(x, np.ndarray):
            y = x.copy()
        else:
            import torch
            y = x.clone()
            if y.is_cuda:
                torch.cuda.current_stream(y.device).synchronize()
        self.boxes[(self.rank, dst, tag)].put(y)

    def recv(self, src, tag, like=None):
        y = self.boxes[(src, self.rank, tag)].get(timeout=self.timeout)
        if like is None:
            return y
        import torch
        x = like[:y.numel()]
        x.copy_(y)
        if x.is_cuda:
            torch.cuda.current_stream(x.device).synchronize()
        return x

    def drain(self):
        pass


def run_rank(engine, rank, world, scan_fn, n_scans, transport, on_back=None):
    """Mode S, this rank's part of scans 0 .. n_scans-1: scan k's front end
    on rank k % world, every back end on rank 0 (the owner).  scan_fn(k) ->
    (scan, t), scan in the engine's own form.  The owner calls on_back(k,
    flags) after each back end; returns the owner's flags.  Per pair of ranks
    the messages go in one order (features of scan k, then its carry), so a
    transport without tags (RCCL) pairs them as well as one with (gloo)."""
    flags = []
    for k in range(n_scans):
        f = front_rank(k, world)
        scan, t = scan_fn(k)
        feat = None
        if rank == f:
            prev = front_rank(k - 1, world) if k > 0 else None
            carry_in = None   # the previous scan's front end ran here (its state is this engine's), or none ran
            if prev is not None and prev != rank:
                carry_in = transport.recv(prev, TAG_CARRY, engine.recv_buffer(TAG_CARRY))
            nxt = front_rank(k + 1, world)
            need = k + 1 < n_scans and nxt != rank
            carry, feat = engine.rank_front(scan, t, carry_in, need)
            if rank != 0:
                transport.send(feat, 0, TAG_FEATURES)
            if need:
                transport.send(carry, nxt, TAG_CARRY)
        if rank == 0:
            if f != 0:
                feat = transport.recv(f, TAG_FEATURES, engine.recv_buffer(TAG_FEATURES))
            fl = engine.rank_back(feat, scan, t)
            flags.append(fl)
            if on_back:
                on_back(k, fl)
        transport.drain()
    return flags


def run_rank3(engine, rank, world, scan_fn, n_scans, transport, on_back=None):
    """Mode S with the back end split over two ranks, the reference's three
    processes (launch/run.launch:14-17) as ranks: rank 0 the mapping stage
    (transformFusion, mapOptimization, Scan Context: the owner), rank 1 the
    odometry, ranks 2 .. world-1 the front ends in turn (world >= 3).  Scan
    k's features go from its front rank to rank 1, its odometry buffer from
    rank 1 to rank 0.  Returns the owner's flags (rank 0), as run_rank."""
    assert world >= 3, "a front rank, the odometry rank and the owner"
    nf = world - 2
    flags = []
    for k in range(n_scans):
        f = 2 + k % nf
        scan, t = scan_fn(k)
        if rank == f:
            prev = 2 + (k - 1) % nf if k > 0 else None
            carry_in = None
            if prev is not None and prev != rank:
                carry_in = transport.recv(prev, TAG_CARRY, engine.recv_buffer(TAG_CARRY))
            nxt = 2 + (k + 1) % nf
            need = k + 1 < n_scans and nxt != rank
            carry, feat = engine.rank_front(scan, t, carry_in, need)
            transport.send(feat, 1, TAG_FEATURES)
            if need:
                transport.send(carry, nxt, TAG_CARRY)
        elif rank == 1:
            feat = transport.recv(f, TAG_FEATURES, engine.recv_buffer(TAG_FEATURES))
            transport.send(engine.rank_odometry(feat, scan, t), 0, TAG_ODOM)
        elif rank == 0:
            fl = engine.rank_mapping(transport.recv(1, TAG_ODOM, engine.recv_buffer(TAG_ODOM)), scan, t)
            flags.append(fl)
            if on_back:
                on_back(k, fl)
        transport.drain()
    return flags


def run_local_slo(engine, world, d_scans, d_counts, times, on_back=None):
    """Mode S inside one process on one GPU: `world` front contexts take the
    scans' front ends in turn (engine.fronts[k % world]), the owner runs every
    back end; the carry and features move as device buffers (the ranks of a
    multi-GPU run move the same buffers with RCCL send / recv).  d_scans[k]:
    the device pointer of scan k's points."""
    carry = [engine.buffers()[0] for _ in range(2)]
    feat = engine.buffers()[1]
    for k in range(len(times)):
        cin = carry[(k + 1) & 1] if k > 0 else None
        engine.front(k % world, d_scans[k], d_counts, times[k], cin, carry[k & 1], feat)
        engine.back(feat, d_scans[k], d_counts, times[k])
        if on_back:
            on_back(k)


def run_pipelined_slo(engine, world, d_scans, d_counts, times, depth=3, on_back=None):
    """Mode S as a two-stage pipeline on one GPU — the reference's own
    process split (imageProjection + feature extraction | odometry +
    mapOptimization) — with a host thread per stage: the front thread runs
    scan k + 1's front end while the owner runs scan k's back end, through a
    ring of `depth` feature buffers.  Only when the work runs changes, not
    what: the owner's results equal run_local_slo's (tests/test_gpu_modes.py).
    Returns (front seconds, back seconds) summed over the scans, each stage
    timed on its own thread."""
    import queue
    import threading
    import time
    n = len(times)
    feats = [engine.buffers()[1] for _ in range(depth)]
    carry = [engine.buffers()[0] for _ in range(2)] if world > 1 else [None, None]
    free, ready = queue.Queue(), queue.Queue()
    for i in range(depth):
        free.put(i)
    err, tf = [], [0.0]

    def fronts():
        try:
            for k in range(n):
                slot = free.get()
                if slot is None:   # the owner stopped
                    ready.put(None)
                    return
                t0 = time.perf_counter()
                cin = carry[(k + 1) & 1] if (k > 0 and world > 1) else None
                engine.front(k % world, d_scans[k], d_counts, times[k], cin, carry[k & 1], feats[slot])
                tf[0] += time.perf_counter() - t0
                ready.put((k, slot))
        except Exception as e:   # handed to the owner thread, which raises it
            err.append(e)
            ready.put(None)

    th = threading.Thread(target=fronts)
    th.start()
    tb = 0.0
    try:
        for _ in range(n):
            item = ready.get()
            if item is None:
                break
            k, slot = item
            t0 = time.perf_counter()
            engine.back(feats[slot], d_scans[k], d_counts, times[k])
            engine.owner.synchronize()   # the owner has read the slot
            tb += time.perf_counter() - t0
            free.put(slot)
            if on_back:
                on_back(k)
    except BaseException:
        free.put(None)   # a front thread waiting for a slot stops instead of waiting forever
        raise
    finally:
        th.join()
    if err:
        raise err[0]
    return tf[0], tb


def run_pipelined3_slo(engine, world, d_scans, d_counts, times, depth=6, on_back=None):
    """Mode S as three stages on one GPU, the reference's three processes
    (imageProjection + feature extraction | odometry | mapOptimization with
    transformFusion and Scan Context, launch/run.launch:14-17): a host thread
    per stage, each on its own contexts (engine built with split_back=True),
    rings of `depth` feature and odometry buffers between them.  The mapping
    stage is bursty (a ~3 ms mapping step every mapping_process_interval,
    little in between): the rings absorb the bursts — on C3, depth 3 gave 933
    scans/s, depth 6 1184 (tools/pipe_depth.py).  Scan k + 2's
    front end, scan k + 1's odometry and scan k's mapping step run at once.
    The mapping context's results equal a one-context run's
    (tests/test_gpu_modes.py).  Returns (front, odometry, mapping) seconds
    summed over the scans, each stage timed on its own thread."""
    import queue
    import threading
    import time
    assert engine.odo is not None, "run_pipelined3_slo needs SloEngine(split_back=True)"
    n = len(times)
    feats = [engine.buffers()[1] for _ in range(depth)]
    odoms = [engine.odom_buffer() for _ in range(depth)]
    carry = [engine.buffers()[0] for _ in range(2)] if world > 1 else [None, None]
    ffree, fready, ofree, oready = queue.Queue(), queue.Queue(), queue.Queue(), queue.Queue()
    for i in range(depth):
        ffree.put(i)
        ofree.put(i)
    err, tf, to = [], [0.0], [0.0]

    def fronts():
        try:
            for k in range(n):
                slot = ffree.get()
                if slot is None:   # a later stage stopped
                    fready.put(None)
                    return
                t0 = time.perf_counter()
                cin = carry[(k + 1) & 1] if (k > 0 and world > 1) else None
                engine.front(k % world, d_scans[k], d_counts, times[k], cin, carry[k & 1], feats[slot])
                tf[0] += time.perf_counter() - t0
                fready.put((k, slot))
        except Exception as e:   # handed on down the pipeline, raised by the caller
            err.append(e)
            fready.put(None)

    def odometry():
        try:
            for _ in range(n):
                item = fready.get()
                if item is None:
                    break
                k, fs = item
                os_ = ofree.get()
                if os_ is None:
                    break
                t0 = time.perf_counter()
                engine.odometry(feats[fs], d_scans[k], d_counts, times[k], odoms[os_])
                to[0] += time.perf_counter() - t0
                ffree.put(fs)
                oready.put((k, os_))
            else:
                return
            ffree.put(None)   # stopped early: stop the other stages too
            oready.put(None)
        except Exception as e:
            err.append(e)
            ffree.put(None)
            oready.put(None)

    ths = [threading.Thread(target=fronts), threading.Thread(target=odometry)]
    for th in ths:
        th.start()
    tm = 0.0
    try:
        for _ in range(n):
            item = oready.get()
            if item is None:
                break
            k, os_ = item
            t0 = time.perf_counter()
            engine.mapping(odoms[os_], d_scans[k], d_counts, times[k])
            engine.owner.synchronize()   # the mapping context has read the slot
            tm += time.perf_counter() - t0
            ofree.put(os_)
            if on_back:
                on_back(k)
    except BaseException:
        ofree.put(None)
        ffree.put(None)
        raise
    finally:
        for th in ths:
            th.join()
    if err:
        raise err[0]
    return tf[0], to[0], tm
