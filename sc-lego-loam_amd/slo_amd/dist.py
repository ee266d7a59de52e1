"""Multi-GPU layout of the batched path (mode M).

One process per GPU.  Streams are independent (each owns its pose chain,
local map and Scan Context history), so rank r owns the contiguous global
stream ids [r*S, (r+1)*S) and the data path needs no collective: every rank
advances its own S streams one scan per step (weak scaling).  The only
exchange is one batched all-gather per step of a fixed 4960-byte record per
stream (odometry pose, mapped pose, keyframe count, loop result, newest ring
key and, on a keyframe, the exact Scan Context descriptor; slo_pack_records),
so every rank holds every stream's descriptor history for cross-stream
(multi-session) loop candidates (slo_amd.xsc).  Over RCCL that is
world*S*4960 B per step: each rank contributes 2.5 MB at S = 512 and receives
the other ranks' (17.8 MB at 8 ranks), on the order of 0.1 ms of ring time on
xGMI against a ~21 ms step; measured at world size 1 (pack + gather + store
ingest + query) the exchange costs 0.73 ms per step, mostly the query.
"""
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def stream_shard(rank, world, streams_per_rank):
    """(first global stream id, count) owned by `rank`."""
    if not (0 <= rank < world) or streams_per_rank <= 0:
        raise ValueError("bad shard")
    return rank * streams_per_rank, streams_per_rank


def group_slices(streams_per_rank, groups):
    """Split a rank's streams into `groups` contiguous (offset, count) slices,
    one per context.  Each context runs on its own HIP stream and host thread,
    so one group's latency-bound phases and host round trips (the VoxelGrid
    size read) overlap the other's kernels."""
    if groups <= 0 or streams_per_rank < groups:
        raise ValueError("bad groups")
    base, extra = divmod(streams_per_rank, groups)
    out, o = [], 0
    for g in range(groups):
        n = base + (1 if g < extra else 0)
        out.append((o, n))
        o += n
    return out


def gather_records(rec, out=None):
    """All-gather the [S, F] per-stream records of every rank into
    [world*S, F], rank-major (= global stream order)."""
    world = dist.get_world_size()
    if out is None:
        out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    if dist.get_backend() == "gloo":   # CPU rehearsal: gloo has no all_gather_into_tensor
        parts = list(out.view(world, *rec.shape).unbind(0))
        dist.all_gather(parts, rec)
    else:
        dist.all_gather_into_tensor(out, rec)
    return out


def max_over_ranks(seconds, device="cpu"):
    """The slowest rank's time (bench.py reports whole-job throughput)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stop(procs):
    """SIGTERM the given processes (their own PIDs), SIGKILL what is left after 30 s"""
    for q in procs:
        q.terminate()
    t_end = time.time() + 30
    for q in procs:
        try:
            q.wait(timeout=max(0.1, t_end - time.time()))
        except subprocess.TimeoutExpired:
            q.kill()
            q.wait()


def launch_ranks(n, argv, script, poll_s=0.2, stdout=None, timeout_s=None):
    """Run `n` copies of `python script argv` as ranks 0 .. n-1 of one node
    (one process per GPU: RANK = LOCAL_RANK = r, WORLD_SIZE = n,
    MASTER_ADDR = 127.0.0.1 and a free MASTER_PORT), the way
    `torch.distributed.run --nproc-per-node n` would; the children inherit
    stdout / stderr (or write stdout to `stdout`, a file), so rank 0's output
    is the command's.  The caller's own launcher variables (TORCHELASTIC_*)
    are not passed on.  Returns 0 when every rank exits 0; otherwise the first
    failing rank's exit code, after the other ranks are stopped (their own
    PIDs, SIGTERM then SIGKILL); 124 when `timeout_s` passes first (every
    rank stopped)."""
    port = str(free_port())
    procs = []
    base = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env, stdout=stdout))
    rc = 0
    live = list(procs)
    t_end = time.time() + timeout_s if timeout_s else None
    while live:
        if t_end is not None and time.time() > t_end:
            print(f"launch_ranks: {len(live)} rank(s) still running after {timeout_s} s; stopping them",
                  file=sys.stderr, flush=True)
            _stop(live)
            return 124
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"launch_ranks: rank {procs.index(p)} exited with {c}; stopping the others", file=sys.stderr,
                      flush=True)
                _stop(live)
                live = []
                break
        time.sleep(poll_s)
    return rc
