"""bench.py — scans/sec of the MI355X-native SC-LeGO-LOAM hot path.

Metric (BASELINE.json): scans/sec end-to-end (projection + segmentation +
features + odometry LM + mapping LM + Scan Context make/detect) on the
KITTI-shaped 64x1800 stream (config C3, preset hdl64_1800), synthetic data.

A step = one scan of every stream on this rank through the whole pipeline
(slo_batch_process: the reference's imageProjection -> featureAssociation ->
mapOptimization + SCManager, with the deterministic gating of SURVEY §8(d):
mapping on every 4th scan, SC detect per saved keyframe).  Each rank owns
--streams independent streams (weak scaling); per step the ranks all-gather a
160-byte record per stream (poses + newest SC ring key) over RCCL.
Inputs are generated on the host and resident in HBM before timing.  Each
stream's Scan Context history is seeded with --history earlier scans of its
own trajectory so loop detection does its full 10-NN + 10-candidate work.

The roofline object prices the dominant kernel (largest share of the timed
device time, from HIP events on the context's stream in a separate
instrumented pass) by its algorithmic bytes / average launch duration against
HBM peak.  cpu_baseline times the oracle (the C++ restatement of the
reference, oracle/) on this host's cores with the same workload, rank 0 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md); 6290 measured float4 copy


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--streams", type=int, default=64, help="streams per GPU")
    ap.add_argument("--preset", default="hdl64_1800")
    ap.add_argument("--config-id", type=int, default=3)
    ap.add_argument("--history", type=int, default=60, help="seeded Scan Context history per stream")
    ap.add_argument("--profile-steps", type=int, default=8, help="instrumented steps for the per-kernel roofline")
    ap.add_argument("--cpu-scans", type=int, default=48, help="scans per CPU thread in the baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores available)")
    return ap.parse_args()


def kernel_bytes(name, st, cfg):
    """Algorithmic HBM bytes per launch of the kernels we price (SURVEY §8(d),
    DESIGN.md "roofline"); st = summed per-stream counts of this rank."""
    H = cfg.n_scan * cfg.horizon_scan
    S = st["streams"]
    if name == "ip_project":    # read 16 B point, scatter 4 B owner
        return S * cfg.max_points * 20
    if name == "ip_image":      # owner 4 + point 16 (+2 ground pair reads on gsi rows) ; write range 4, full 16, ground 1, label 4, parent 4, csize 4, rows 16
        return S * H * (4 + 16 + 53) + S * cfg.horizon_scan * cfg.ground_scan_ind * 2 * 20
    if name == "fa_odometry":   # per search iteration: queries read the target clouds once (broadcast)
        return st["odom_bytes"]
    if name == "mo_corr":       # per LM iteration: query 16 B + 27-cell candidate reads + 5 neighbours
        return st["mocorr_bytes"]
    return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    import slo_amd

    from slo_amd import dist as sdist
    rank, world, local = sdist.env_rank()
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = slo_amd.preset(a.preset)
    pid = slo_amd.PRESETS[a.preset]
    P = cfg.max_points
    S = a.streams
    ntot = a.warmup + a.steps + a.profile_steps
    try:
        ncpu = len(os.sched_getaffinity(0))
    except Exception:
        ncpu = os.cpu_count() or 8
    gthreads = max(1, min(16, ncpu))

    # ---- inputs (host generation, then resident in HBM)
    t_gen = time.time()
    stream0, _ = sdist.stream_shard(rank, world, S)
    host = slo_amd.gen_batch(pid, a.config_id, stream0, S, 0, ntot, P, gthreads)
    dev = torch.from_numpy(host).to(f"cuda:{local}")
    del host
    cnt = torch.full((S,), P, dtype=torch.int32, device=f"cuda:{local}")

    ctx = slo_amd.Context(cfg, local, S)
    rec_n = ctx.L.slo_record_floats()
    rec = torch.zeros((S, rec_n), dtype=torch.float32, device=f"cuda:{local}")
    gathered = torch.zeros((world * S, rec_n), dtype=torch.float32, device=f"cuda:{local}") if world > 1 else None
    ext = torch.cuda.ExternalStream(ctx.stream_handle)

    # seed Scan Context history (makeAndSaveScancontextAndKeys) in chunks
    chunk = 8
    for h0 in range(-a.history, 0, chunk):
        nh = min(chunk, -h0)
        hist = slo_amd.gen_batch(pid, a.config_id, stream0, S, h0, nh, P, gthreads)
        for h in range(nh):
            d = torch.from_numpy(hist[h]).to(f"cuda:{local}")
            ctx.batch_sc_make(d.data_ptr(), cnt.data_ptr())
            ctx.synchronize()
        del hist
    t_gen = time.time() - t_gen

    def step(k):
        ctx.batch_process(dev[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        if world > 1:
            ctx.pack_records(rec.data_ptr())
            with torch.cuda.stream(ext):
                sdist.gather_records(rec, gathered)

    for k in range(a.warmup):
        step(k)
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(a.warmup, a.warmup + a.steps):
        step(k)
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    el = sdist.max_over_ranks(el, f"cuda:{local}")
    scans = S * a.steps * world
    value = scans / el

    # ---- instrumented pass: per-kernel HIP-event times on the context stream
    roof = None
    kt = {}
    if a.profile_steps > 0:
        ctx.timing(True)
        ctx.timing_reset()
        k0 = a.warmup + a.steps
        st_counts = {"streams": S, "odom_bytes": 0, "mocorr_bytes": 0}
        for k in range(k0, k0 + a.profile_steps):
            step(k)
        ctx.synchronize()
        kt = ctx.timing_read()
        ctx.timing(False)
        # algorithmic bytes for the odometry sweep and mapping correspondences
        ns = [ctx.get(s, "surf_last").shape[0] for s in range(S)]
        nc = [ctx.get(s, "corner_last").shape[0] for s in range(S)]
        nf = [ctx.get(s, "flat").shape[0] for s in range(S)]
        nsh = [ctx.get(s, "sharp").shape[0] for s in range(S)]
        it = [ctx.get(s, "fa_iters") for s in range(S)]
        # per launch: every search iteration (iter % 5 == 0) of each wave sweeps
        # the whole target cloud once (16 B/pt, broadcast) ; the other
        # iterations read queries + 2-3 neighbours (16 B each)
        ob = 0
        for s in range(S):
            srch_s = (int(it[s][0]) + 4) // 5
            srch_c = (int(it[s][1]) + 4) // 5
            waves_s = max(1, (nf[s] + 63) // 64)
            waves_c = max(1, (nsh[s] + 63) // 64)
            ob += srch_s * waves_s * ns[s] * 16 + srch_c * waves_c * nc[s] * 16
            ob += int(it[s][0]) * nf[s] * 64 + int(it[s][1]) * nsh[s] * 48
        st_counts["odom_bytes"] = ob
        total_ms = sum(v[0] for v in kt.values())
        dom = max(kt.items(), key=lambda kv: kv[1][0]) if kt else None
        if dom:
            name, (ms, n) = dom
            avg_s = ms / 1e3 / max(1, n)
            b = kernel_bytes(name, st_counts, cfg)
            if b is not None and avg_s > 0:
                ach = b / avg_s / 1e9
                roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None, "kernel": name,
                        "avg_launch_us": round(avg_s * 1e6, 2), "share_of_device_time": round(ms / total_ms, 4)}
            else:
                roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                        "traffic": None, "kernel": name, "avg_launch_us": round(avg_s * 1e6, 2),
                        "share_of_device_time": round(ms / total_ms, 4)}

    # ---- CPU baseline (oracle = C++ restatement of the reference), rank 0, N = 1
    cpu = None
    if rank == 0 and world == 1 and a.cpu_scans > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import ctypes
        import oracle_py as O
        th = a.cpu_threads or max(1, min(16, ncpu))
        stage = (ctypes.c_double * 4)()
        secs = O.lib().oracle_bench(pid, a.config_id, th, a.cpu_scans, 4, a.history, stage)
        cpu = {"value": round(th * a.cpu_scans / secs, 3), "unit": "scans/s", "cores": th, "kind": "port",
               "sample": f"{th} independent {a.preset} streams x {a.cpu_scans} scans (after 4 warm-up scans, "
                         f"{a.history}-entry SC history), oracle/ C++ restatement -O2, one stream per thread",
               "seconds": round(secs, 2),
               "stage_seconds": {"ip": round(stage[0], 2), "fa": round(stage[1], 2), "mo": round(stage[2], 2),
                                 "sc": round(stage[3], 2)}}

    if rank == 0:
        out = {
            "metric": "scans/sec end-to-end (proj+feat+LM+SC), 64-ring 1800-col",
            "value": round(value, 2), "unit": "scans/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "C3 KITTI-shaped HDL-64 64x1800 stream, full pipeline + Scan Context 20x60 K=10",
                       "preset": a.preset, "streams_per_gpu": S, "scans_per_step": S * world,
                       "sc_history_seed": a.history, "parallelism": f"streams sharded over {world} GPU(s)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "speedup_vs_cpu": round(value / cpu["value"], 2) if cpu else None,
            "kernels_ms": {k: [round(v[0], 3), int(v[1])] for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])},
            "gen_seconds": round(t_gen, 1),
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
