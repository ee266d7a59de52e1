"""bench.py — scans/sec of the MI355X-native SC-LeGO-LOAM hot path.

Metric (BASELINE.json): scans/sec end-to-end (projection + segmentation +
features + odometry LM + mapping LM + Scan Context make/detect) on the
KITTI-shaped 64x1800 stream (config C3, preset hdl64_1800), synthetic data.

A step = one scan of every stream on this rank through the whole pipeline
(slo_batch_process: the reference's imageProjection -> featureAssociation ->
mapOptimization + SCManager, with the deterministic gating of SURVEY §8(d):
mapping on every 4th scan, SC detect per saved keyframe).  Each rank owns
--streams independent streams (weak scaling, slo_amd/dist.py); per step the
ranks all-gather a 4960-byte record per stream (poses, ids, loop result and —
when the stream saved a keyframe — its exact Scan Context descriptor) over
RCCL, and every rank's cross-stream store (slo_amd.xsc) ingests the gathered
table and runs the multi-session loop query for its own streams (SURVEY
§8(e)).

Steady state: every stream first runs --preroll scans untimed (default 210:
the local map holds its full 50 keyframes, MO:1127-1166, and Scan Context
detect has >= 51 contexts, SCc:257), fed in chunks; then the --warmup and
timed --steps scans are generated and resident in HBM before timing.  Inputs
come from the device generator (csrc/slo_gendev.hip), bit-identical to the
host generator the CPU baseline uses.  A one-stream leg (single_stream)
reports the same pipeline for a single C3 stream: scans/s and per-scan
latency.

roofline: the dominant kernel (--roofline-kernel auto: the largest single
kernel by device time in the instrumented pass — with the reference's
VoxelGrid order, pc_finish_b, the LDS finish of the PCL-order sort) timed by
in-stream device timestamps on its context's stream inside the timed region
(the same for --roofline-also, reported under roofline_also); achieved = its
algorithmic bytes per launch (DESIGN.md "Roofline", from the per-stream counts
of a separate instrumented pass with the same
launch mix) / that average launch time, against HBM peak.  `isolated` repeats
it for the instrumented pass, where the contexts run one after the other.  cpu_baseline: the
oracle (oracle/, C++ restatement of the reference path), rank 0 at N = 1, on
the same steady-state window: (B) one stream per usable host core (min of
sched_getaffinity and the cgroup CPU quota), --cpu-scans scans each after the
pre-roll;
(A) the reference's topology — one stream as a 3-stage pipeline
(imageProjection | featureAssociation | mapOptimization, launch/run.launch) on
3 cores — bounded by its slowest stage's per-scan time, measured.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md:36); 6290 measured float4 copy
# f64 MFMA peak (v_mfma_f64_16x16x4_f64, every SIMD issuing back to back), measured by
# tools/mfma_f64_check.hip (profiles/r04/mfma_f64.txt); the Scan Context Gram's roof
MFMA_F64_PEAK_TFLOPS = 75.2   # measured, profiles/r04/mfma_f64.txt (spec 78.6)
# MFMA flop issued per Scan Context pair (slo_scdist.h sc_gram_mfma): 4 x 4 tiles x 4 accumulators x
# ceil(NR / 16) MFMAs of 16 x 16 x 4 x 2 flop
def sc_pair_mfma_flop(nr):
    return 16 * 4 * ((nr + 15) // 16) * 16 * 16 * 4 * 2
METRIC = "scans/sec end-to-end (proj+feat+LM+SC), 64-ring 1800-col, 1/2/4/8 GPU"


def parse(argv=None):
    """the command line; `--config c2|c5` stands for that BASELINE config's arguments (EXTRA), so the profiling
    runs (tools/profile_round.sh) and the config lines measure the same workload"""
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--config" in argv:
        i = argv.index("--config")
        name = argv[i + 1]
        argv = argv[:i] + argv[i + 2:] + (EXTRA[name] if name != "c3" else [])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node: N > 1 starts N ranks (one process per GPU) unless a launcher did; "
                         "default: the launcher's WORLD_SIZE, else 1")
    ap.add_argument("--dry-dist", action="store_true",
                    help="only the rank plumbing on gloo (no GPU): launch, barrier, max-over-ranks, rank 0's JSON line")
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help="--dry-dist: this rank exits with 3 (launcher test)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--preroll", type=int, default=210,
                    help="untimed scans per stream before the warmup (fills the 50-keyframe local map)")
    ap.add_argument("--chunk", type=int, default=8, help="scans per device-generation chunk of the pre-roll")
    ap.add_argument("--streams", type=int, default=512, help="streams per GPU")
    ap.add_argument("--groups", type=int, default=3,
                    help="contexts per GPU, each on its own HIP stream and host thread (slo_amd.dist.group_slices)")
    ap.add_argument("--stagger", action="store_true",
                    help="context g runs g scans ahead (with 4 contexts each maps on its own step)")
    ap.add_argument("--preset", default="hdl64_1800")
    ap.add_argument("--keyframe-cap", type=int, default=32768,
                    help="slo_config.keyframe_cloud_cap: points per keyframe surf/outlier cloud (0 = worst case); "
                         "an overflow sets the stream's error bit, reported as stream_errors")
    ap.add_argument("--config-id", type=int, default=3)
    ap.add_argument("--voxel-order", type=int, default=0,
                    help="0: PCL's std::sort order inside a voxel (the reference's; default), 1: stable (radix sort)")
    ap.add_argument("--history", type=int, default=1000,
                    help="extra Scan Context history per stream (scans before scan 0, a KITTI-00 mid-drive history: "
                         "detects search ~1000 keyframes, SCc:264-289); the pre-roll builds the recent part")
    ap.add_argument("--profile-steps", type=int, default=8, help="instrumented steps for the per-kernel roofline")
    ap.add_argument("--roofline-also", default="fa_ring_ds,mo_knn,pc_tail,sc_detect",
                    help="further kernels timed live the same way, reported under roofline_also (comma list; each "
                         "launch of a timed kernel adds two one-thread stamp kernels to the timed steps, so the "
                         "many-launch pc_lpairs / fa_search_corner are left to kernels_algo_gbs unless named here)")
    ap.add_argument("--roofline-kernel", default="auto",
                    help="kernel timed inside the timed region (the roofline's kernel); auto = the largest kernel by "
                         "device time in the instrumented pass, which runs before the timed window")
    ap.add_argument("--cpu-scans", type=int, default=8, help="timed scans per CPU stream in the baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core in sched_getaffinity")
    ap.add_argument("--cpu-distinct", type=int, default=8,
                    help="distinct CPU streams pre-rolled in parallel; the others continue from copies of them")
    ap.add_argument("--single-steps", type=int, default=100, help="timed scans of the one-stream leg (0 = skip)")
    ap.add_argument("--no-graphs", action="store_true",
                    help="launch every kernel eagerly instead of replaying the captured per-step HIP graphs")
    ap.add_argument("--force-gather", action="store_true",
                    help="run the per-step record all-gather even at world size 1 (exercises the N>1 path)")
    ap.add_argument("--xsc-cap", type=int, default=64,
                    help="keyframes per stream in the cross-stream Scan Context store (gather mode)")
    ap.add_argument("--icp-jobs", type=int, default=64,
                    help="loop-verification ICP alignments per batch in the separate ICP measurement (0 = skip)")
    ap.add_argument("--trace-marker", action="store_true",
                    help="launch a torch spin kernel before and after the timed steps, so a rocprofv3 kernel trace of "
                         "the run can be cut to exactly the timed window (tools/trace_window.py)")
    ap.add_argument("--traffic-from", default=None,
                    help="PMC summary (tools/pmc_summary.py) for roofline.traffic; default: the newest "
                         "profiles/r*/<--profile-tag>/summary.json")
    ap.add_argument("--profile-tag", default="c3",
                    help="the config's profile directory under profiles/rNN/ (c3, c2, c5): roofline.traffic's source")
    ap.add_argument("--sc-k", type=int, default=0, help="Scan Context candidates (NUM_CANDIDATES_FROM_TREE); 0 = preset")
    ap.add_argument("--sc-off", action="store_true", help="loopClosureEnableFlag = false (C2: radius-search local map)")
    ap.add_argument("--map-keyframes", type=int, default=0, help="slo_config.map_keyframes (radius branch); 0 = default")
    ap.add_argument("--keyframe-ring", type=int, default=0, help="slo_config.keyframe_ring; 0 = default")
    ap.add_argument("--workload", default="C3 KITTI-shaped HDL-64 64x1800 stream, full pipeline + Scan Context 20x60 "
                                          "K=10, steady state")
    ap.add_argument("--window", type=int, default=0,
                    help="steps of input resident at once (0 = as many as the HBM budget allows); more steps than "
                         "that are timed in segments, each segment's scans generated untimed before it")
    ap.add_argument("--hbm-reserve-gb", type=float, default=8.0,
                    help="HBM left free after the contexts, the cross-stream store and the input window")
    ap.add_argument("--detail-out", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="side file (relative to the repo root) for the per-kernel detail the JSON line leaves out")
    ap.add_argument("--modes-steps", type=int, default=100,
                    help="timed scans of the Mode S leg (one C3 stream over the ranks, single_stream_ranks; 0 = skip)")
    ap.add_argument("--modes-leg", action="store_true",
                    help="internal: run only the Mode S leg as one rank of a launch_ranks group and print its JSON")
    ap.add_argument("--modes-transport", default="nccl", choices=("nccl", "gloo"),
                    help="the Mode S leg's point-to-point backend at N > 1: RCCL on device buffers, or gloo through "
                         "pinned host copies (the fallback when the RCCL group fails)")
    ap.add_argument("--extra", default="c2,c5,c4",
                    help="further BASELINE.json configs measured at 1 GPU after the headline, each by its own bench.py "
                         "process, reported under config_lines (outside value); 'none' = none")
    a = ap.parse_args(argv)
    if a.gpus is None:   # a launcher (torch.distributed.run) without --gpus: its world size
        a.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    return a


# BASELINE.json configs measured beside the headline (C3) at 1 GPU: bench.py arguments
EXTRA = {
    "c2": ["--profile-tag", "c2", "--preset", "os64_1800", "--config-id", "2", "--sc-off", "--streams", "512", "--map-keyframes", "32",
           "--keyframe-ring", "128", "--workload",
           "C2 Ouster-64 synthetic 64x1800 stream, segmentation + features + LM, Scan Context off (radius-search "
           "local map, MO:1167-1222), steady state"],
    "c4": ["--profile-tag", "c4", "--preset", "os1_64", "--config-id", "4", "--streams", "512", "--force-gather",
           "--workload",
           "C4 Ouster OS1-64 64x1024 streams (MulRan-shaped), full pipeline + Scan Context K=10, per-step RCCL "
           "all-gather of the pose / SC-key records into the cross-stream store (1 GPU, one-rank group), steady state"],
    "c5": ["--profile-tag", "c5", "--preset", "dense128", "--config-id", "5", "--sc-k", "50", "--streams", "128", "--keyframe-cap", "65536",
           "--workload",
           "C5 128-ring x 2048-col dense synthetic scan, Scan Context K=50, LM against the ~1M-point raw local "
           "map (HBM-bound stress), steady state"],
}


def cfg_edit(cfg, a):
    """the command line's configuration edits, for the GPU and the CPU baseline alike"""
    if a.sc_k:
        cfg.sc_num_candidates = a.sc_k
    if a.sc_off:
        cfg.loop_closure_enable = 0
    if a.map_keyframes:
        cfg.map_keyframes = a.map_keyframes
    if a.keyframe_ring:
        cfg.keyframe_ring = a.keyframe_ring


def extra_lines(a):
    """run each --extra config as its own bench.py process at 1 GPU (after this one has released the device) and
    return its JSON line, trimmed to the fields a config line needs"""
    import subprocess
    out = {}
    for name in [x for x in a.extra.split(",") if x and x != "none"]:
        cmd = [sys.executable, os.path.abspath(__file__), "--extra", "none", "--single-steps", "0", "--icp-jobs", "0",
               "--modes-steps", "0", "--steps", "12", "--warmup", "3", "--profile-steps", "4", "--cpu-scans", "4",
               "--cpu-distinct", "4", "--detail-out", detail_path(a, name), "--config", name]
        t0 = time.time()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            j = json.loads(line[-1]) if (r.returncode == 0 and line) else None
        except subprocess.TimeoutExpired:
            r, j = None, None
        if j is None:
            out[name] = {"error": f"rc={getattr(r, 'returncode', 'timeout')}",
                         "stderr_tail": (r.stderr[-600:] if r else "")}
            continue
        out[name] = j   # the child's own contract line; its per-kernel detail is in its side file
        out[name]["wall_seconds"] = round(time.time() - t0, 1)
    return out


def detail_path(a, tag=None):
    """the side file for the per-kernel detail (relative to the repo root unless absolute)"""
    p = a.detail_out if os.path.isabs(a.detail_out) else os.path.join(ROOT, a.detail_out)
    if tag:
        b, e = os.path.splitext(p)
        p = f"{b}_{tag}{e or '.json'}"
    return p


def write_detail(a, out):
    """the whole result (per-kernel times and byte rates, every roofline, the
    legs' full records) to the side file; returns its path for the line"""
    p = detail_path(a)
    try:
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            json.dump(out, f, indent=1)
        return os.path.relpath(p, ROOT)
    except OSError as e:
        print(f"bench.py: could not write {p}: {e}", file=sys.stderr)
        return None


def _pick(d, keys):
    return {k: d[k] for k in keys if k in d} if isinstance(d, dict) else d


def compact_roofline(r):
    """a roofline record without its notes: the contract's fields, the live
    launch, the isolated rate, the compulsory-bytes rate and the whole path"""
    if not isinstance(r, dict):
        return r
    o = _pick(r, ("bound", "dtype", "achieved", "peak", "unit", "frac", "traffic", "traffic_source", "kernel",
                  "avg_launch_us", "launches_timed", "bytes_per_launch", "flop_per_launch",
                  "share_of_device_time"))
    if isinstance(r.get("isolated"), dict):
        o["isolated"] = _pick(r["isolated"], ("achieved", "frac", "avg_launch_us"))
    if isinstance(r.get("compulsory"), dict):
        o["compulsory"] = _pick(r["compulsory"], ("bytes_per_launch", "achieved", "frac"))
    if isinstance(r.get("path"), dict):
        o["path"] = _pick(r["path"], ("achieved", "unit", "bytes_per_step", "frac_of_spec_8000",
                                      "frac_of_measured_copy_6290"))
    return o


def contract_line(out):
    """the one JSON line the driver parses: the contract's fields, the
    roofline and cpu_baseline, the one-stream legs' headline numbers and one
    small record per extra config; everything else stays in the side file
    (tests/test_bench_line.py bounds its size)"""
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config") if k in out}
    line["roofline"] = compact_roofline(out.get("roofline"))
    also = out.get("roofline_also") or {}
    if isinstance(also.get("sc_detect"), dict):   # north_star: MFMA utilisation of the Scan Context Gram
        line["mfma"] = compact_roofline(also["sc_detect"])
    cpu = out.get("cpu_baseline")
    if isinstance(cpu, dict):
        c = _pick(cpu, ("value", "unit", "cores", "kind", "sample", "seconds", "one_stream_scans_per_s"))
        if isinstance(cpu.get("A_reference_topology"), dict):
            c["A_reference_topology"] = _pick(cpu["A_reference_topology"], ("value", "unit", "cores",
                                                                            "stage_ms_per_scan"))
        if isinstance(cpu.get("host"), dict):
            c["host"] = _pick(cpu["host"], ("nproc", "cgroup_cpu_quota", "cpu_model", "glibc"))
        line["cpu_baseline"] = c
    else:
        line["cpu_baseline"] = cpu
    for k in ("speedup_vs_cpu", "speedup_vs_cpu_A", "stream_errors"):
        if k in out:
            line[k] = out[k]
    one = out.get("single_stream")
    if isinstance(one, dict):
        line["single_stream"] = _pick(one, ("value", "unit", "latency_ms", "err"))
    for k in ("single_stream_ctx_pipeline", "single_stream_pipelined", "single_stream_pipelined3", "single_stream_ranks"):
        v = out.get(k)
        if isinstance(v, dict):
            line[k] = _pick(v, ("value", "unit", "ranks", "contexts", "depth", "transport", "stage_ms_per_scan",
                                "owner_ms_per_scan", "bit_exact_vs_one_context", "err", "error"))
    for k in ("single_stream_speedup_vs_cpu_A", "single_stream_ctx_pipeline_speedup_vs_cpu_A",
              "single_stream_pipelined3_speedup_vs_cpu_A", "single_stream_ranks_speedup_vs_cpu_A"):
        if out.get(k) is not None:
            line[k] = out[k]
    if isinstance(out.get("hbm"), dict):
        line["hbm"] = out["hbm"]
    cl = out.get("config_lines")
    if isinstance(cl, dict):
        line["config_lines"] = {}
        for name, j in cl.items():
            if not isinstance(j, dict) or "error" in j:
                line["config_lines"][name] = j
                continue
            r = j.get("roofline") or {}
            line["config_lines"][name] = {
                "workload": (j.get("config") or {}).get("workload"), "value": j.get("value"), "unit": j.get("unit"),
                "ms_per_step": j.get("ms_per_step"), "steps": j.get("steps"),
                "roofline": _pick(r, ("kernel", "achieved", "frac", "avg_launch_us", "traffic")),
                "cpu_baseline_value": (j.get("cpu_baseline") or {}).get("value"),
                "speedup_vs_cpu": j.get("speedup_vs_cpu"), "stream_errors": j.get("stream_errors"),
                "wall_seconds": j.get("wall_seconds")}
    return line


# slo_get "counts" (csrc/slo_ctx.hip): the stream's cloud sizes in one read
CNT = ("seg_pts", "outlier", "sharp", "less_sharp", "flat", "less_flat", "lf_scan", "corner_last", "surf_last",
       "kd_corner", "kd_surf", "corner_ds", "surf_total_ds", "map_corner_ds", "map_surf_ds", "raw_ds")


def stream_counts(ctx, S):
    """Per-stream sizes of the last step (for algorithmic bytes)."""
    rows = [ctx.get(s, "counts").astype(np.int64) for s in range(S)]
    c = {n: np.array([r[i] for r in rows], np.int64) for i, n in enumerate(CNT)}
    seg = np.diff(np.array([r[len(CNT):] for r in rows], np.int64), axis=1)   # [S][R] less-flat ring segments
    c["lf_short"] = np.where(seg <= 512, seg, 0).sum(axis=1)   # x-sorted by k_fa_sx_rings (one wave per ring)
    c["lf_long"] = np.where(seg > 512, seg, 0).sum(axis=1)     # by k_fa_sx_long
    c["fa_iters"] = np.array([ctx.get(s, "fa_iters") for s in range(S)], np.int64)
    c["vg_in"] = np.array([ctx.get(s, "vg_in") for s in range(S)], np.int64)   # [S][7] VoxelGrid items
    c["mo_iters"] = np.array([int(ctx.get(s, "mo_iters")[0]) for s in range(S)], np.int64)
    c["map_raw_n"] = np.array([ctx.get(s, "map_raw_n") for s in range(S)], np.int64)   # [S][2] before the VoxelGrids
    c["n_keyframes"] = np.array([int(ctx.get(s, "n_keyframes")[0]) for s in range(S)], np.int64)
    return c


def path_bytes(c, cfg, history):
    """SURVEY §8(d)'s algorithmic bytes of the whole path, from the logged
    per-stream counts: (every scan, summed over streams; a mapping step adds,
    summed over streams) — projection 16P + 24H, ground + labels 32 C gsi +
    9H, components 20H, compaction 25H + 25S, deskew / curvature / occlusion
    48S, feature selection + DS 25S + 16 (F_s + F_ls + F_f + F_lf), odometry
    LM 64 per query-iteration; map build 16 M_raw + 16 M, mapping LM 96 per
    query-iteration, Scan Context 16 P_ds + 9.6 KB + the detect 80 L + K 10.1 KB."""
    P, H, C = cfg.max_points, cfg.n_scan * cfg.horizon_scan, cfg.horizon_scan
    gsi = cfg.ground_scan_ind + 1
    seg = c["seg_pts"]
    front = (16 * P + 24 * H + 32 * C * gsi + 9 * H + 20 * H + 25 * H + 25 * seg + 48 * seg + 25 * seg
             + 16 * (c["sharp"] + c["corner_last"] + c["flat"] + c["surf_last"])
             + 64 * (c["fa_iters"][:, 0] * c["flat"] + c["fa_iters"][:, 1] * c["sharp"]))
    L = np.maximum(c["n_keyframes"] + history - cfg.sc_num_exclude_recent, 0)
    mapping = (16 * c["map_raw_n"].sum(axis=1) + 16 * (c["map_corner_ds"] + c["map_surf_ds"])
               + 96 * c["mo_iters"] * (c["corner_ds"] + c["surf_total_ds"])
               + 16 * c["raw_ds"] + 9600 + 80 * L + cfg.sc_num_candidates * 10100)
    return int(front.sum()), int(mapping.sum())


def algo_bytes(name, c, cfg, S, steps, map_steps):
    """Algorithmic HBM bytes of ALL launches of `name` in the profiled window
    (SURVEY §8(d) per-unit figures; points are 16 B; DESIGN.md §4 lists each
    model).  The per-stream sizes are the last instrumented step's (`c`, from
    stream_counts); per-scan kernels count `steps` scans of every stream, the
    mapping step's `map_steps`.  Cumulative device counters (pcl_work, the
    long-voxel and Scan Context work) are exact deltas over the window.
    None = not priced (kernels under 1 % of device time in every config)."""
    H = cfg.n_scan * cfg.horizon_scan
    P = cfg.max_points
    tot = lambda x: int(np.asarray(x).sum())  # noqa: E731
    per_scan = lambda x: steps * tot(x)        # noqa: E731
    per_map = lambda x: map_steps * tot(x)     # noqa: E731
    seg, outl = c["seg_pts"], c["outlier"]
    # ---- imageProjection (IP:199-460), per scan
    if name == "ip_init":         # the owner image reset
        return steps * S * H * 4
    if name == "ip_project":      # read the point, scatter a 4 B owner
        return steps * S * P * (16 + 4)
    if name == "ip_tile":         # per pixel: owner in, its point in (every pixel counted: an upper bound on the
        # owned ones), range / full cloud / ground / label / parent / csize out
        return steps * S * H * (4 + 16 + 4 + 16 + 1 + 4 + 4 + 4)
    if name == "ip_cc_stats":     # per pixel: parent and csize in
        return steps * S * H * 8
    if name == "ip_rowcount":     # per pixel: label and ground in, the final label out
        return steps * S * H * 9
    if name == "ip_compact":      # per pixel: label, ground, range in; per kept point 25 B out (point, ground
        # flag, column, range), per outlier 16 B
        return steps * (S * H * 9) + per_scan(25 * seg + 16 * outl)
    # ---- featureAssociation (FA:491-784, 1044-1815), per scan
    if name == "fa_halfpass":     # the segmented point
        return per_scan(16 * seg)
    if name == "fa_points":       # point, range, column in; deskewed point, curvature, label, smoothness, picked out
        return per_scan(seg * (16 + 4 + 4 + 16 + 4 + 4 + 8 + 4))
    if name == "fa_sort":         # smoothness in/out, curvature, ground flag, candidate list out
        return per_scan(seg * (8 + 8 + 4 + 1 + 2))
    if name == "fa_pick":         # picked, label in/out, column, candidates, points of the outputs
        return per_scan(seg * (4 + 4 + 4 + 4 + 4 + 2 + 16))
    if name == "fa_ring_ds":      # FA:779-780: each ring's less-flat points in, their VoxelGrid centroids out
        return per_scan(16 * c["lf_scan"] + 16 * c["less_flat"])
    if name == "fa_gather":       # the four feature clouds, per-ring slabs in, concatenated out
        return per_scan(32 * (c["sharp"] + c["less_sharp"] + c["flat"] + c["less_flat"]))
    if name == "fa_odo_begin":    # the sharp points in, their x order out
        return per_scan(20 * c["sharp"])
    srch = lambda it: (it + 4) // 5  # noqa: E731  search iterations actually run
    if name == "fa_search_surf":  # per search: queries + 3 indices, the target cloud once
        return steps * int((srch(c["fa_iters"][:, 0]) * (c["flat"] * 28 + c["surf_last"] * 16)).sum())
    if name == "fa_search_corner":  # per search: queries + 2 indices, the target cloud once
        return steps * int((srch(c["fa_iters"][:, 1]) * (c["sharp"] * 24 + c["corner_last"] * 16)).sum())
    if name == "fa_iter_surf":    # per iteration: query + 3 indices + 3 matched points
        return steps * int((c["fa_iters"][:, 0] * c["flat"] * (16 + 12 + 48)).sum())
    if name == "fa_iter_corner":
        return steps * int((c["fa_iters"][:, 1] * c["sharp"] * (16 + 8 + 32)).sum())
    if name == "fa_to_end":       # TransformToEnd: less sharp / less flat in, *_next and the tree copies out
        return per_scan(48 * (c["less_sharp"] + c["less_flat"]))
    if name == "fa_sx_rings":     # x-sort of the rings of <= 512 less-flat points: point in, (point, index) out
        return per_scan(32 * c["lf_short"])
    if name == "fa_sx_long":      # the longer rings
        return per_scan(32 * c["lf_long"])
    if name == "fa_sx_kd":        # the corner tree cloud, x-sorted
        return per_scan(32 * c["kd_corner"])
    if name == "grid_build_lds":  # the odometry surf grid (T = 2^15 buckets): point in, entry out, offsets out
        return per_scan(32 * c["kd_surf"]) + steps * S * 4 * ((1 << 15) + 1)
    # ---- mapOptimization (MO:1122-1522), per mapping step
    if name == "mo_prepare":      # adjustOutlierCloud (outliers in and out); the radius branch reads the key poses
        return per_map(32 * outl + (0 if cfg.loop_closure_enable else 24 * c["n_keyframes"]))
    if name == "mo_assemble":     # the local map's keyframe clouds in (body frame), transformed out
        return per_map(32 * c["map_raw_n"])
    if name == "mo_concat":       # surf DS + outlier DS into the surf-total cloud
        return per_map(32 * c["surf_total_ds"])
    if name == "grid_count":      # the two map grids: point in, bucket count read-modify-write
        return per_map(24 * (c["map_corner_ds"] + c["map_surf_ds"]))
    if name == "grid_scan":       # every bucket's count in, offset out (2^19 + 1 buckets, two grids)
        return map_steps * S * 2 * ((1 << 19) + 1) * 8
    if name == "grid_scatter":    # point in, bucket offset in, count read-modify-write, entry out
        return per_map(44 * (c["map_corner_ds"] + c["map_surf_ds"]))
    if name == "mo_corr":         # per iteration: query + 5 neighbour indices + 5 neighbours
        per = (c["corner_ds"] + c["surf_total_ds"]) * (16 + 20 + 80)
        return map_steps * int((c["mo_iters"] * per).sum())
    if name == "mo_knn":          # per iteration: query + 5 neighbour indices out, the map clouds once
        per = (c["corner_ds"] + c["surf_total_ds"]) * (16 + 20) + (c["map_corner_ds"] + c["map_surf_ds"]) * 16
        return map_steps * int((c["mo_iters"] * per).sum())
    # ---- the mapping step's batched VoxelGrids (MO:1224-1263)
    vin = per_map(c["vg_in"]) if "vg_in" in c else 0
    if name == "vg_bounds":       # every input point once
        return 16 * vin
    if name == "vg_heads":        # the sorted keys
        return 4 * vin
    if name == "vg_reduce":       # sorted (key, index) in, the point gathered, per item
        return vin * (8 + 16)
    if name == "vg_long" and c.get("long_items") is not None:   # long voxels: index + point per item, centroid out
        return int(20 * c["long_items"] + 16 * c["long_voxels"])
    if name in ("vg_scatter", "vg_onesweep"):   # the stable radix sort: 4 passes, pass 0 reads the point (16 B)
        # and writes (key, index) 8 B, passes 1-3 read and write 8 B
        return vin * (16 + 8 + 3 * 16)
    if name == "vg_ghist":        # every pass's digit counts from one read of the points
        return vin * 16
    if name == "vg_hist":         # pass 0 reads the point, passes 1-3 the 4 B key
        return vin * (16 + 3 * 4)
    pw = c.get("pcl_work")        # PCL-order sort work counters over the instrumented pass (slo_vgpcl.hip PW_*)
    if pw is not None:
        if name == "pc_lcount":   # the keys of every stepped range
            return int(4 * pw[0])
        if name == "pc_lrank":    # the keys again, the pair positions out
            return int(4 * pw[0] + 8 * pw[1])
        if name == "pc_lpairs":   # per pair: both positions in, both items (key + index) read and written
            return int(40 * pw[1])
        if name in ("pc_finish_w", "pc_finish_s", "pc_finish_b"):   # a finish entry's items in and out
            b = int(16 * pw[2 + ("pc_finish_w", "pc_finish_s", "pc_finish_b").index(name)])
            if name == "pc_finish_b":   # + the spent-depth heapsorts it runs first (PW_FALL; std::sort's heapsort):
                b += int(32 * pw[21])   # each item in, to the 8-B scratch, back, out
            return b
        if name == "pc_finish_bx":   # the 4 Ki entries too wide for 32-bit items (PW_FINX)
            return int(16 * pw[20])
        if name == "pc_tail":     # per stepped item: its key counted (4 B) and read again on its side of the
            # crossing (4 B) plus the left side's index (4 B); per pair: partner position out and in, both
            # items read and written
            return int(12 * pw[7] + 40 * pw[8])
        if name == "pc_count":    # the points
            return int(16 * pw[5])
        if name == "pc_write":    # the points in, (key, index) out
            return int(24 * pw[5])
    if name == "sc_detect" and c.get("sc_pairs") is not None:   # MFMA flop (bound "mfma")
        return int(c["sc_pairs"]) * sc_pair_mfma_flop(cfg.sc_num_ring)
    return None


PCL_SORT_FAMILY = ("pc_count", "pc_write", "pc_lcount", "pc_lrank", "pc_lpairs", "pc_lscan", "pc_lsplit", "pc_tail",
                   "pc_finish_w", "pc_finish_s", "pc_finish_b", "pc_finish_bx", "vg_reduce")


def compulsory_bytes(name, c):
    """SURVEY §8(d) compulsory bytes of the PCL-order VoxelGrid family over the
    instrumented window: every filter input point read once (16 B); the
    implementation's own passes (algo_bytes) come on top.  None outside the
    family or without the work counters."""
    pw = c.get("pcl_work") if c else None
    if name not in PCL_SORT_FAMILY or pw is None or not int(pw[5]):
        return None
    return int(16 * pw[5])


def pmc_traffic(path, kernel, tag=None):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary
    (FETCH_SIZE x2 x1024 + WRITE_SIZE x1024, MI355X_MICROARCH.md), or None.
    Default source: the newest round's profile of this config
    (profiles/rNN[a-z]/<tag>/summary.json, tag = c3 / c2 / c5), else the newest
    round-level profile (profiles/rNN[a-z]/summary.json, C3 only)."""
    import glob
    import re
    if path is None:
        pats = ([(os.path.join(ROOT, "profiles", "r*", tag, "summary.json"),
                  r"profiles/r(\d+)([a-z]?)/" + tag + r"/summary\.json$")] if tag else [])
        if tag in (None, "c3"):
            pats.append((os.path.join(ROOT, "profiles", "r*", "summary.json"), r"profiles/r(\d+)([a-z]?)/summary\.json$"))
        for pat, rx in pats:
            cands = [((int(m.group(1)), m.group(2)), p) for p in glob.glob(pat) for m in [re.search(rx, p)] if m]
            if cands:
                path = max(cands)[1]
                break
    if path is None or not os.path.exists(path):
        return None, None
    k = json.load(open(path))["kernels"].get(kernel)
    if not k or not k.get("hbm_bytes_per_launch"):
        return None, os.path.relpath(path, ROOT)
    return k["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)


def icp_bench(torch, slo_amd, pid, a, local, gthreads, reps=3):
    """ICP alignments/s of slo_icp_align_batch + the lc_corr kernel's roofline."""
    import numpy as np
    J = a.icp_jobs
    cfg = slo_amd.preset(a.preset)
    cfg.loop_verify = 1
    P = cfg.max_points
    raw = slo_amd.gen_batch(pid, a.config_id, 0, J, 0, 1, P, gthreads)[0]   # [J][P][4]
    fin = np.isfinite(raw[..., :3]).all(axis=2)
    srcs, tgts = [], []
    rng = np.random.default_rng(5)
    for j in range(J):
        pts = raw[j][fin[j]]
        tgt = pts[::4]
        src = pts[::16].copy()
        yaw, t = rng.uniform(-0.02, 0.02), rng.uniform(-0.3, 0.3, size=3).astype(np.float32)
        c, s_ = np.float32(np.cos(yaw)), np.float32(np.sin(yaw))
        x, y = src[:, 0].copy(), src[:, 1].copy()
        src[:, 0], src[:, 1], src[:, 2] = c * x - s_ * y + t[0], s_ * x + c * y + t[1], src[:, 2] + t[2]
        srcs.append(src)
        tgts.append(tgt)
    ss, ts = max(len(x) for x in srcs), max(len(x) for x in tgts)
    cfg.loop_archive_points = int(ts)
    hs = np.zeros((J, ss, 4), np.float32)
    ht = np.zeros((J, ts, 4), np.float32)
    for j in range(J):
        hs[j, :len(srcs[j])] = srcs[j]
        ht[j, :len(tgts[j])] = tgts[j]
    dsrc, dtgt = torch.from_numpy(hs).cuda(local), torch.from_numpy(ht).cuda(local)
    ns = torch.tensor([len(x) for x in srcs], dtype=torch.int32, device=f"cuda:{local}")
    nt = torch.tensor([len(x) for x in tgts], dtype=torch.int32, device=f"cuda:{local}")
    ctx = slo_amd.Context(cfg, local, J)
    run = lambda: ctx.icp_align_batch(dsrc.data_ptr(), ss, ns.data_ptr(), dtgt.data_ptr(), ts, nt.data_ptr())  # noqa: E731
    res = run()   # warm-up
    t0 = time.perf_counter()
    for _ in range(reps):
        res = run()
    el = (time.perf_counter() - t0) / reps
    ctx.timing(True)
    ctx.timing_reset()
    res = run()
    kt = ctx.timing_read()
    ctx.timing(False)
    ctx.close()
    iters = res["iters"].astype(np.int64)
    nsrc = np.array([len(x) for x in srcs], np.int64)
    ntgt = np.array([len(x) for x in tgts], np.int64)
    ms, n = kt.get("lc_corr", (0.0, 0))
    # per launch: every live job reads its query and writes it back moved
    # (16 + 16 B) plus the correspondence (8 B); the target once (16 B / point)
    b = int(((nsrc * 40 + ntgt * 16) * iters).sum())
    ach = b / (ms / 1e3) / 1e9 if ms > 0 else None
    return {"metric": "ICP alignments/s (pcl::IterativeClosestPoint::align + getFitnessScore, max 100 iterations)",
            "value": round(J / el, 2), "jobs": J, "ms_per_batch": round(el * 1e3, 3),
            "source_points_mean": round(float(nsrc.mean()), 1), "target_points_mean": round(float(ntgt.mean()), 1),
            "iterations_mean": round(float(iters.mean()), 2), "accepted": int(res["accepted"].sum()),
            "roofline": {"bound": "hbm", "kernel": "lc_corr", "achieved": round(ach, 2) if ach else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5) if ach else None,
                         "avg_launch_us": round(ms / max(1, n) * 1e3, 2), "launches": int(n)},
            "kernels_ms": {k: [round(v[0], 3), int(v[1])] for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])}}


def host_info():
    """nproc, cores this process may run on, cgroup CPU quota, CPU model, glibc"""
    import platform
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cores"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity_cores"] = os.cpu_count()
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        info["cgroup_cpu_quota"] = None
    try:
        info["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        info["cpu_model"] = platform.processor() or None
    try:
        info["glibc"] = os.confstr("CS_GNU_LIBC_VERSION")
    except Exception:
        info["glibc"] = " ".join(platform.libc_ver())
    return info


def cpu_baseline(a, pid, ncpu, start):
    """SURVEY §8(d) CPU baselines on the oracle (C++ restatement, g++ -O2), same window as the GPU
    (scans from `start`); (B) runs one stream per core this process can actually use: min(affinity, the
    cgroup CPU quota)"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes
    import oracle_py as O
    info = host_info()
    quota = info.get("cgroup_cpu_quota")
    eff = max(1, min(ncpu, int(quota))) if quota else ncpu
    th = a.cpu_threads or eff
    stage = (ctypes.c_double * 4)()
    one = (ctypes.c_double * 4)()
    ocfg = O.preset(pid)
    cfg_edit(ocfg, a)
    t0 = time.time()
    secs = O.lib().oracle_bench_cfg(ctypes.byref(ocfg), a.config_id, th, a.cpu_scans, start, a.history,
                                    min(a.cpu_distinct, th), stage, one)
    wall = time.time() - t0
    n = a.cpu_scans
    # (A): one stream as the reference's 3 processes on 3 cores; the pipeline
    # runs at the pace of its slowest stage (mapOptimization includes SC)
    per = {"ip": one[0] / n, "fa": one[1] / n, "mo_sc": (one[2] + one[3]) / n}
    a_val = 1.0 / max(per.values())
    return {"value": round(th * n / secs, 3), "unit": "scans/s", "cores": th, "affinity_cores": ncpu, "kind": "port",
            "sample": f"(B) {th} independent {a.preset} streams, one per usable core (min of sched_getaffinity "
                      f"{ncpu} and the cgroup CPU quota {quota}), each timed over "
                      f"scans {start}..{start + n - 1} after an untimed pre-roll "
                      f"(the GPU's steady-state window); {min(a.cpu_distinct, th)} streams pre-rolled, the rest "
                      f"continue from copies; oracle/ C++ restatement g++ -O2",
            "seconds": round(secs, 2), "wall_seconds_incl_preroll": round(wall, 1),
            "one_stream_scans_per_s": round(n / sum(one), 3),
            "stage_seconds": {"ip": round(stage[0], 2), "fa": round(stage[1], 2), "mo": round(stage[2], 2),
                              "sc": round(stage[3], 2)},
            "A_reference_topology": {"value": round(a_val, 3), "unit": "scans/s", "cores": 3,
                                     "stage_ms_per_scan": {k: round(v * 1e3, 3) for k, v in per.items()},
                                     "note": "one stream, imageProjection | featureAssociation | mapOptimization "
                                             "(launch/run.launch:14-17) on 3 cores: 1 / slowest stage's measured "
                                             "per-scan time"},
            "host": info}


def single_stream(torch, slo_amd, a, cfg, pid, local):
    """one C3 stream through the same pipeline: scans/s (async) and per-scan latency (synchronised)"""
    P = cfg.max_points
    ctx = slo_amd.Context(cfg, local, 1)
    ctx.graph_mode(not a.no_graphs)
    gen = slo_amd.DeviceGenerator(pid, a.config_id, 0, 1, local)
    n = a.preroll + a.warmup + a.single_steps
    try:
        buf = torch.empty((n, 1, P, 4), dtype=torch.float32, device=f"cuda:{local}")
        gen.scans(0, n, buf.data_ptr())
        cnt = torch.full((1,), P, dtype=torch.int32, device=f"cuda:{local}")
        k0 = a.preroll + a.warmup
        for k in range(k0):
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ctx.synchronize()
        half = a.single_steps // 2
        t0 = time.perf_counter()
        for k in range(k0, k0 + half):    # back to back: launch overlap, the stream's throughput
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ctx.synchronize()
        thr = half / (time.perf_counter() - t0)
        lat = []
        for k in range(k0 + half, k0 + a.single_steps):   # one at a time: the latency of a scan
            t1 = time.perf_counter()
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            ctx.synchronize()
            lat.append(time.perf_counter() - t1)
        lat = np.array(lat) * 1e3
        kf = int(ctx.get(0, "n_keyframes")[0])
        state = {nm: ctx.get(0, nm).copy() for nm in MODES_STATE}
        return {"value": round(thr, 2), "unit": "scans/s", "streams": 1, "scans_timed": half,
                "latency_ms": {"mean": round(float(lat.mean()), 3), "p50": round(float(np.median(lat)), 3),
                               "p99": round(float(np.percentile(lat, 99)), 3), "scans": len(lat)},
                "keyframes_at_end": kf, "err": int(ctx.get(0, "err")[0])}, state
    finally:
        gen.close()
        ctx.close()


def single_stream_ctx_pipeline(torch, slo_amd, a, cfg, pid, local, ref_state, depth=6):
    """one C3 stream in ONE context with slo_pipeline: its front end, odometry
    and mapping stage on three HIP streams of the context (the reference's
    three processes), the host only enqueuing slo_batch_process calls; the
    scans of single_stream, the last half timed back to back, the final state
    compared bit for bit with single_stream's plain context"""
    P = cfg.max_points
    ctx = slo_amd.Context(cfg, local, 1)
    ctx.pipeline(depth)
    gen = slo_amd.DeviceGenerator(pid, a.config_id, 0, 1, local)
    n = a.preroll + a.warmup + a.single_steps
    try:
        buf = torch.empty((n, 1, P, 4), dtype=torch.float32, device=f"cuda:{local}")
        gen.scans(0, n, buf.data_ptr())
        cnt = torch.full((1,), P, dtype=torch.int32, device=f"cuda:{local}")
        k0 = a.preroll + a.warmup + a.single_steps // 2
        for k in range(k0):
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ctx.synchronize()
        t0 = time.perf_counter()
        for k in range(k0, n):
            ctx.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
        ctx.synchronize()
        el = time.perf_counter() - t0
        got = {nm: ctx.get(0, nm) for nm in MODES_STATE}
        same = ref_state is not None and all(
            ref_state[nm].shape == got[nm].shape and np.array_equal(ref_state[nm].view(np.uint8), got[nm].view(np.uint8))
            for nm in MODES_STATE)
        return {"value": round((n - k0) / el, 2), "unit": "scans/s", "streams": 1, "contexts": 1, "depth": depth,
                "scans_timed": n - k0, "bit_exact_vs_one_context": bool(same), "err": int(got["err"][0]),
                "note": "one context, slo_pipeline: front end | odometry | mapping + Scan Context on three HIP streams"}
    finally:
        gen.close()
        ctx.close()


def single_stream_pipelined(torch, slo_amd, a, cfg, pid, local, stages=2):
    """one C3 stream as Mode S on one GPU, each stage on its own context, HIP
    stream and host thread — the reference's own process split
    (launch/run.launch:14-17).  stages=2 (slo_amd.modes.run_pipelined_slo): a
    front context (imageProjection + feature extraction) and the owner
    (odometry, mapping, Scan Context), scan k + 1's front end beside scan k's
    back end.  stages=3 (run_pipelined3_slo): the back end split into
    odometry | mapping + transformFusion + Scan Context.  Same results as the
    one-context leg (tests/test_gpu_modes.py)."""
    from slo_amd import modes
    P = cfg.max_points
    eng = modes.SloEngine(cfg, fronts=1, device=local, split_back=stages == 3)
    run = modes.run_pipelined3_slo if stages == 3 else modes.run_pipelined_slo
    gen = slo_amd.DeviceGenerator(pid, a.config_id, 0, 1, local)
    n = a.preroll + a.warmup + a.single_steps
    try:
        buf = torch.empty((n, 1, P, 4), dtype=torch.float32, device=f"cuda:{local}")
        gen.scans(0, n, buf.data_ptr())
        cnt = torch.full((1,), P, dtype=torch.int32, device=f"cuda:{local}")
        ptr = [buf[k].data_ptr() for k in range(n)]
        tim = [0.1 * k for k in range(n)]
        k0 = a.preroll + a.warmup
        run(eng, 1, ptr[:k0], cnt.data_ptr(), tim[:k0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = run(eng, 1, ptr[k0:], cnt.data_ptr(), tim[k0:])
        el = time.perf_counter() - t0
        m = n - k0
        names = ("front", "odometry", "mapping") if stages == 3 else ("front", "back")
        return {"value": round(m / el, 2), "unit": "scans/s", "streams": 1, "scans_timed": m,
                "stage_ms_per_scan": {k: round(t / m * 1e3, 3) for k, t in zip(names, ts)},
                "keyframes_at_end": int(eng.owner.get(0, "n_keyframes")[0]),
                "err": int(eng.owner.get(0, "err")[0]) | int(eng.fronts[0].get(0, "err")[0]),
                "note": ("Mode S on one GPU: front | odometry | mapping contexts pipelined (three host threads)"
                         if stages == 3 else "Mode S on one GPU: front context and owner pipelined (two host threads)")}
    finally:
        gen.close()
        eng.close()


MODES_STATE = ("transform_sum", "integrated", "mapped", "keyposes", "n_keyframes", "ring_key", "err")


def modes_leg_run(torch, slo_amd, a, cfg, pid, local, engine, rank, world, transport):
    """one C3 stream through modes.run_rank (world 2) or run_rank3 (world >= 3):
    scans [0, preroll + warmup + modes_steps) generated on this rank's device,
    the owner (rank 0) timing the last modes_steps back ends; then rank 0 runs
    the same scans through one context and compares the owner's final state
    and every scan's flags bit for bit.  Returns rank 0's record (None on the
    other ranks)."""
    from slo_amd import modes
    P = cfg.max_points
    n = a.preroll + a.warmup + a.modes_steps
    k0 = a.preroll + a.warmup
    gen = slo_amd.DeviceGenerator(pid, a.config_id, 0, 1, local)
    buf = torch.empty((n, 1, P, 4), dtype=torch.float32, device=f"cuda:{local}")
    gen.scans(0, n, buf.data_ptr())
    gen.close()
    cnt = torch.full((1,), P, dtype=torch.int32, device=f"cuda:{local}")
    torch.cuda.synchronize()
    stamps = {}

    def on_back(k, fl):
        if k in (k0 - 1, n - 1):
            stamps[k] = time.perf_counter()

    run = modes.run_rank3 if world >= 3 else modes.run_rank
    flags = run(engine, rank, world, lambda k: ((buf[k].data_ptr(), cnt.data_ptr()), 0.1 * k), n, transport,
                on_back=on_back if rank == 0 else None)
    if rank != 0:
        return None
    el = stamps[n - 1] - stamps[k0 - 1]
    got = {nm: engine.owner.get(0, nm).copy() for nm in MODES_STATE}
    one = slo_amd.Context(cfg, local, 1)
    try:
        ref_flags = []
        for k in range(n):
            one.batch_process(buf[k].data_ptr(), cnt.data_ptr(), 0.1 * k)
            ref_flags.append(int(one.get(0, "flags")[0]))
        ref = {nm: one.get(0, nm).copy() for nm in MODES_STATE}
    finally:
        one.close()
    same = ref_flags == list(flags) and all(
        ref[nm].shape == got[nm].shape and np.array_equal(ref[nm].view(np.uint8), got[nm].view(np.uint8))
        for nm in MODES_STATE)
    return {"value": round(a.modes_steps / el, 2), "unit": "scans/s", "ranks": world, "streams": 1,
            "scans_timed": a.modes_steps, "owner_ms_per_scan": round(el / a.modes_steps * 1e3, 3),
            "bit_exact_vs_one_context": bool(same), "keyframes_at_end": int(got["n_keyframes"][0]),
            "err": int(got["err"][0]),
            "layout": ("rank 0 mapping + Scan Context (owner), rank 1 odometry, ranks 2.. front ends in turn "
                       "(modes.run_rank3)" if world >= 3 else
                       "front ends on ranks 0 and 1 in turn, back end on rank 0 (modes.run_rank)")}


def modes_leg_local(torch, slo_amd, a, cfg, pid, local, world=3):
    """Mode S at N = 1: the ranks of run_rank3 as threads of this process on
    one GPU, the carry / features / odometry buffers moved by LocalTransport"""
    import threading
    from slo_amd import modes
    engs = [modes.SloEngine.for_rank(cfg, r, world, split_back=True, device=local, read_flags=r == 0)
            for r in range(world)]
    tr = modes.LocalTransport.group(world)
    res, errs = {}, []

    def go(r):
        try:
            res[r] = modes_leg_run(torch, slo_amd, a, cfg, pid, local, engs[r], r, world, tr[r])
        except BaseException as e:   # noqa: BLE001
            errs.append(f"rank {r}: {e!r}")
            for q in tr:   # the others' receives time out instead of waiting forever
                q.timeout = 1.0

    try:
        ths = [threading.Thread(target=go, args=(r,)) for r in range(world)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    finally:
        for e in engs:
            e.close()
    if errs or res.get(0) is None:
        return {"error": "; ".join(errs)[:400] or "no result"}
    out = res[0]
    out["transport"] = "LocalTransport: 3 ranks as threads on 1 GPU"
    return out


def modes_leg_launch(a, world, timeout_s=(150, 120)):
    """Mode S at N > 1: a fresh group of `world` processes, one per GPU
    (bench.py --modes-leg, slo_amd.dist.launch_ranks), the buffers moved by
    RCCL point-to-point (modes.DistTransport); rank 0's JSON record, or the
    failure"""
    import tempfile
    from slo_amd import dist as sdist
    argv = ["--modes-leg", "--gpus", str(world), "--preset", a.preset, "--config-id", str(a.config_id),
            "--preroll", str(a.preroll), "--warmup", str(a.warmup), "--modes-steps", str(a.modes_steps)]
    if a.sc_k:
        argv += ["--sc-k", str(a.sc_k)]
    if a.sc_off:
        argv.append("--sc-off")
    failed = None
    # RCCL first; gloo through host copies if the RCCL group fails.  The leg
    # takes ~40 s (process start, group init, 310 scans, the one-context
    # replay); the limits keep a hung group from costing the bench its line
    for tr, lim in zip(("nccl", "gloo"), timeout_s):
        with tempfile.TemporaryFile("w+") as f:
            rc = sdist.launch_ranks(world, argv + ["--modes-transport", tr], os.path.abspath(__file__), stdout=f,
                                    timeout_s=lim)
            f.seek(0)
            lines = [x for x in f.read().splitlines() if x.startswith("{")]
        if rc == 0 and lines:
            out = json.loads(lines[-1])
            out["transport"] = (f"RCCL point-to-point over {world} GPUs (modes.DistTransport)" if tr == "nccl" else
                                f"gloo point-to-point over {world} GPUs through pinned host copies (modes.HostTransport)")
            if failed:
                out["rccl_error"] = failed
            return out
        failed = f"{tr} ranks exited with {rc}"
    return {"error": failed, "ranks": world}


def modes_leg_rank(a):
    """bench.py --modes-leg: this process is one rank of the Mode S group"""
    import torch
    import torch.distributed as dist
    import slo_amd
    from slo_amd import dist as sdist
    from slo_amd import modes
    rank, world, local = sdist.env_rank()
    if a.modes_transport == "gloo":   # host-staged messages: ranks may share a GPU (the 1-GPU rehearsal)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if a.modes_transport == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    try:
        cfg = slo_amd.preset(a.preset)
        cfg_edit(cfg, a)
        pid = slo_amd.PRESETS[a.preset]
        eng = modes.SloEngine.for_rank(cfg, rank, world, split_back=world >= 3, device=local, read_flags=rank == 0)
        try:
            dist.barrier()
            tr = modes.DistTransport() if a.modes_transport == "nccl" else modes.HostTransport()
            rec = modes_leg_run(torch, slo_amd, a, cfg, pid, local, eng, rank, world, tr)
            dist.barrier()
        finally:
            eng.close()
        if rank == 0:
            print(json.dumps(rec), flush=True)
    finally:
        dist.destroy_process_group()


def dry_dist(a, rank, world):
    """--dry-dist: the multi-rank plumbing alone on gloo (no GPU): every rank
    takes part in a barrier and the max-over-ranks timing, and rank 0 prints
    the contract's JSON line with n_gpus = the world size
    (tests/test_bench_launch.py runs `bench.py --gpus 2 --dry-dist`)"""
    import torch.distributed as dist
    from slo_amd import dist as sdist
    if rank == a.dry_fail_rank:   # the launcher must stop the ranks left waiting for this one
        sys.exit(3)
    dist.init_process_group("gloo")
    try:
        dist.barrier()
        el = sdist.max_over_ranks(0.01 * (rank + 1))
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "scans/s", "n_gpus": world, "steps": a.steps,
                              "warmup": a.warmup, "ms_per_step": round(el * 1e3, 3), "dry_dist": True,
                              "ranks_seen": world}), flush=True)
    finally:
        dist.destroy_process_group()


def main():
    a = parse()
    from slo_amd import dist as sdist
    if a.gpus > 1 and "RANK" not in os.environ:
        # one process per GPU (the driver may also start them itself with
        # torch.distributed.run): nothing here has touched a GPU yet
        sys.exit(sdist.launch_ranks(a.gpus, sys.argv[1:], os.path.abspath(__file__)))
    rank, world, local = sdist.env_rank()
    if world != a.gpus and not (a.gpus == 1 and a.force_gather):
        print(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    if a.dry_dist:
        dry_dist(a, rank, world)
        return
    if a.modes_leg:
        modes_leg_rank(a)
        return
    import torch
    import torch.distributed as dist
    import slo_amd
    from slo_amd import budget

    torch.cuda.set_device(local)
    gather = world > 1 or a.force_gather
    if gather:
        if "RANK" not in os.environ:   # --force-gather outside torch.distributed.run: a 1-rank group
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = slo_amd.preset(a.preset)
    cfg.keyframe_cloud_cap = a.keyframe_cap
    cfg.voxel_order = a.voxel_order
    cfg_edit(cfg, a)
    pid = slo_amd.PRESETS[a.preset]
    P = cfg.max_points
    S = a.streams
    try:
        ncpu = len(os.sched_getaffinity(0))
    except Exception:
        ncpu = os.cpu_count() or 8
    gthreads = max(1, min(16, ncpu))

    # ---- contexts, then the resident window [preroll, preroll + warmup + steps + profile)
    t_gen = time.time()
    stream0, _ = sdist.stream_shard(rank, world, S)
    groups = sdist.group_slices(S, a.groups)
    free0 = torch.cuda.mem_get_info(local)[0]
    ctxs = [slo_amd.Context(cfg, local, n) for _, n in groups]
    for c in ctxs:
        c.graph_mode(not a.no_graphs)
        c.prepare_mapping()   # the mapping workspaces now, so the budget below sees them
    ctx_bytes = free0 - torch.cuda.mem_get_info(local)[0]
    n_ctx = len(ctxs)
    # --stagger: context g runs lag(g) = g scans ahead, so with as many
    # contexts as the mapping period the contexts map on different steps
    lag = (lambda g: g) if a.stagger else (lambda g: 0)
    maxlag = max(lag(g) for g in range(len(groups)))
    total = a.profile_steps + a.warmup + a.steps
    # HBM budget (slo_amd.budget): the cross-stream store first, then as many
    # steps of resident input as fit beside it with --hbm-reserve-gb left free
    xsc_b = budget.xsc_bytes(world * S, a.xsc_cap, cfg.sc_num_ring, cfg.sc_num_sector) if gather else 0
    free_ctx = torch.cuda.mem_get_info(local)[0]
    step_b = budget.step_bytes(S, P)
    try:
        wscans = budget.window_scans(free_ctx, step_b, max(total, a.chunk), maxlag, xsc_b,
                                     int(a.hbm_reserve_gb * budget.GIB), a.window)
    except MemoryError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(4)
    seg_len = wscans - maxlag   # steps per timed segment
    xsc, matches = None, None
    if gather:   # cross-stream Scan Context store over every rank's streams
        from slo_amd import xsc as X
        xsc = X.CrossSession(cfg, world * S, a.xsc_cap, local)
        matches = torch.zeros((S, X.MATCH_DTYPE.itemsize // 4), dtype=torch.int32, device=f"cuda:{local}")
    dev = torch.empty((wscans, S, P, 4), dtype=torch.float32, device=f"cuda:{local}")
    free_after = torch.cuda.mem_get_info(local)[0]   # what is left for the runtime's scratch and the legs after
    cnt = torch.full((S,), P, dtype=torch.int32, device=f"cuda:{local}")
    gen = slo_amd.DeviceGenerator(pid, a.config_id, stream0, S, local)
    rec_n = ctxs[0].L.slo_record_floats()
    rec = torch.zeros((S, rec_n), dtype=torch.float32, device=f"cuda:{local}")
    gathered = torch.zeros((world * S, rec_n), dtype=torch.float32, device=f"cuda:{local}") if gather else None
    exts = [torch.cuda.ExternalStream(c.stream_handle) for c in ctxs]
    pool = ThreadPoolExecutor(max_workers=len(ctxs)) if len(ctxs) > 1 else None

    def each(fn):
        """fn(g, ctx, offset, count) for every group, concurrently (ctypes drops the GIL)"""
        if pool is None:
            fn(0, ctxs[0], *groups[0])
            return
        for f in [pool.submit(fn, g, c, *groups[g]) for g, c in enumerate(ctxs)]:
            f.result()

    def sync_all():
        each(lambda g, c, o, n: c.synchronize())

    # optional extra Scan Context history (makeAndSaveScancontextAndKeys of scans before 0)
    chunk = min(a.chunk, wscans)
    for h0 in range(-a.history, 0, chunk):
        nh = min(chunk, -h0)
        gen.scans(h0, nh, dev.data_ptr())
        for h in range(nh):
            each(lambda g, c, o, n: c.batch_sc_make(dev[h, o].data_ptr(), cnt[o].data_ptr()))
        sync_all()
    t_gen = time.time() - t_gen

    # ---- pre-roll: scans [0, preroll), generated on the device a chunk at a time
    t_pre = time.time()
    for k0 in range(0, a.preroll + maxlag, chunk):
        nk = min(chunk, a.preroll + maxlag - k0)
        sync_all()
        gen.scans(k0, nk, dev.data_ptr())
        for j in range(nk):
            each(lambda g, c, o, n: c.batch_process(dev[j, o].data_ptr(), cnt[o].data_ptr(), 0.1 * (k0 + j))
                 if k0 + j < a.preroll + lag(g) else None)
    sync_all()
    t_pre = time.time() - t_pre
    base = a.preroll
    win = [0, 0]   # the resident window holds steps [win[0], win[0] + win[1]) (+ maxlag scans for the lags)

    def load(k0, n):
        """generate steps [k0, k0 + n) of every stream into the window (untimed)"""
        sync_all()
        t1 = time.time()
        gen.scans(base + k0, n + maxlag, dev.data_ptr())
        torch.cuda.synchronize()
        win[0], win[1] = k0, n
        return time.time() - t1

    def ensure(k0, n):   # make steps [k0, k0 + n) resident; the window starts at k0 when it is reloaded
        if not (win[0] <= k0 and k0 + n <= win[0] + win[1]):
            return load(k0, min(seg_len, total - k0))
        return 0.0

    t_gen += ensure(0, min(seg_len, total))

    def step(k, serial=False):   # k = step index; context g processes scan base + lag(g) + k
        j = k - win[0]   # its slot in the resident window
        if serial:   # instrumented pass: one context at a time, so its kernels have the device alone
            for g, c in enumerate(ctxs):
                c.batch_process(dev[j + lag(g), groups[g][0]].data_ptr(), cnt[groups[g][0]].data_ptr(),
                                0.1 * (base + lag(g) + k))
                c.synchronize()
        else:
            each(lambda g, c, o, n: c.batch_process(dev[j + lag(g), o].data_ptr(), cnt[o].data_ptr(),
                                                    0.1 * (base + lag(g) + k)))
        if gather:   # records of every group, then one all-gather after all of them
            evs = []
            for g, c in enumerate(ctxs):
                c.pack_records(rec[groups[g][0]].data_ptr())
                ev = torch.cuda.Event()
                ev.record(exts[g])
                evs.append(ev)
            for ev in evs[1:]:
                exts[0].wait_event(ev)
            with torch.cuda.stream(exts[0]):
                sdist.gather_records(rec, gathered)
                h = exts[0].cuda_stream
                xsc.ingest(gathered.data_ptr(), h)
                xsc.query(gathered[stream0].data_ptr(), S, stream0, matches.data_ptr(), h)
                done = torch.cuda.Event()
                done.record(exts[0])
            for e in exts[1:]:
                e.wait_event(done)   # next step's records overwrite rec

    # ---- instrumented pass first (scans [0, profile) of the window): per-kernel
    # HIP-event times on each context's stream, the contexts one after the other
    # so the events time each kernel alone; it names the dominant kernel, which
    # is then timed live inside the timed region
    roof, roof_also, kt, workload, gbs, path = None, None, {}, None, {}, None
    counts, map_steps = None, 0
    P0 = a.profile_steps
    if P0 > 0:
        for c in ctxs:
            c.timing(True)
            c.timing_reset()
        pw0 = [c.get(0, "pcl_work").astype(np.int64) for c in ctxs]
        wk0 = [c.get(0, "work").astype(np.int64) for c in ctxs]
        for k in range(P0):
            t_gen += ensure(k, 1)
            step(k, serial=True)
            sync_all()
            map_steps += int(int(ctxs[0].get(0, "flags")[0]) & 2 != 0)
        for c in ctxs:
            for kn, (kms, kcalls) in c.timing_read().items():
                m0, c0 = kt.get(kn, (0.0, 0))
                kt[kn] = (m0 + kms, c0 + kcalls)
            c.timing(False)
        parts = [stream_counts(c, c.n_streams) for c in ctxs]
        counts = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
        counts["pcl_work"] = sum(c.get(0, "pcl_work").astype(np.int64) - w0 for c, w0 in zip(ctxs, pw0))
        wk = sum(c.get(0, "work").astype(np.int64) - w0 for c, w0 in zip(ctxs, wk0))
        counts["sc_pairs"] = int(wk[0])
        counts["long_items"], counts["long_voxels"] = int(wk[1]), int(wk[2])
        workload = {k: round(float(v.mean()), 1) for k, v in counts.items()
                    if k not in ("pcl_work", "sc_pairs", "long_items", "long_voxels") and v.ndim == 1}
    # the largest single kernel by device time (vg_sort:<filter> entries time groups of launches)
    dominant = max(((kn, v) for kn, v in kt.items() if not kn.startswith("vg_sort:")),
                   key=lambda kv: kv[1][0])[0] if kt else None
    rk0 = dominant if a.roofline_kernel == "auto" else a.roofline_kernel
    rks = ([rk0] if rk0 else []) + [k for k in a.roofline_also.split(",") if k and k != rk0]

    for k in range(P0, P0 + a.warmup):
        t_gen += ensure(k, 1)
        step(k)
    sync_all()
    torch.cuda.synchronize()
    # the roofline kernels alone are timed inside the timed region: two
    # in-stream device timestamps per launch on its context's stream (captured
    # into the step graphs), nothing else
    for c in ctxs:
        c.timing(True)
        c.timing_filter(",".join(rks))
        c.timing_reset()
    if a.trace_marker:   # a torch spin kernel on either side of the timed steps (tools/trace_window.py)
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    # the timed steps, in segments of what the window holds (one segment
    # unless --steps exceeds the HBM budget): each segment's scans resident
    # before it, the segment bracketed by barrier + synchronize on both sides,
    # the job's time = the sum over segments of the slowest rank's
    el, n_seg = 0.0, 0
    for k0, n in budget.segments(P0 + a.warmup, total, seg_len):
        t_gen += ensure(k0, n)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(k0, k0 + n):
            step(k)
        sync_all()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el += sdist.max_over_ranks(time.perf_counter() - t0, f"cuda:{local}")
        n_seg += 1
    gen.close()
    if a.trace_marker:
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    live = {k: [0.0, 0] for k in rks}
    for c in ctxs:
        for kn, (kms, kcalls) in c.timing_read().items():
            if kn in live:
                live[kn][0] += kms
                live[kn][1] += kcalls
        c.timing(False)
        c.timing_filter(None)
    value = S * a.steps * world / el
    # every stream's sticky error bits (capacity clips; since round 4 also the
    # PCL-order sorts' guards, PclWs::serr) and the sorts' guard counters
    errs = sum(int(c.get(s, "err")[0]) != 0 for c in ctxs for s in range(c.n_streams))
    vgs = sum(c.get(0, "vg_stats").astype(np.int64) for c in ctxs)
    guards = {"fallback_ranges": int(vgs[0]), "inconsistent_steps": int(vgs[2] + vgs[3] + vgs[4]),
              "clipped_outputs": int(vgs[1] != 0),
              "note": "PCL-order VoxelGrid sort over the whole run: fallback_ranges = ranges over 4 Ki items whose "
                      "introsort depth budget ran out (std::sort's heapsort, done exactly by one wave), guards of "
                      "impossible steps (must be 0; each also sets its stream's err bit)"}
    kfs = np.array([int(c.get(s, "n_keyframes")[0]) for c in ctxs for s in range(c.n_streams)])

    if counts is not None:
        total_ms = sum(v[0] for kn, v in kt.items() if not kn.startswith("vg_sort:"))   # groups double count
        for kn, (kms, kcalls) in kt.items():
            kb = algo_bytes(kn, counts, cfg, S, P0, map_steps)
            if kb is not None and kms > 0:
                gbs[kn] = round(kb / (kms / 1e3) / 1e9, 1)

        # achieved = algorithmic bytes per launch (instrumented pass, same
        # launch mix) / the average launch time inside the timed region,
        # where the contexts' kernels share the device
        def roof_of(rk):
            rms, rn = kt.get(rk, (0.0, 0))
            rb = algo_bytes(rk, counts, cfg, S, P0, map_steps)
            bpl = rb / rn if (rb and rn) else None   # an empty work counter prices nothing: null, not 0
            lms, ln = live.get(rk, (0.0, 0))
            live_s = lms / 1e3 / ln if ln else None
            ach = bpl / live_s / 1e9 if (bpl is not None and live_s) else None
            iso = bpl / (rms / 1e3 / rn) / 1e9 if (bpl is not None and rms > 0) else None
            if rk == "sc_detect":   # the Scan Context Gram on the matrix cores: flop, not bytes
                tf = lambda f, t: f / t / 1e12 if (f is not None and t) else None  # noqa: E731
                live_t, iso_t = tf(bpl, live_s), tf(bpl, rms / 1e3 / rn if rn else None)
                pk = MFMA_F64_PEAK_TFLOPS
                return {"bound": "mfma", "dtype": "f64", "achieved": round(live_t, 4) if live_t else None,
                        "peak": pk, "unit": "TFLOP/s",
                        "frac": round(live_t / pk, 6) if (live_t and pk) else None, "kernel": rk,
                        "avg_launch_us": round(live_s * 1e6, 2) if live_s else None, "launches_timed": ln,
                        "flop_per_launch": int(bpl) if bpl is not None else None,
                        "pairs_in_window": counts.get("sc_pairs"),
                        "isolated": {"achieved": round(iso_t, 4) if iso_t else None,
                                     "frac": round(iso_t / pk, 6) if (iso_t and pk) else None,
                                     "avg_launch_us": round(rms / rn * 1e3, 2) if rn else None},
                        "share_of_device_time": round(rms / total_ms, 4) if total_ms else None,
                        "note": "issued MFMA flop (64 x 64 padded Gram, ceil(NR/16) k-steps per Eigen accumulator) "
                                "per distance pair; the kernel's other work (ring-key K-NN, sector-key alignment) is VALU"}
            traffic, tsrc = pmc_traffic(a.traffic_from, rk, a.profile_tag)
            comp = None
            cb = compulsory_bytes(rk, counts)
            if cb and rn:   # SURVEY §8(d)'s compulsory bytes: the sort family's VoxelGrid input once (16 B / item)
                cpl = cb / rn
                cach = cpl / live_s / 1e9 if live_s else None
                comp = {"bytes_per_launch": int(cpl), "achieved": round(cach, 2) if cach else None,
                        "frac": round(cach / HBM_PEAK_GBS, 5) if cach else None,
                        "note": "16 B x the PCL-order VoxelGrid input items of the window / this kernel's launches "
                                "(a lower bound: the filter's input read once); bytes_per_launch above models "
                                "the implementation's passes"}
            return {"bound": "hbm", "achieved": round(ach, 2) if ach is not None else None, "peak": HBM_PEAK_GBS,
                    "compulsory": comp,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5) if ach is not None else None,
                    "traffic": traffic, "traffic_source": tsrc, "kernel": rk,
                    "avg_launch_us": round(live_s * 1e6, 2) if live_s else None, "launches_timed": ln,
                    "bytes_per_launch": int(bpl) if bpl is not None else None,
                    "isolated": {"achieved": round(iso, 2) if iso is not None else None,
                                 "frac": round(iso / HBM_PEAK_GBS, 5) if iso is not None else None,
                                 "avg_launch_us": round(rms / rn * 1e3, 2) if rn else None,
                                 "note": "instrumented steps, contexts one after the other"},
                    "share_of_device_time": round(rms / total_ms, 4) if total_ms else None}

        roof = roof_of(rks[0])
        roof["largest_kernel"] = dominant
        roof_also = {rk: roof_of(rk) for rk in rks[1:] if rk in kt}
        # the whole path: per-scan algorithmic bytes from the
        # logged counts, the mapping share from the instrumented pass, over the
        # timed window's wall time
        fb, mb = path_bytes(counts, cfg, a.history)
        per_step = fb + mb * map_steps / P0
        ach = per_step * a.steps * world / el / 1e9
        roof["path"] = {"achieved": round(ach, 2), "unit": "GB/s", "bytes_per_step": int(per_step),
                        "frac_of_measured_copy_6290": round(ach / 6290.0, 5),
                        "frac_of_spec_8000": round(ach / 8000.0, 5), "mapping_share": round(map_steps / P0, 3),
                        "note": "SURVEY §8(d) per-scan formula on the logged counts (last instrumented step's sizes)"}
    elif rks and live.get(rks[0], [0, 0])[1]:   # no instrumented pass: the live launch time alone (no byte counts)
        lms, ln = live[rks[0]]
        roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None, "kernel": rks[0], "avg_launch_us": round(lms / ln * 1e3, 2), "launches_timed": ln}
    for c in ctxs:
        c.close()
    ctxs = []
    del dev
    if pool is not None:
        pool.shutdown()
    if xsc is not None:
        xsc.close()
    torch.cuda.empty_cache()
    if gather:
        if world > 1:
            dist.barrier()
        dist.destroy_process_group()
    if rank != 0:   # the other ranks are done: their GPUs are free for rank 0's Mode S leg
        return

    # ---- one stream alone (C3 is defined on one KITTI replay)
    one = one_p = one_p3 = one_c = None
    if a.single_steps > 0:
        one, one_state = single_stream(torch, slo_amd, a, cfg, pid, local)
        one_c = single_stream_ctx_pipeline(torch, slo_amd, a, cfg, pid, local, one_state)
        one_p = single_stream_pipelined(torch, slo_amd, a, cfg, pid, local)
        one_p3 = single_stream_pipelined(torch, slo_amd, a, cfg, pid, local, stages=3)

    # ---- Mode S over the ranks: one stream, front ends dealt over the GPUs,
    # the back end on the owner; at N = 1 the ranks are threads
    # of this process on one GPU (LocalTransport), at N > 1 a fresh group of N
    # processes over RCCL, started once every rank has released its GPU
    ranks_leg = None
    if a.modes_steps > 0:
        ranks_leg = modes_leg_local(torch, slo_amd, a, cfg, pid, local) if world == 1 else modes_leg_launch(a, world)

    # ---- loop verification (MO:964-1110), measured apart
    # from the headline (not part of the metric): a batch of --icp-jobs ICP
    # alignments through slo_icp_align_batch, each a 1/16-subsampled scan
    # displaced by a loop-closure-sized drift (<= 0.3 m, 0.02 rad) onto every
    # 4th point of the same scan (~29k points, a voxelised submap's density)
    icp = None
    if a.icp_jobs > 0:
        icp = icp_bench(torch, slo_amd, pid, a, local, gthreads)

    # ---- CPU baseline (oracle = C++ restatement of the reference), rank 0, N = 1
    cpu = None
    if world == 1 and a.cpu_scans > 0:
        cpu = cpu_baseline(a, pid, ncpu, a.preroll + P0 + a.warmup)

    A = cpu["A_reference_topology"]["value"] if cpu else None
    vs_a = lambda leg: round(leg["value"] / A, 2) if (leg and A and leg.get("value")) else None  # noqa: E731
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "scans/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": a.workload, "sc_candidates": cfg.sc_num_candidates,
                   "loop_closure": bool(cfg.loop_closure_enable),
                   "preset": a.preset, "streams_per_gpu": S, "contexts_per_gpu": n_ctx,
                   "scans_per_step": S * world, "preroll_scans": a.preroll,
                   "context_phase_lag": [lag(g) for g in range(n_ctx)],
                   "timed_scans": [base + P0 + a.warmup, base + P0 + a.warmup + a.steps - 1],
                   "timed_segments": n_seg, "resident_steps": seg_len,
                   "voxel_order": "pcl std::sort (reference)" if a.voxel_order == 0 else "stable",
                   "keyframes_per_stream_at_end": {"min": int(kfs.min()), "mean": round(float(kfs.mean()), 1)},
                   "local_map_keyframes": min(int(kfs.min()), cfg.surrounding_keyframe_search_num),
                   "sc_history_seed": a.history,
                   "launch": "eager" if a.no_graphs else "one HIP graph per context and step",
                   "parallelism": f"streams sharded over {world} GPU(s)"},
        "roofline": roof,
        "roofline_also": roof_also,
        "cpu_baseline": cpu,
        "speedup_vs_cpu": round(value / cpu["value"], 2) if cpu else None,
        "speedup_vs_cpu_A": vs_a({"value": value}),
        "single_stream": one,
        "single_stream_speedup_vs_cpu_A": vs_a(one),
        "single_stream_ctx_pipeline": one_c,
        "single_stream_ctx_pipeline_speedup_vs_cpu_A": vs_a(one_c),
        "single_stream_pipelined": one_p,
        "single_stream_pipelined_speedup_vs_cpu_A": vs_a(one_p),
        "single_stream_pipelined3": one_p3,
        "single_stream_pipelined3_speedup_vs_cpu_A": vs_a(one_p3),
        "single_stream_ranks": ranks_leg,
        "single_stream_ranks_speedup_vs_cpu_A": vs_a(ranks_leg),
        "stream_errors": errs,
        "sort_guards": guards,
        "kernels_ms": {k: [round(v[0], 3), int(v[1])] for k, v in sorted(kt.items(), key=lambda kv: -kv[1][0])},
        "kernels_algo_gbs": gbs, "workload_mean_last_step": workload,
        "setup_seconds": round(t_gen, 1), "preroll_seconds": round(t_pre, 1),
        "hbm": {"context_gb": round(ctx_bytes / 2**30, 2), "window_gb": round(wscans * step_b / 2**30, 2),
                "xsc_store_gb": round(xsc_b / 2**30, 3), "free_after_window_gb": round(free_after / 2**30, 2)},
        "loop_verify_icp": icp,
    }
    if world == 1 and a.extra not in ("", "none"):   # the other BASELINE configs at 1 GPU, each by its own process
        out["config_lines"] = extra_lines(a)
    line = contract_line(out)
    line["detail"] = write_detail(a, out)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
