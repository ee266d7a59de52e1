"""Experiment: G independent contexts (S/G streams each) driven by G host
threads, so one group's latency-bound phases overlap another's
throughput-bound ones.  python tools/overlap_exp.py S G steps warmup"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
import torch  # noqa: E402
import slo_amd  # noqa: E402

S, G, K, W = (int(x) for x in sys.argv[1:5])
offset = float(sys.argv[5]) if len(sys.argv) > 5 else 0.0
cfg = slo_amd.preset("hdl64_1800")
pid = slo_amd.PRESETS["hdl64_1800"]
P = cfg.max_points
Sg = S // G
ntot = K + W
dev = torch.empty((ntot, S, P, 4), dtype=torch.float32, device="cuda")
for k0 in range(0, ntot, 4):
    nk = min(4, ntot - k0)
    dev[k0:k0 + nk].copy_(torch.from_numpy(slo_amd.gen_batch(pid, 3, 0, S, k0, nk, P, 16)))
cnt = torch.full((S,), P, dtype=torch.int32, device="cuda")
ctxs = [slo_amd.Context(cfg, 0, Sg) for _ in range(G)]


def run(g, k0, k1):
    c = ctxs[g]
    for k in range(k0, k1):
        c.batch_process(dev[k, g * Sg].data_ptr(), cnt[g * Sg].data_ptr(), 0.1 * k + offset * g)
    c.synchronize()


def phase(k0, k1):
    th = [threading.Thread(target=run, args=(g, k0, k1)) for g in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join()


phase(0, W)
torch.cuda.synchronize()
t0 = time.perf_counter()
phase(W, W + K)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"S={S} G={G} offset={offset}: {S * K / el:.1f} scans/s ({el / K * 1e3:.3f} ms/step)")
