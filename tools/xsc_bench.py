"""Cross-stream Scan Context store at multi-GPU sizes on one GPU: a store of
N streams x cap keyframes filled with synthetic descriptors, then the time of
slo_xsc_query for S own records (all carrying a keyframe: the worst step).
python tools/xsc_bench.py [N] [S] [cap]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sc-lego-loam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import slo_amd  # noqa: E402
from slo_amd import xsc as X  # noqa: E402
from slo_amd import _abi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 512
CAP = int(sys.argv[3]) if len(sys.argv) > 3 else 64
cfg = slo_amd.preset("hdl64_1800")
R = _abi.RECORD_FLOATS
REC = _abi.REC
rng = np.random.default_rng(0)
st = X.CrossSession(cfg, N, CAP, 0)
tab = torch.zeros((N, R), dtype=torch.float32, device="cuda")
tab[:, REC["kf_saved"]] = 1.0
for k in range(CAP):
    d = rng.random((N, 1200), dtype=np.float32) * (rng.random((N, 1200)) < 0.3)
    tab[:, REC["desc"]:REC["desc"] + 1200] = torch.from_numpy(d.astype(np.float32)).cuda()
    tab[:, REC["kf_index"]] = float(k)
    st.ingest(tab.data_ptr())
torch.cuda.synchronize()
matches = torch.zeros((S, X.MATCH_DTYPE.itemsize // 4), dtype=torch.int32, device="cuda")
for _ in range(3):
    st.query(tab.data_ptr(), S, 0, matches.data_ptr())
torch.cuda.synchronize()
reps = 10
t0 = time.perf_counter()
for _ in range(reps):
    st.query(tab.data_ptr(), S, 0, matches.data_ptr())
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / reps * 1e3
print(f"xsc_query N={N} streams x {CAP} keyframes, {S} queries: {ms:.3f} ms", flush=True)
st.close()
