"""Trace the windowed K1's first wave on the GPU (gpudiff_k1_trace) for a small mixed batch."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from kcp_amd import gpudiff as G
from tests.workload import make_pairs
pairs = make_pairs(500, seed=5, mutate_frac=0.2)[0]
eng = G.Engine(device=0, flags=0 << 30)
hb = eng.encode(pairs)
info = hb.info()
db = eng.device_batch(info.pool_bytes + 1024, len(pairs))
buf = torch.zeros(12 * 4096, dtype=torch.int32, device="cuda")
eng.k1_trace(buf.data_ptr(), 4096)
db.append(hb)
eng.sync()
eng.k1_trace(0, 0)
t = buf.view(4096, 12).cpu().numpy().astype(np.int64)
t = t[: int((t[:, 4] != 0).sum())]
print(json.dumps(t.tolist()))
