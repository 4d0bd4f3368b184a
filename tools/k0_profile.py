#!/usr/bin/env python3
"""K0 phase profile on synthetic config3 documents (run on the GPU box):
docs/s of one K0 launch through gpudiff_encode_objects and where a wave's time
goes (per-phase wall-clock ticks summed over waves)."""
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kcp_amd import gpudiff as G  # noqa: E402
from kcp_amd import synth as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
cfg = S.make_cfg("config3", n_pairs=n, n_clusters=max(1, n // 100))
pop = S.Population(cfg)
buf, offs, _ = pop.json_range(0, n, 8)
docs = [bytes(buf[offs[2 * i + 1]:offs[2 * i + 2]]) for i in range(n)]
print("docs %d, mean %.0f B" % (n, np.mean([len(d) for d in docs])))
variants = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0"])]
for var in variants:
    eng = G.Engine(device=0, flags=0)
    eng.encode_objects(docs[:256])  # warm
    for on in (False, True):
        eng.k0_profile(on)
        t = time.time()
        res = eng.encode_objects(docs)
        dt = time.time() - t
        prof = eng.k0_profile(False)
        bad = sum(1 for i, _ in res if i["status"] != 0)
        print("variant %d profile=%s: %.1f ms incl. staging, %d deferred" % (var, on, dt * 1e3, bad))
    names = ["scan", "tree", "values", "hashes", "sort", "blob"]
    tot = sum(prof[:6])
    for k, nm in enumerate(names):
        print("  %-7s %6.1f%%  %.2f us/doc-wave" % (nm, 100.0 * prof[k] / max(1, tot), prof[k] / 100.0 / n))
    eng.close()
