#!/usr/bin/env python3
"""K10 (write path) phase profile on config3 documents (run on the GPU box):
bodies/s of one K10 launch over a resident gpudiff_wbatch and where a wave's
time goes (per-phase wall-clock ticks summed over waves)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench_upsert  # noqa: E402
from kcp_amd import gpudiff as G  # noqa: E402
from kcp_amd import synth as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
pop = S.Population(S.make_cfg("config3"))
buf, offs, _ = pop.json_range(0, n, 8)
docs = [bench_upsert.add_owner_refs(bytes(buf[offs[2 * i + 1]:offs[2 * i + 2]]), i) for i in range(n)]
kinds = {}
for d in docs:
    k = d[d.find(b'"kind":"') + 8:][:12].split(b'"')[0].decode()
    kinds[k] = kinds.get(k, 0) + 1
print("docs %d, mean %.0f B, kinds %s" % (n, np.mean([len(d) for d in docs]), kinds))
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
eng = G.Engine(device=0, timing=True, flags=0)
print("K10 variant", variant)
wb = eng.wbatch(docs)
wb.run()
r = wb.fetch()
for on in (False, True):
    eng.k0_profile(on)
    t = time.time()
    wb.run()
    eng.sync()
    dt = time.time() - t
    prof = eng.k0_profile(False)
    print("profile=%s: %.2f ms per launch, %d host-completed" % (on, dt * 1e3, r.n_host))
names = ["scan", "tree", "M1 sizes", "M5 ranks+depth sort", "M6-M8", "M9 emit", "M1 floats", "M2-M4"]
tot = sum(prof[:8])
for k, nm in enumerate(names):
    print("  %-9s %6.1f%%  %.2f us/doc-wave" % (nm, 100.0 * prof[k] / max(1, tot), prof[k] / 100.0 / n))
# per-kind launch times
for kind in sorted(kinds):
    sub = [d for d in docs if (b'"kind":"%s"' % kind.encode()) in d][:20000]
    w2 = eng.wbatch(sub)
    w2.run()
    w2.fetch()
    t = time.time()
    for _ in range(3):
        w2.run()
    eng.sync()
    dt = (time.time() - t) / 3
    print("  kind %-10s %6d docs, mean %5.0f B: %.2f ms/launch, %.2f M docs/s" % (
        kind, len(sub), np.mean([len(d) for d in sub]), dt * 1e3, len(sub) / dt / 1e6))
    w2.close()
wb.close()
eng.close()
