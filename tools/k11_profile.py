#!/usr/bin/env python3
"""K11 phase profile (run on the GPU box): where a wave's time goes when it
extracts the roll-up fields of a Deployment -- structural scan, tree walk,
passes R0-R3 (per-phase wall-clock ticks summed over waves)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcp_amd import gpudiff as G  # noqa: E402
from kcp_amd import synth as S  # noqa: E402

roots = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
docs, _ = S.rollup_population(roots, 4)
n = len(docs)
eng = G.Engine(device=0, timing=True)
rb = eng.rbatch(docs)
rb.run()
rb.fetch()
for on in (False, True):
    eng.k0_profile(on)
    t = time.time()
    rb.run()
    eng.sync()
    dt = time.time() - t
    prof = eng.k0_profile(False)
    print("profile=%s: K11+K12 %.2f ms for %d docs" % (on, dt * 1e3, n))
tot = sum(prof[:3])
for k, nm in enumerate(["scan", "tree", "R0-R3"]):
    print("  %-6s %6.1f%%  %.2f us/doc-wave" % (nm, 100.0 * prof[k] / max(1, tot), prof[k] / 100.0 / n))
rb.close()
eng.close()
