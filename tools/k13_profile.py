#!/usr/bin/env python3
"""K13 phase profile (run on the GPU box): where a wave's time goes when it
extracts the negotiation classifier's fields of an APIResourceImport /
NegotiatedAPIResource -- structural scan, tree walk, the N0-N4 sweep (one slot since round 6)
(per-phase wall-clock ticks summed over waves)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kcp_amd import gpudiff as G  # noqa: E402
from kcp_amd import synth as S  # noqa: E402

n_pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
pairs, _ = S.negotiate_population(n_pairs, variants=False)
n = 2 * len(pairs)
eng = G.Engine(device=0, timing=True)
nb = eng.nbatch(pairs)
nb.run()
nb.fetch()
for on in (False, True):
    eng.k0_profile(on)
    t = time.time()
    nb.run()
    eng.sync()
    dt = time.time() - t
    prof = eng.k0_profile(False)
    print("profile=%s: K13+K14 %.2f ms for %d docs" % (on, dt * 1e3, n))
tot = sum(prof[:3])
for k, nm in [(0, "scan"), (1, "tree"), (2, "N0-N4 sweep + out")]:
    print("  %-18s %6.1f%%  %.2f us/doc-wave" % (nm, 100.0 * prof[k] / max(1, tot), prof[k] / 100.0 / n))
nb.close()
eng.close()
