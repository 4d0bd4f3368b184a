#!/usr/bin/env python3
"""Interleaved A/B of decision-kernel (K2) variants on one resident
population, in one process (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/ab_k2.py [--pairs N] [--rounds R] [--variants v:b,...]
  variant v = GPUDIFF_OPT_K2_VARIANT (0 NT x4, 1 plain x4, 2 NT x8, 3 plain x8, 4 NT x2)
  b = resident blocks per CU (0 = 8)
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--pairs", type=int, default=4_000_000)
    ap.add_argument("--clusters", type=int, default=40_000)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--variants", default="0:0,1:0,2:0,3:0,4:0,0:6,0:4")
    args = ap.parse_args()
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    base = G.Engine(device=0, encode_threads=16, timing=True)
    pop = S.Population(S.make_cfg(args.config, n_pairs=args.pairs, n_clusters=args.clusters))
    first = pop.chunk(base, 0, min(262144, pop.n), 16)
    db = base.device_batch(int(first.pool_bytes / first.truth.size * pop.n * 1.2) + (64 << 20), pop.n)
    db.append(first.hb)
    pos, stage, k = first.truth.size, [first.hb, None], 1
    while pos < pop.n:
        m = min(262144, pop.n - pos)
        ch = pop.chunk(base, pos, m, 16, reuse=stage[k & 1])
        stage[k & 1] = ch.hb
        db.append(ch.hb)
        pos += m
        k += 1
    base.sync()
    st = db.stats()
    variants = []
    for spec in args.variants.split(","):
        v, b = (int(x) for x in spec.split(":"))
        flags = (v << 8) | (b << 12)
        variants.append((spec, G.Engine(device=0, timing=True, flags=flags)))
    res = {spec: [] for spec, _ in variants}
    ref = None
    for r in range(args.rounds):
        for spec, e in variants:
            e.timing_reset()
            for _ in range(args.passes):
                e.diff(db)
            t = e.timings()
            res[spec].append(t.compare_ms)
            if r == 0:
                out = e.wait(e.diff(db))
                sig = (out.spec_dirty_ids.tobytes(), out.status_dirty_ids.tobytes(), out.path_hashes.tobytes())
                ref = ref or sig
                assert sig == ref, "variant %s changed the results" % spec
    summary = {}
    for spec, xs in res.items():
        summary[spec] = dict(median_ms=statistics.median(xs), min_ms=min(xs),
                             gbps=st.compare_bytes / (statistics.median(xs) * 1e-3) / 1e9)
    print(json.dumps(dict(pairs=pop.n, compare_bytes=st.compare_bytes, variants=summary), indent=1))


if __name__ == "__main__":
    main()
