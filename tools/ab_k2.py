#!/usr/bin/env python3
"""Interleaved A/B of diff-pass variants on one resident population, in one
process (cdna_hip_programming.md §5.4 rule 24).  Each variant is an engine
opened with different tuning flags (include/gpudiff.h GPUDIFF_OPT_*); all
variants must produce identical results.

usage: python tools/ab_k2.py [--pairs N] [--rounds R] [--variants name=flags,...]
  flags bits: 8-11 K2 variant (wave per pair: 1 plain x4, 2 NT x8, 3 plain x8, 4 NT x2,
              5 NT x4 <=80 VGPRs, 6 NT x2 <=64 VGPRs, 7 NT x2 <=80 VGPRs;
              flattened stream, static items: 8 x4, 9 x2, 10 x4 <= 128 VGPRs, 11 x2 5 waves/SIMD,
              12 x4 5 waves/SIMD; dynamic items + tail: 0 = x4 (the default), 13 = the default with the
              next item's rows prefetched into LDS, 15 x2), 12-15 K2 blocks/CU (0 = the measured
              occupancy), 16-19 forced segments, 0x100000 no alternate K2 stream, 4-6 tail t (t - 1
              quarters of the waves in chunks; 0 = default 2, 1 = no tail + late tickets), 0x80 8-pair
              tail items, 28-29 items per wave (0 = 6 / 8 for deep pairs, 1: 4, 2: 8, 3: 16);
              variant 14 = the default kernel + per-wave timeline (tools/k2_wave_profile.py)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("seg1=0x10000,seg2=0x20000,seg4=0x40000,seg8=0x80000,seg8noalt=0x180000,"
           "seg4noalt=0x140000,seg1b8=0x18000,seg4b6=0x46000")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--pairs", type=int, default=10_000_000)
    ap.add_argument("--clusters", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--variants", default=DEFAULT)
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
        name, flags = spec.split("=")
        variants.append((name, G.Engine(device=0, timing=True, flags=int(flags, 0))))
    res = {name: [] for name, _ in variants}
    ref = None
    for r in range(args.rounds):
        for name, e in variants:
            e.timing_reset()
            for _ in range(args.passes):
                e.diff(db)
            t = e.timings()
            res[name].append((t.total_ms, t.compare_ms, t.join_ms, t.emit_ms, t.k2_launches))
            if r == 0:
                out = e.wait(e.diff(db))
                sig = (out.spec_dirty_ids.tobytes(), out.status_dirty_ids.tobytes(), out.path_hashes.tobytes())
                ref = ref or sig
                assert sig == ref, "variant %s changed the results" % name
    summary = {}
    for name, xs in res.items():
        tot = [x[0] for x in xs]
        summary[name] = dict(pass_ms_median=statistics.median(tot), pass_ms_min=min(tot),
                             k2_span_ms=statistics.median(x[1] for x in xs),
                             join_exposed_ms=statistics.median(x[2] for x in xs),
                             emit_ms=statistics.median(x[3] for x in xs), k2_launches=xs[0][4],
                             k2_gbps=st.compare_bytes / (statistics.median(x[1] for x in xs) * 1e-3) / 1e9)
    print(json.dumps(dict(pairs=pop.n, compare_bytes=st.compare_bytes, variants=summary), indent=1))


if __name__ == "__main__":
    main()
