#!/usr/bin/env python3
"""K0 (k_encode_docs, encode mode) on one config5-sized batch of config3 documents: the JSON bytes per
launch and docs/s, for rocprofv3 runs (kernel-trace stats / PMC passes) of the same command.

    python tools/k0_bench.py [--docs 65536] [--reps 6] [--profile]

Prints one JSON object: documents, JSON bytes per launch (the algorithmic bytes K0 must read), mean size,
wall time per gpudiff_encode_objects call (H2D + K0 + D2H), deferrals; with --profile the per-phase split
of the in-kernel wall-clock stamps (gpudiff_k0_profile)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--lib", default="", help="A/B: another build of libgpudiff.so (e.g. a K0 launch shape)")
    args = ap.parse_args()
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S
    if args.lib:
        G.LIB_PATH = os.path.abspath(args.lib)
        G._lib = G._load()

    n = args.docs
    cfg = S.make_cfg("config3", n_pairs=n, n_clusters=max(1, n // 100))
    pop = S.Population(cfg)
    buf, offs, _ = pop.json_range(0, n, 8)
    docs = [bytes(buf[offs[2 * i + 1]:offs[2 * i + 2]]) for i in range(n)]
    nbytes = sum(len(d) for d in docs)
    eng = G.Engine(device=0)
    eng.encode_objects(docs[:512])  # warm
    times = []
    res = None
    for _ in range(args.reps):
        t = time.perf_counter()
        res = eng.encode_objects(docs)
        times.append(time.perf_counter() - t)
    out = dict(lib=args.lib or "kcp_amd/libgpudiff.so", docs=n, json_bytes_per_launch=nbytes, mean_doc_bytes=nbytes / n,
               call_ms_min=min(times) * 1e3, deferred=sum(1 for i, _ in res if i["status"] != 0))
    if args.profile:
        eng.k0_profile(True)
        eng.encode_objects(docs)
        prof = eng.k0_profile(False)
        names = ["scan", "tree", "values", "hashes", "sort", "blob"]
        tot = max(1, sum(prof[:6]))
        out["phases"] = {nm: dict(share=prof[k] / tot, us_per_doc_wave=prof[k] / 100.0 / n)
                         for k, nm in enumerate(names)}
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
