#!/usr/bin/env python3
"""Interleaved A/B of device-encoded JSON-in streaming (batch k + 1 submitted before batch k is waited) across
engine variants chosen by environment knobs read when the context's store is created: each variant's engine is
built once, then rounds alternate between them.  Prints one JSON object: per variant, the pairs/s of every round.

    python tools/json_in_ab.py [--pairs 131072] [--rounds 4] [--zero-copy]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {"default": {}, "k0_coupled": {"GPUDIFF_K0_COUPLED": "1"}, "one_k0_stream": {"GPUDIFF_K0_ONE_STREAM": "1"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--zero-copy", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S
    torch.cuda.set_device(0)
    pop = S.Population(S.make_cfg("config3", n_pairs=args.pairs))
    buf, offs, _ = pop.json_range(0, pop.n, 16)
    engs = {}
    for name, env in VARIANTS.items():
        os.environ.update(env)
        e = G.Engine(device=0, encode_threads=16, device_encode=True)
        pj = G.PinnedJson(e, buf, offs) if args.zero_copy else None
        arr = pj.pairs if pj is not None else G.json_pair_array(buf, offs)
        for _ in range(2):
            e.wait(e.submit_array(arr))  # creates the store (reads the environment) and warms both ring slots
        for k in env:
            os.environ.pop(k)
        engs[name] = (e, arr, pj)
    out = {name: [] for name in VARIANTS}
    want = None
    for _ in range(args.rounds):
        for name, (e, arr, _pj) in engs.items():
            t0 = time.perf_counter()
            tk = e.submit_array(arr)
            for _ in range(args.batches - 1):
                nxt = e.submit_array(arr)
                r = e.wait(tk)
                tk = nxt
            r = e.wait(tk)
            dt = time.perf_counter() - t0
            want = r.pair_flags if want is None else want
            assert np.array_equal(r.pair_flags, want)
            out[name].append(round(pop.n * args.batches / dt))
    for e, _arr, pj in engs.values():
        if pj is not None:
            pj.free()
        e.close()
    print(json.dumps(dict(pairs=pop.n, batches=args.batches, zero_copy=args.zero_copy, pairs_per_s=out,
                          best={k: max(v) for k, v in out.items()})), flush=True)


if __name__ == "__main__":
    main()
