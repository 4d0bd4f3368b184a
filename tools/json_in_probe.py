#!/usr/bin/env python3
"""JSON-in end-to-end rates and phase split alone (bench.py's json_in block without the 10M resident
population): the first --pairs pairs of config3 as JSON in host memory -> gpudiff_submit -> gpudiff_wait, with
host encoding, device encoding (staged, streaming, zero copy).  Prints one JSON object.

    python tools/json_in_probe.py [--pairs 131072] [--threads 16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--pairs", type=int, default=131072)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--device-only", type=int, default=0, metavar="REPS",
                    help="only REPS device-encode submit+wait rounds after two warm ones (a timeline to profile)")
    args = ap.parse_args()
    import torch
    import bench
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S
    torch.cuda.set_device(0)
    pop = S.Population(S.make_cfg(args.config, n_pairs=args.pairs))
    if args.device_only:
        import time
        buf, offs, _ = pop.json_range(0, pop.n, args.threads)
        arr = G.json_pair_array(buf, offs)
        e = G.Engine(device=0, encode_threads=args.threads, device_encode=True)
        for _ in range(2):
            e.wait(e.submit_array(arr))
        walls = []
        for _ in range(args.device_only):
            t0 = time.perf_counter()
            tk = e.submit_array(arr)
            t1 = time.perf_counter()
            e.wait(tk)
            t2 = time.perf_counter()
            walls.append(dict(submit_ms=(t1 - t0) * 1e3, wait_ms=(t2 - t1) * 1e3, pairs_per_s=pop.n / (t2 - t0)))
        e.close()
        print(json.dumps(dict(config=args.config, pairs=pop.n, json_bytes=int(offs[-1]), rounds=walls)), flush=True)
        return
    out = bench.json_in_rates(G, pop, pop.n, args.threads, 0)
    out["config"] = args.config
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
