#!/usr/bin/env python3
"""JSON-in end-to-end rates and phase split alone (bench.py's json_in block without the 10M resident
population): the first --pairs pairs of config3 as JSON in host memory -> gpudiff_submit -> gpudiff_wait, with
host encoding, device encoding and its A/B variants.  Prints one JSON object.

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
    args = ap.parse_args()
    import torch
    import bench
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S
    torch.cuda.set_device(0)
    pop = S.Population(S.make_cfg(args.config, n_pairs=args.pairs))
    out = bench.json_in_rates(G, pop, pop.n, args.threads, 0)
    out["config"] = args.config
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
