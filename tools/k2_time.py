"""One population, K2 and the diff pass timed over isolated passes, plus the full-size parity check of the first pass
against the CPU merge over the same CSR (oracle/csr_ref.cpp: flags and every changed path).  Run from a tree made by
tools/ab_tree.py (its own kcp_amd first on sys.path) to A/B builds on one box, one process per measurement.

    python tools/k2_time.py --config config2 [--pairs N] [--passes 20] [--pipeline-steps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
MAIN = os.environ.get("KCP_AB_MAIN")  # the main repo: oracle/ (the checker) when run from an A/B tree
if MAIN and MAIN not in sys.path:
    sys.path.append(MAIN)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config2")
    ap.add_argument("--pairs", type=int, default=0)
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--pipeline-steps", type=int, default=20, help="two passes in flight (bench.py's step), 0: skip")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    import torch

    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    cfg = S.make_cfg(args.config, n_pairs=args.pairs, n_clusters=max(1, args.pairs // 100) if args.pairs else 0)
    pop = S.Population(cfg, 1, 0)
    n = pop.n
    eng = G.Engine(device=0, encode_threads=args.threads, stream=stream.cuda_stream, timing=True)
    chunk = 262144
    first = pop.chunk(eng, 0, min(chunk, n), args.threads)
    per_pair = first.pool_bytes / max(1, min(chunk, n))
    db = eng.device_batch(int(per_pair * n * (1.4 if args.config == "config4" else 1.15)) + (64 << 20), n)
    parts = []

    def cpu(hb):
        if args.no_check:
            return
        from oracle import cpu_ref
        inf = hb.info()
        parts.append(cpu_ref.csr_paths_ptr(inf.pool, hb.rows(), args.threads))
    cpu(first.hb)
    db.append(first.hb)
    pos, k, stage = first.truth.size, 1, [first.hb, None]
    while pos < n:
        m = min(chunk, n - pos)
        ch = pop.chunk(eng, pos, m, args.threads, reuse=stage[k & 1])
        cpu(ch.hb)
        stage[k & 1] = ch.hb
        db.append(ch.hb)
        pos += m
        k += 1
    eng.sync()
    res = eng.wait(eng.diff(db))
    out = {"config": args.config, "pairs": n, "build_id": getattr(G, "BUILD_ID", None), "tree": HERE,
           "format_bytes": db.stats().compare_bytes}
    if parts:
        c_flags = np.concatenate([q[0] for q in parts])
        c_offs, base = [np.zeros(1, np.int64)], 0
        for q in parts:
            c_offs.append(q[1][1:].astype(np.int64) + base)
            base += int(q[1][-1])
        c_offs = np.concatenate(c_offs)
        out["flags_eq"] = bool(np.array_equal(res.pair_flags & 7, c_flags))
        out["paths_eq"] = bool(np.array_equal(res.path_offsets.astype(np.int64), c_offs) and
                               np.array_equal(res.path_hashes, np.concatenate([q[2] for q in parts])) and
                               np.array_equal(res.path_kinds, np.concatenate([q[3] for q in parts])))
    del res
    k2, pas = [], []
    for _ in range(args.passes):
        eng.timing_reset()
        eng.wait(eng.diff(db))
        tm = eng.timings()
        k2.append(tm.compare_ms)
        pas.append(tm.total_ms)
    out["k2_ms"] = float(np.median(k2))
    out["k2_ms_min"] = float(np.min(k2))
    out["pass_ms"] = float(np.median(pas))
    out["k2_frac"] = out["format_bytes"] / (out["k2_ms"] * 1e-3) / 8e12
    if args.pipeline_steps:
        # bench.py's default step: two passes in flight, each on its own context over a view of the batch
        s2 = torch.cuda.Stream(device=dev)
        eng2 = G.Engine(device=0, encode_threads=args.threads, stream=s2.cuda_stream)
        view = db.view(eng2)
        engs, dbs = [eng, eng2], [db, view]
        eng2.wait(eng2.diff(view))
        for i in range(4):
            engs[i & 1].diff(dbs[i & 1])
        for stagger in (0.0, 1e-4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.pipeline_steps):  # bench.py's timed loop
                engs[i & 1].diff(dbs[i & 1])
                if i == 0 and stagger:
                    time.sleep(stagger)  # the first pass's K2 holds every CU slot before the second is launched
            torch.cuda.synchronize()
            out["step_ms_2inflight" if not stagger else "step_ms_2inflight_staggered"] = (
                (time.perf_counter() - t0) / args.pipeline_steps * 1e3)
        view.free()
        eng2.close()
    print(json.dumps(out), flush=True)
    db.free()
    eng.close()


if __name__ == "__main__":
    main()
