"""K1 (value digests) variants A/B on MI355X: ingest a config3 population per variant
(GPUDIFF_OPT_K1_VARIANT_SHIFT), then time stand-alone K1 passes over it with HIP events and check
that every variant leaves the pool byte-identical to variant 0's.

    python tools/k1_ab.py --pairs 2500000 [--variants 0,1,2,3] > out.json
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2500000)
    ap.add_argument("--config", default="config3")
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--passes", type=int, default=5)
    args = ap.parse_args()
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S
    cfg = S.make_cfg(args.config, n_pairs=args.pairs, n_clusters=max(1, args.pairs // 100))
    pop = S.Population(cfg, 1, 0)
    n = pop.n
    out = {"pairs": n, "config": args.config}
    for v in [int(x) for x in args.variants.split(",")]:
        eng = G.Engine(device=0, encode_threads=16, timing=True, flags=v << 30, device_value_hash=True)
        first = pop.chunk(eng, 0, min(262144, n), 16)
        per_pair = first.pool_bytes / max(1, min(262144, n))
        db = eng.device_batch(int(per_pair * n * (1.4 if args.config == "config4" else 1.15)) + (64 << 20), n)
        db.append(first.hb)
        pos, k, stage = first.truth.size, 1, [first.hb, None]
        while pos < n:
            m = min(262144, n - pos)
            ch = pop.chunk(eng, pos, m, 16, reuse=stage[k & 1])
            stage[k & 1] = ch.hb
            db.append(ch.hb)
            pos += m
            k += 1
        eng.sync()
        st = db.stats()
        ms = []
        for _ in range(args.passes):
            db.hash_values()
            eng.sync()
            ms.append(eng.timings().value_hash_ms)
        h = hashlib.sha256()
        step = 1 << 28
        for o in range(0, st.pool_bytes, step):
            h.update(db.read_pool(o, min(step, st.pool_bytes - o)))
        best = min(ms)
        out["variant%d" % v] = {"k1_ms": ms, "best_ms": best, "hash_bytes": st.hash_bytes,
                                "tb_s": st.hash_bytes / (best * 1e-3) / 1e12,
                                "frac_of_8tbs": st.hash_bytes / (best * 1e-3) / 8e12,
                                "pool_sha": h.hexdigest()[:16]}
        print(json.dumps({v: out["variant%d" % v]}), file=sys.stderr, flush=True)
        db.free()
        eng.close()
    shas = {out[k]["pool_sha"] for k in out if k.startswith("variant")}
    out["pools_identical"] = len(shas) == 1
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
