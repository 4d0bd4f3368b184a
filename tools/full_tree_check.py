"""Full-size changed-path parity independent of the product encoder.

bench.py's full-size check compares the GPU with the CPU merge over the SAME host-encoded CSR bytes, so an
encoder defect would be reproduced on both sides.  Here every one of the 10M config3 pairs is decided and
path-diffed a second time from its JSON text: the generator renders each chunk's pairs as JSON
(gpudiff_synth_json_range) and the C++ tree-walk restatement of specsyncer.go:17-41 / statussyncer.go:15-27
(oracle/deepequal_ref.cpp: its own JSON decoder, Go-like value trees, the field-path diff) decides them;
its flags and changed-path lists must equal the GPU's first pass over the host-encoded population, pair for
pair.  The only thing taken from the encoder is each pair's path-hash seed (the row's seed byte: the
encoder re-seeds the rare pair whose paths collide under seed 0; the tree walk hashes under the same seed).
With --k0 every chunk's JSON also goes through the device-encode submit path (kernel K0 parses it on the
GPU) and must give the same flags and paths.  Not a timed bench.

    python tools/full_tree_check.py [--pairs 10000000] [--chunk 131072] [--k0] > full_tree_check.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print("[full_tree_check]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--pairs", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=131072)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--k0", action="store_true", help="also submit every chunk's JSON through K0 (device encode)")
    args = ap.parse_args()
    import torch
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S
    from oracle import cpu_ref

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    T = args.threads
    cfg = S.make_cfg(args.config, n_pairs=args.pairs)
    pop = S.Population(cfg)
    n = pop.n
    eng = G.Engine(device=0, encode_threads=T, stream=stream.cuda_stream)
    t0 = time.time()
    # ---- the GPU's first pass over the host-encoded population (as bench.py ingests it)
    first = pop.chunk(eng, 0, min(args.chunk, n), T)
    db = eng.device_batch(int(first.pool_bytes / max(1, min(args.chunk, n)) * n * 1.2) + (64 << 20), n)
    seeds = np.zeros(n, np.uint8)
    stage = [first.hb, None]
    pos, k = 0, 0
    ch = first
    while True:
        m = ch.truth.size
        seeds[pos:pos + m] = ((ch.hb.rows()["flags_a"] >> G.OBJ_SEED_SHIFT) & 0xFF).astype(np.uint8)
        db.append(ch.hb)
        pos += m
        k += 1
        if pos >= n:
            break
        ch = pop.chunk(eng, pos, min(args.chunk, n - pos), T, reuse=stage[k & 1])
        stage[k & 1] = ch.hb
    res = eng.wait(eng.diff(db))
    t_gpu = time.time() - t0
    log("GPU pass over %d host-encoded pairs: %d dirty, %d paths (%.1f s incl. ingest)" % (
        n, res.dirty_ids.size, res.path_hashes.size, t_gpu))
    db.free()
    for h in stage:
        if h is not None:
            h.free()
    gflags = res.pair_flags & 7
    dirty_pairs = np.nonzero(gflags & 3)[0]
    goffs = res.path_offsets.astype(np.int64)
    engk = G.Engine(device=0, encode_threads=T, device_encode=True, stream=stream.cuda_stream) if args.k0 else None
    out = dict(pairs=n, config=args.config, chunk=args.chunk, threads=T, flags_eq=True, paths_eq=True,
               gpu_dirty=int(dirty_pairs.size), gpu_paths=int(res.path_hashes.size), tree_dirty=0, tree_paths=0,
               reseeded_pairs=int(np.count_nonzero(seeds)), mismatches=[])
    if args.k0:
        out.update(k0_flags_eq=True, k0_paths_eq=True)
    t_tree = t_json = t_k0 = 0.0
    for pos in range(0, n, args.chunk):
        m = min(args.chunk, n - pos)
        t1 = time.time()
        buf, offs, _ = pop.json_range(pos, m, T)
        t_json += time.time() - t1
        t1 = time.time()
        f, o, h, kk = cpu_ref.tree_check(buf, offs, seeds[pos:pos + m], T)
        t_tree += time.time() - t1
        out["tree_dirty"] += int(o.size - 1)
        out["tree_paths"] += int(h.size)
        d0, d1 = np.searchsorted(dirty_pairs, [pos, pos + m])
        go = goffs[d0:d1 + 1] - goffs[d0]
        gh = res.path_hashes[goffs[d0]:goffs[d1]]
        gk = res.path_kinds[goffs[d0]:goffs[d1]]
        feq = bool(np.array_equal(f, gflags[pos:pos + m]))
        peq = feq and bool(np.array_equal(o.astype(np.int64), go) and np.array_equal(h, gh) and np.array_equal(kk, gk))
        if not feq or not peq:
            bad = np.nonzero(f != gflags[pos:pos + m])[0]
            out["mismatches"].append(dict(chunk=pos, flags_bad=bad[:5].tolist(), paths_eq=peq))
        out["flags_eq"] &= feq
        out["paths_eq"] &= peq
        if engk is not None:
            t1 = time.time()
            arr = G.json_pair_array(buf, offs, ids=np.arange(pos, pos + m, dtype=np.uint32))
            rk = engk.wait(engk.submit_array(arr))
            t_k0 += time.time() - t1
            kf = rk.pair_flags & 7
            kfe = bool(np.array_equal(kf, f))
            kpe = kfe and bool(np.array_equal(rk.path_offsets.astype(np.int64), o.astype(np.int64)) and
                               np.array_equal(rk.path_hashes, h) and np.array_equal(rk.path_kinds, kk))
            out["k0_flags_eq"] &= kfe
            out["k0_paths_eq"] &= kpe
            if not (kfe and kpe):
                out["mismatches"].append(dict(chunk=pos, k0_flags_eq=kfe, k0_paths_eq=kpe))
        if pos // args.chunk % 8 == 0:
            log("%d/%d pairs checked (json %.0f s, tree %.0f s, k0 %.0f s)" % (pos + m, n, t_json, t_tree, t_k0))
    out.update(seconds=dict(gpu_ingest_and_pass=round(t_gpu, 1), json_render=round(t_json, 1),
                            tree_walk=round(t_tree, 1), k0_submit=round(t_k0, 1)),
               checker="oracle/deepequal_ref.cpp oracle_tree_check: own JSON decoder + tree walk of "
                       "specsyncer.go:17-41 / statussyncer.go:15-27 + field-path diff, over JSON rendered by "
                       "gpudiff_synth_json_range; the encoder contributes only each pair's path-hash seed")
    out["mismatches"] = out["mismatches"][:20]
    print(json.dumps(out), flush=True)
    return 0 if out["flags_eq"] and out["paths_eq"] and out.get("k0_flags_eq", True) and out.get("k0_paths_eq", True) else 1


if __name__ == "__main__":
    sys.exit(main())
