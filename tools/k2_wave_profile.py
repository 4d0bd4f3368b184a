"""K2's per-wave timeline on MI355X: where a diff pass loses time against a pure stream.

Ingests config3 (optionally resized) like bench.py, times the default K2 ("variant0") and then runs its
timeline build ("variant14", selected by gpudiff_k2_profile: the same kernel plus wall-clock stamps, 100 MHz), recording
per wave: start, end of
its first item, items taken, start of its last item, end, ticks spent streaming and in the join.

    python tools/k2_wave_profile.py --pairs 1250000 [--passes 5] [--config config4 --flags 0xF00000] > out.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(a, qs=(0, 1, 5, 25, 50, 75, 95, 99, 100)):
    return {str(q): round(float(np.percentile(a, q)), 2) for q in qs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1250000)
    ap.add_argument("--config", default="config3")
    ap.add_argument("--flags", type=lambda x: int(x, 0), default=0, help="extra engine flags (e.g. 0xF << 21: every join in K4)")
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    import torch
    from kcp_amd import gpudiff as G
    from kcp_amd import synth as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(device=dev)  # the engine's stream, made torch's current one: exports,
    torch.cuda.set_stream(stream)            # copies and collectives all order on it (never the null stream)
    cfg = S.make_cfg(args.config, n_pairs=args.pairs, n_clusters=max(1, args.pairs // 100))
    pop = S.Population(cfg, 1, 0)
    n = pop.n
    out = {"pairs": n}
    for variant in (0, 14):  # 14: the timeline build (installed buffer; the record names of earlier rounds)
        eng = G.Engine(device=0, encode_threads=args.threads, stream=stream.cuda_stream, timing=True, flags=args.flags)
        cap = 1 << 16
        buf = torch.zeros(cap * 12, dtype=torch.int64, device=dev)
        if variant == 14:  # the timeline build runs while a buffer is installed (gpudiff_k2_profile)
            eng.k2_profile(buf.data_ptr(), cap)
        first = pop.chunk(eng, 0, min(262144, n), args.threads)
        per_pair = first.pool_bytes / max(1, min(262144, n))
        db = eng.device_batch(int(per_pair * n * (1.4 if args.config == "config4" else 1.15)) + (64 << 20), n)
        db.append(first.hb)
        pos, k, stage = first.truth.size, 1, [first.hb, None]
        while pos < n:
            m = min(262144, n - pos)
            ch = pop.chunk(eng, pos, m, args.threads, reuse=stage[k & 1])
            stage[k & 1] = ch.hb
            db.append(ch.hb)
            pos += m
            k += 1
        eng.sync()
        eng.wait(eng.diff(db))
        eng.timing_reset()
        for _ in range(args.passes):
            eng.diff(db)
        eng.sync()
        tm = eng.timings()
        rec = {"k2_ms": tm.compare_ms, "pass_ms": tm.total_ms, "join_ms": tm.join_ms, "emit_ms": tm.emit_ms,
               "compact_ms": tm.compact_ms, "format_bytes": db.stats().compare_bytes}
        if variant == 14:
            buf.zero_()
            eng.diff(db)
            eng.sync()
            eng.k2_profile(0, 0)
            r = buf.view(cap, 12).cpu().numpy().astype(np.int64)
            r = r[r[:, 4] != 0]
            t0 = r[:, 0].min()
            us = lambda x: (x.astype(np.float64)) / 100.0  # 100 MHz ticks -> us
            start, end = us(r[:, 0] - t0), us(r[:, 4] - t0)
            span = float(end.max())
            busy = end - start
            rec.update({
                "waves": int(r.shape[0]),
                "span_us": span,
                "start_us": pct(start),
                "first_item_end_us": pct(us(r[:, 1] - t0)),
                "last_item_start_us": pct(us(r[:, 3] - t0)),
                "end_us": pct(end),
                "items_per_wave": pct(r[:, 2].astype(np.float64)),
                "busy_frac_of_span": float(busy.sum() / (r.shape[0] * span)),
                "stream_frac_of_busy": float(us(r[:, 5]).sum() / busy.sum()),
                "join_frac_of_busy": float(us(r[:, 6]).sum() / busy.sum()),
                "other_frac_of_busy": float(1 - (us(r[:, 5]).sum() + us(r[:, 6]).sum()) / busy.sum()),
                # the "other" time, split: rows (+ result stores, ticket), rows -> first pass, after the
                # joins (counts, stores), item end -> next item start (ticket); per item, us
                "per_item_us": {k: float(us(r[:, c]).sum() / max(1, r[:, 2].sum()))
                                for k, c in (("rows", 8), ("pre_stream", 9), ("post_join", 10), ("advance", 11),
                                             ("stream", 5), ("join", 6))},
                "idle_before_us_mean": float(start.mean()),
                "idle_after_us_mean": float((span - end).mean()),
            })
            # the end of the pass: how many waves are still running at each point of the last 20%
            grid = np.linspace(0.8 * span, span, 11)
            rec["running_at"] = {"%.1f" % g: int(((start <= g) & (end > g)).sum()) for g in grid}
            # the 40 waves that end last: when their last item started, and their totals
            late = np.argsort(end)[-40:]
            rec["late_waves"] = [dict(last_item_start_us=round(float(us(r[k, 3] - t0)), 1), end_us=round(float(end[k]), 1),
                                      items=int(r[k, 2]), stream_us=round(float(us(r[k, 5])), 1),
                                      join_us=round(float(us(r[k, 6])), 1)) for k in late]
        out["variant%d" % variant] = rec
        db.free()
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
