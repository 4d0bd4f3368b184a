#!/usr/bin/env python3
"""GPU occupancy of a bench run with two passes in flight, from a rocprofv3 kernel (+ memory copy) trace: over
the window of the last --steps K2 launches, the union of all GPU operations' intervals (busy), the union of the
K2 launches alone, and the idle gaps -- whether the step is bound by the GPU's own work or by the host's
enqueue / the collective.

    python tools/busy_union.py <trace dir> [--steps 20] > out.json
"""
import argparse
import csv
import json
import os


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    ops = []
    for name, kind in (("run_kernel_trace.csv", "k"), ("run_memory_copy_trace.csv", "c")):
        p = os.path.join(a.dir, name)
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            nm = r.get("Kernel_Name", r.get("Direction", "copy"))
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm, kind))
    ops.sort()
    k2 = [o for o in ops if "k_compare_flat" in o[2]]
    k2 = k2[-a.steps:]
    w0, w1 = k2[0][0], max(o[1] for o in k2)
    win = [(max(s, w0), min(e, w1)) for s, e, _, _ in ops if e > w0 and s < w1]
    busy, gaps = union(win)
    k2busy, _ = union([(s, e) for s, e, _, _ in k2])
    span = w1 - w0
    out = dict(steps=len(k2), window_us=span / 1e3, per_step_us=span / 1e3 / len(k2),
               busy_frac=busy / span, k2_union_frac=k2busy / span,
               k2_mean_us=sum(e - s for s, e, _, _ in k2) / len(k2) / 1e3,
               idle_gaps=len(gaps), idle_us_total=sum(gaps) / 1e3,
               idle_gap_max_us=max(gaps) / 1e3 if gaps else 0.0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
