"""Split a bench step into its pieces from a rocprofv3 kernel trace (where the N = 8 share's
step goes beyond its K2 stream).

    python tools/timeline_split.py <dir with run_kernel_trace.csv [run_memory_copy_trace.csv]> [--last 15] > out.json

Steps are delimited by the K2 launches (k_compare_flat); the last --last complete steps are used (run the
bench with --no-cpu-baseline --sample 0 so no other diff follows the timed loop).
Per step (means over the timed steps, microseconds): the reset kernel, K2, K3 (scan tiles / apply /
compact), K4 (slices / gather), K5 + K6 (scan tiles / apply / copy paths), the collective's kernels (RCCL
all-gather) and copies (exports, count read-back), every idle gap between consecutive GPU operations
inside the step, and the gap from the step's last operation to the next step's first -- the host's turn
(reading the gathered counts back, enqueuing the next pass)."""
import argparse
import csv
import glob
import json
import os
import sys


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    return rows


def col(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    raise KeyError(names)


def classify(name):
    n = name
    if "k_pass_reset" in n:
        return "reset"
    if "k_compare" in n:
        return "K2"
    if "k_compact" in n:
        return "K3_compact"
    if "k_scan_tiles" in n or "k_scan_apply" in n:
        return "scan_V4" if "V4" in n else "scan_u32"
    if "k_join_slices" in n:
        return "K4a"
    if "k_join_gather" in n:
        return "K4b"
    if "k_copy_paths" in n:
        return "K6"
    if "nccl" in n.lower() or "rccl" in n.lower():
        return "rccl"
    return "other:" + n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=15, help="use the last N complete steps (the timed ones)")
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not kt:
        sys.exit("no kernel trace under %s" % a.dir)
    ops = []
    for r in load(kt[0]):
        name = col(r, "Kernel_Name", "KernelName")
        ops.append((int(col(r, "Start_Timestamp", "BeginNs")), int(col(r, "End_Timestamp", "EndNs")),
                    classify(name)))
    mc = glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    if mc:
        for r in load(mc[0]):
            kind = col(r, "Direction", "Kind", "Operation")
            ops.append((int(col(r, "Start_Timestamp", "BeginNs")), int(col(r, "End_Timestamp", "EndNs")),
                        "copy_" + str(kind).lower().replace("memory_copy_", "")))
    ops.sort()
    k2 = [i for i, o in enumerate(ops) if o[2] == "K2"]
    # a step starts at the reset kernel before its K2 (if any) and runs to the next step's start
    starts = []
    for i in k2:
        j = i - 1 if i > 0 and ops[i - 1][2] == "reset" else i
        starts.append(j)
    steps = []
    for s in range(len(starts) - 1):
        seg = ops[starts[s]:starts[s + 1]]
        nxt = ops[starts[s + 1]][0]
        d = {}
        gaps = 0.0
        end = seg[0][0]
        for b, e, c in seg:
            d[c] = d.get(c, 0.0) + (e - b) / 1e3
            if b > end:
                gaps += (b - end) / 1e3
            end = max(end, e)
        k2_b = [o for o in seg if o[2] == "K2"][0]
        d["gaps_inside"] = gaps
        d["host_turn"] = max(0.0, (nxt - end) / 1e3)
        d["step"] = (nxt - seg[0][0]) / 1e3
        d["after_K2_to_end"] = (end - k2_b[1]) / 1e3
        steps.append(d)
    timed = steps[-a.last:]
    keys = sorted({k for d in timed for k in d})
    mean = {k: round(sum(d.get(k, 0.0) for d in timed) / len(timed), 2) for k in keys}
    out = {"steps_total": len(steps), "steps_used": len(timed), "mean_us": mean,
           "kernels_per_step": round(sum(1 for o in ops if not o[2].startswith("copy")) / max(1, len(steps) + 1), 1),
           "source": os.path.relpath(kt[0])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
