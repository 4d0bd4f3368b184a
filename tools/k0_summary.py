#!/usr/bin/env python3
"""K0 rate from a tools/k0_bench.py run under `rocprofv3 --kernel-trace --output-format csv`.

    python tools/k0_summary.py <k0_kernel_trace.csv> <k0_bench.json> [--reps 6]

k0_bench.py launches K0 once on 512 documents (warm), then --reps times on the full batch, then (with --profile)
once more with the in-kernel phase stamps on. The timed launches are the --reps in between: their durations,
the JSON bytes they read (k0_bench.json's json_bytes_per_launch) and the rate, one JSON object on stdout."""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    bench = json.load(open(a.bench))
    rows = [r for r in csv.DictReader(open(a.trace)) if "k_encode_docs" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    timed = rows[1:1 + a.reps]
    if len(timed) != a.reps:
        raise SystemExit(f"expected {a.reps + 1}+ K0 launches, found {len(rows)}")
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in timed]
    nbytes = bench["json_bytes_per_launch"]
    med = statistics.median(us)
    out = dict(kernel=timed[0]["Kernel_Name"].split("(")[0], docs=bench["docs"], json_bytes_per_launch=nbytes,
               launches_us=us, median_us=med, min_us=min(us), json_gb_s_median=nbytes / med / 1e3,
               json_gb_s_best=nbytes / min(us) / 1e3, docs_per_s_median=bench["docs"] / med * 1e6,
               vgpr=int(timed[0]["VGPR_Count"]), scratch=int(timed[0]["Scratch_Size"]),
               lds=int(timed[0]["LDS_Block_Size"]), grid=int(timed[0]["Grid_Size_X"]),
               wg=int(timed[0]["Workgroup_Size_X"]))
    if "phases" in bench:
        out["phase_share"] = {k: round(v["share"], 4) for k, v in bench["phases"].items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
