#!/bin/bash
# Round 6 (z): a kernel trace of config2's timed loop (two passes in flight): do the two passes' K2 launches overlap
# end to end (synchronized) or does one fill the other's drain?
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/$O/kt -o run --output-format csv -- \
    python3 $R/bench.py --config config2 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $R/$O/bench.json 2> $R/$O/bench.log ) || { tail -30 $O/bench.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -n 1); cp "$f" $O/kernel_trace.csv
python - <<'PY'
import csv, json
rows = [r for r in csv.DictReader(open("gpurun_out/r06z/kernel_trace.csv"))]
k2 = sorted([(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id") or r.get("Stream_Id")) for r in rows
             if "k_compare_flat" in r["Kernel_Name"]])
print("K2 launches", len(k2), "queues", sorted({q for _, _, q in k2}))
t0 = k2[-40][0]
for s, e, q in k2[-12:]:
    print(q, round((s - t0) / 1e3, 1), round((e - t0) / 1e3, 1), "dur", round((e - s) / 1e3, 1))
PY
echo done
