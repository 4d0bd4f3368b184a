#!/bin/bash
# Round 6 (y): K10's occupancy now that its arrays live in scratch -- 6 and 7 waves/SIMD vs 8 (.).
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/ab_tree.py run .,k10w6,k10w7 --script bench.py --config upsert --rounds 3 -- --no-cpu-baseline --steps 10 > $O/ab_upsert.jsonl 2> $O/ab_upsert.log || { tail -20 $O/ab_upsert.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06y/ab_upsert.jsonl"):
    d = json.loads(l)
    print(d["variant"], d["round"], round(d["value"] / 1e6, 3), round(d["ms_per_step"], 4), d["checks"]["full_size"]["device_vs_host_mismatches"], d["checks"]["sample"])
PY
echo done
