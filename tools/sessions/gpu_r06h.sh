#!/bin/bash
# Round 6 (h): K10 occupancy -- tokenize.hip without private-array-to-LDS promotion (nopromote) vs as built (base):
# the write-path bench (upsert), and roll-up / negotiation as controls.
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/ab_tree.py run base,nopromote --script bench.py --config upsert --rounds 3 -- --no-cpu-baseline --steps 10 > $O/ab_upsert.jsonl 2> $O/ab_upsert.log || { tail -20 $O/ab_upsert.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,nopromote --script bench.py --config rollup --rounds 2 -- --no-cpu-baseline --steps 10 > $O/ab_rollup.jsonl 2> $O/ab_rollup.log || { tail -20 $O/ab_rollup.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,nopromote --script bench.py --config negotiate --rounds 2 -- --no-cpu-baseline --steps 10 > $O/ab_neg.jsonl 2> $O/ab_neg.log || { tail -20 $O/ab_neg.log; exit 1; }
python - <<'PY'
import json
for f in ["ab_upsert", "ab_rollup", "ab_neg"]:
    for l in open("gpurun_out/r06h/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], round(d["value"] / 1e6, 3), d.get("ms_per_step"), json.dumps(d.get("kernels_ms"))[:200], d.get("checks", {}) if f == "ab_upsert" else "")
PY
echo done
