#!/bin/bash
# Round 6 (m): config3 at full size (10M pairs) -- the round-start kernel (r5, e76128f) vs the current one (.),
# alternating on one box: isolated K2 / pass and the two-in-flight step.
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/ab_tree.py run r5,.,r5,. --config config3 --rounds 1 --timeout 400 -- --no-check --passes 10 > $O/ab_c3_10m.jsonl 2> $O/ab_c3_10m.log || { tail -20 $O/ab_c3_10m.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06m/ab_c3_10m.jsonl"):
    d = json.loads(l)
    print(d["variant"], d["round"], round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3), d["wall_s"])
PY
echo done
