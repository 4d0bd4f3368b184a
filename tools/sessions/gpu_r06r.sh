#!/bin/bash
# Round 6 (r): the default kernel with the block-cooperative final round (help8) vs without (.): config2, config3 2M
# and 10M (K2 parity through the A/B tool's full CPU CSR check on config2 / config3 2M).
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/ab_tree.py run .,help8 --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run .,help8 --config config3 --pairs 2000000 --rounds 2 > $O/ab_c3.jsonl 2> $O/ab_c3.log || { tail -20 $O/ab_c3.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run .,help8,.,help8 --config config3 --rounds 1 --timeout 400 -- --no-check --passes 10 > $O/ab_c3_10m.jsonl 2> $O/ab_c3_10m.log || { tail -20 $O/ab_c3_10m.log; exit 1; }
python - <<'PY'
import json
for f in ("ab_c2", "ab_c3", "ab_c3_10m"):
    for l in open("gpurun_out/r06r/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
