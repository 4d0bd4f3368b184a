#!/bin/bash
# Round 6 (n): K2 without the LDS-staged join (nostage: 123 VGPRs, 4 waves/SIMD) vs the current kernel (., 137 VGPRs,
# 3 waves/SIMD) vs the round-start kernel (r5): config3 at full size and config2.
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/ab_tree.py run r5,nostage,.,r5,nostage,. --config config3 --rounds 1 --timeout 400 -- --no-check --passes 10 > $O/ab_c3_10m.jsonl 2> $O/ab_c3_10m.log || { tail -20 $O/ab_c3_10m.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run r5,nostage,. --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
python - <<'PY'
import json
for f in ("ab_c3_10m", "ab_c2"):
    for l in open("gpurun_out/r06n/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
