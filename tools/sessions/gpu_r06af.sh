#!/bin/bash
# Round 6 (af): where the two-in-flight half grid stops paying -- config3 at 2.5M (12.8 GB, the N = 4 share) and 5M
# pairs (25.7 GB, the N = 2 share): never (hg0), up to 16 GiB (.), up to 64 GiB (hg64).
set -o pipefail
O=gpurun_out/r06af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u tools/ab_tree.py run hg0,.,hg64 --config config3 --pairs 2500000 --rounds 2 -- --no-check > $O/ab_2500k.jsonl 2> $O/ab_2500k.log || { tail -20 $O/ab_2500k.log; exit 1; }
timeout -k 10 800 python -u tools/ab_tree.py run hg0,hg64,hg0,hg64 --config config3 --pairs 5000000 --rounds 1 -- --no-check > $O/ab_5m.jsonl 2> $O/ab_5m.log || { tail -20 $O/ab_5m.log; exit 1; }
python - <<'PY'
import json
for f in ("ab_2500k", "ab_5m"):
    for l in open("gpurun_out/r06af/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d.get("step_ms_2inflight_staggered", 0), 4), round(d["k2_frac"], 3))
PY
echo done
