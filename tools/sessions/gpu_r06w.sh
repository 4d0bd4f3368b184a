#!/bin/bash
# Round 6 (w): small launches' drain -- 8-pair tail items (t8), 16-pair main items (ipw12), a tail twice as long (tq4)
# vs the final kernel (.): config2 and a 1.25M-pair config3 population (the N = 8 share's size).
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u tools/ab_tree.py run .,t8,ipw12,tq4 --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
timeout -k 10 800 python -u tools/ab_tree.py run .,t8,ipw12,tq4 --config config3 --pairs 1250000 --rounds 2 > $O/ab_share.jsonl 2> $O/ab_share.log || { tail -20 $O/ab_share.log; exit 1; }
python - <<'PY'
import json
for f in ("ab_c2", "ab_share"):
    for l in open("gpurun_out/r06w/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
