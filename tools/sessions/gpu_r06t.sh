#!/bin/bash
# Round 6 (t): the byte-heaviest N = 8 share (with the world-1 collective) -- round-start kernel (r5) vs current (.),
# alternating on one box; and the same share through k2_time (isolated K2 / pass / two-in-flight step).
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u tools/ab_tree.py run r5,.,r5,. --script bench.py --config config3 --rounds 1 --timeout 300 -- --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 100 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/ab_share.jsonl 2> $O/ab_share.log || { tail -20 $O/ab_share.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06t/ab_share.jsonl"):
    d = json.loads(l)
    print(d["variant"], d["config"]["pairs_per_rank"], round(d["ms_per_step"], 4), json.dumps(d["kernels_ms"])[:300])
PY
echo done
