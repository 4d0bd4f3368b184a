#!/bin/bash
# Round 6 (s): the byte-heaviest rank's share of an 8-way split of config3, timed alone on one GPU at the final
# sources (with the world-1 RCCL collective and without), beside a 10M pass on the same box.
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python -u bench.py --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 100 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share_gather.json 2> $O/share_gather.log || { tail -30 $O/share_gather.log; exit 1; }
timeout -k 10 400 python -u bench.py --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 100 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share.json 2> $O/share.log || { tail -30 $O/share.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/full10m.json 2> $O/full10m.log || { tail -30 $O/full10m.log; exit 1; }
python - <<'PY'
import json
O = "gpurun_out/r06s"
full = json.loads(open(O + "/full10m.json").read().strip().splitlines()[-1])
ideal = full["ms_per_step"] / 8
print("10M", round(full["value"] / 1e6, 1), "M pairs/s", round(full["ms_per_step"], 4), "ms; ideal share", round(ideal, 4))
for f in ("share_gather", "share"):
    d = json.loads(open("%s/%s.json" % (O, f)).read().strip().splitlines()[-1])
    print(f, d["config"]["pairs_per_rank"], round(d["ms_per_step"], 4), "ms/step, of ideal", round(ideal / d["ms_per_step"], 3), json.dumps((d.get("checks") or {}).get("gather"))[:300])
PY
echo done
