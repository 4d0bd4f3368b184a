#!/bin/bash
# Round 6 (aw): bytes_eq 8 bytes a step (K12's label check, K13's repeated-key check, K10's owner-reference name):
# parity (strings, upsert, rollup, negotiate), then interleaved A/B of roll-up and negotiation (api) against HEAD.
set -o pipefail
O=gpurun_out/r06aw; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_strings.py tests/test_gpu_upsert.py tests/test_gpu_rollup.py tests/test_gpu_negotiate.py \
  > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python -u tools/ab_tree.py run base,. --script bench.py --config rollup --rounds 2 -- --no-cpu-baseline --steps 10 \
  > $O/ab_rollup.txt 2>&1 || { tail -20 $O/ab_rollup.txt; exit 1; }
timeout -k 10 300 python -u tools/ab_tree.py run base,. --script bench.py --config negotiate --rounds 2 -- --kind api --no-cpu-baseline --steps 10 \
  > $O/ab_neg_api.txt 2>&1 || { tail -20 $O/ab_neg_api.txt; exit 1; }
for f in $O/ab_rollup.txt $O/ab_neg_api.txt; do
python - $f <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["variant"], d["round"], round(d["value"] / 1e6, 2), d.get("kernels_ms"))
PY
done
echo done
