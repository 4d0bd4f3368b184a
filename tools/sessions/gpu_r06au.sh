#!/bin/bash
# Round 6 (au): K14 compares spans 8 bytes a step: parity (negotiate, strings), then interleaved A/B of the
# negotiation benches (api, crd) against HEAD.
set -o pipefail
O=gpurun_out/r06au; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_strings.py tests/test_gpu_negotiate.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
for k in crd api; do
timeout -k 10 400 python -u tools/ab_tree.py run base,. --script bench.py --config negotiate --rounds 3 -- --kind $k --no-cpu-baseline --steps 10 \
  > $O/ab_neg_$k.txt 2>&1 || { tail -20 $O/ab_neg_$k.txt; exit 1; }
python - $O/ab_neg_$k.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["variant"], d["round"], round(d["value"] / 1e6, 2), d.get("kernels_ms"))
PY
done
echo done
