#!/bin/bash
# Round 6 (aj): K11's R0-R3 as one sweep: parity, then interleaved A/B against HEAD (ab/base).
set -o pipefail
O=gpurun_out/r06aj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_strings.py tests/test_gpu_rollup.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 400 python -u tools/ab_tree.py run base,. --script bench.py --config rollup --rounds 3 -- --no-cpu-baseline --steps 10 \
  > $O/ab_rollup.txt 2>&1 || { tail -20 $O/ab_rollup.txt; exit 1; }
python - $O/ab_rollup.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["variant"], d["round"], round(d["value"] / 1e6, 2), d.get("kernels_ms"))
PY
echo done
