#!/bin/bash
# Round 6 (at): K10 M6 / M8 / M9 load their operands ahead of their branches: parity (strings, upsert, write plan,
# K0), K10 phase profile, then interleaved A/B of the write path against HEAD.
set -o pipefail
O=gpurun_out/r06at; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_strings.py tests/test_gpu_upsert.py tests/test_gpu_write_plan.py tests/test_gpu_tokenize.py tests/test_gpu_json_in.py \
  > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 300 python -u tools/k10_profile.py > $O/k10_profile.txt 2>&1 || { tail -20 $O/k10_profile.txt; exit 1; }
cat $O/k10_profile.txt
timeout -k 10 400 python -u tools/ab_tree.py run base,. --script bench.py --config upsert --rounds 3 -- --no-cpu-baseline --steps 10 \
  > $O/ab_upsert.txt 2>&1 || { tail -20 $O/ab_upsert.txt; exit 1; }
python - $O/ab_upsert.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(d["variant"], d["round"], round(d["value"] / 1e6, 2), d.get("kernels_ms"))
PY
echo done
