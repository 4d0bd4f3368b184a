#!/bin/bash
# Round 6 (b): K2 with the small pairs' joins staged in LDS and the sentinel-only pairs written lane-parallel --
# parity tests first, then an interleaved A/B against the round-start kernel (base) on config2 / config3 / config4.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 600 python -u tools/ab_tree.py run base,new,new4 --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; cat $O/ab_c2.jsonl | cut -c1-600; exit 1; }
timeout -k 10 600 python -u tools/ab_tree.py run base,new,new4 --config config4 --rounds 2 > $O/ab_c4.jsonl 2> $O/ab_c4.log || { tail -20 $O/ab_c4.log; exit 1; }
timeout -k 10 900 python -u tools/ab_tree.py run base,new,new4 --config config3 --pairs 2000000 --rounds 2 > $O/ab_c3.jsonl 2> $O/ab_c3.log || { tail -20 $O/ab_c3.log; exit 1; }
python - <<'PY'
import json
for f in ["ab_c2", "ab_c4", "ab_c3"]:
    for l in open("gpurun_out/r06b/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
