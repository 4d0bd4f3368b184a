#!/bin/bash
# Round 6 (f): every small join moved from K2 to K3's compaction waves (deferjoin, staged in LDS there) vs joins in
# K2 (., with K3's whole deferrals now staged in LDS too) vs the round's first K2 change (base).
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 700 python -u tools/ab_tree.py run base,.,deferjoin --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,.,deferjoin --config config3 --pairs 2000000 --rounds 2 > $O/ab_c3.jsonl 2> $O/ab_c3.log || { tail -20 $O/ab_c3.log; exit 1; }
timeout -k 10 500 python -u tools/ab_tree.py run base,deferjoin --config config4 --rounds 2 > $O/ab_c4.jsonl 2> $O/ab_c4.log || { tail -20 $O/ab_c4.log; exit 1; }
python - <<'PY'
import json
for f in ["ab_c2", "ab_c3", "ab_c4"]:
    for l in open("gpurun_out/r06f/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
