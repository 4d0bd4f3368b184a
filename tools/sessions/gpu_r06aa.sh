#!/bin/bash
# Round 6 (aa): K2 launches half its grid while the other pass of a two-in-flight pair is running (.) vs the full grid
# always (base): parity + collective tests, then config2, a 1.25M-pair config3 population (the N = 8 share's size) and
# config3 at 10M.
set -o pipefail
O=gpurun_out/r06aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_collective.py tests/test_gpu_dist_rehearsal.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 700 python -u tools/ab_tree.py run base,. --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,. --config config3 --pairs 1250000 --rounds 3 > $O/ab_share.jsonl 2> $O/ab_share.log || { tail -20 $O/ab_share.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,.,base,. --config config3 --rounds 1 --timeout 400 -- --no-check --passes 10 > $O/ab_c3_10m.jsonl 2> $O/ab_c3_10m.log || { tail -20 $O/ab_c3_10m.log; exit 1; }
python - <<'PY'
import json
for f in ("ab_c2", "ab_share", "ab_c3_10m"):
    for l in open("gpurun_out/r06aa/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d.get("step_ms_2inflight_staggered", 0), 4), round(d["k2_frac"], 3))
PY
echo done
