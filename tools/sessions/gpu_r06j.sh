#!/bin/bash
# Round 6 (j): K2 with the ticket atomic taken after the item's first pass and the next item's rows prefetched (.),
# the late atomic alone (noprefetch), the current kernel (base): parity (hand-out shapes), wave timeline, A/B.
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python -u tools/k2_wave_profile.py --config config2 --pairs 1000000 > $O/wave_c2.json 2> $O/wave.log || { tail -30 $O/wave.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,.,noprefetch --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run base,.,noprefetch --config config3 --pairs 2000000 --rounds 2 > $O/ab_c3.jsonl 2> $O/ab_c3.log || { tail -20 $O/ab_c3.log; exit 1; }
python - <<'PY'
import json
w = json.load(open("gpurun_out/r06j/wave_c2.json"))["variant14"]
print({k: w[k] for k in ("k2_ms", "waves", "busy_frac_of_span", "stream_frac_of_busy", "join_frac_of_busy", "idle_after_us_mean")}, w["per_item_us"])
for f in ["ab_c2", "ab_c3"]:
    for l in open("gpurun_out/r06j/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
