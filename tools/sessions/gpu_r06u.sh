#!/bin/bash
# Round 6 (u): the final K2 sources (.) against the round-start kernel (r5) on the three shapes that matter: the N = 8
# share with the world-1 collective (bench.py step), config2 and config3 at 10M (k2_time), alternating on one box;
# K2 parity first.
set -o pipefail
O=gpurun_out/r06u; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 900 python -u tools/ab_tree.py run r5,.,r5,. --script bench.py --config config3 --rounds 1 --timeout 300 -- --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 100 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/ab_share.jsonl 2> $O/ab_share.log || { tail -20 $O/ab_share.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run r5,. --config config2 --rounds 3 > $O/ab_c2.jsonl 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
timeout -k 10 700 python -u tools/ab_tree.py run r5,.,r5,. --config config3 --rounds 1 --timeout 400 -- --no-check --passes 10 > $O/ab_c3_10m.jsonl 2> $O/ab_c3_10m.log || { tail -20 $O/ab_c3_10m.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06u/ab_share.jsonl"):
    d = json.loads(l)
    k = d["kernels_ms"]
    print("share", d["variant"], round(d["ms_per_step"], 4), "k2", round(k["compare_all_launches"], 4), "k3", round(k["compact"], 4), "pass", round(k["diff_pass"], 4))
for f in ("ab_c2", "ab_c3_10m"):
    for l in open("gpurun_out/r06u/%s.jsonl" % f):
        d = json.loads(l)
        print(f, d["variant"], d["round"], d.get("flags_eq"), d.get("paths_eq"), round(d["k2_ms"], 4), round(d["pass_ms"], 4), round(d.get("step_ms_2inflight", 0), 4), round(d["k2_frac"], 3))
PY
echo done
