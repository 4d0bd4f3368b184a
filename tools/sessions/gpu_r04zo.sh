#!/bin/bash
# Round 4 (zo): the largest-first rounds defer joins over 1024 keys (sliced deferrals: K4's grid-wide slices, not
# K3's whole-deferral joins) vs joins kept in K2 (0x80), one and two passes in flight, config4.
set -o pipefail
O=gpurun_out/r04zo; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "hand_out or largest_first or deep" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "p1_defer:1:0" "p1_k2join:1:0x80" "p2_defer:2:0" "p2_k2join:2:0x80" "p1_defer_b:1:0" "p1_k2join_b:1:0x80" "p2_defer_b:2:0" "p2_k2join_b:2:0x80"; do
  n=${v%%:*}; r=${v#*:}; pl=${r%%:*}; f=${r#*:}
  timeout -k 10 300 python bench.py --pipeline $pl --config config4 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); k=d['kernels_ms']; print('$n', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['format']['frac'],4), round(k['compare_all_launches'],4), round(k['diff_pass'],4))"
done
