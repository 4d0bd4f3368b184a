#!/bin/bash
# Round 4 (t): K2 variant 11 = 12 chunks a side in flight held to 3 waves/SIMD (167 VGPRs, 12 B/lane spills) vs
# 10 (x8, 3 waves) and 12 (x16, 2 waves) on config4, the N = 8 share and config3 10M.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "variants" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "c4_v11:0xB00" "c4_v12:0xC00" "c4_v10:0xA00" "c4_v11b:0xB00" "c4_v12b:0xC00" "sh_v11:0xB00" "sh_v10:0xA00"; do
  n=${v%%:*}; f=${v#*:}
  case $n in c4*) a="--config config4 --steps 30";; sh*) a="--emulate-world 8 --steps 40";; esac
  timeout -k 10 300 python bench.py --pipeline 1 $a --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
for v in "m_v11:0xB00" "m_v10:0xA00"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 400 python bench.py --pipeline 1 --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
