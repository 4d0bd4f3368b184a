#!/bin/bash
# Round 4 (p): K2 in-flight depth A/B -- variant 0 (x4, 4 waves/SIMD), 10 (x8, 3 waves), 11 (x8 held to 4 waves,
# 36 B/lane spills), 12 (x16, 2 waves) -- on config3 10M (the headline), config4 and the N = 8 share.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "variants" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "c4_v11:0xB00" "c4_v12:0xC00" "c4_v10:0xA00" "c4_v0:0" "sh_v12:0xC00" "sh_v10:0xA00" "sh_v0:0"; do
  n=${v%%:*}; f=${v#*:}
  case $n in c4*) a="--config config4 --steps 30";; sh*) a="--emulate-world 8 --steps 40";; esac
  timeout -k 10 300 python bench.py --pipeline 1 $a --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
for v in "m_v10:0xA00" "m_v0:0" "m_v12:0xC00"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 400 python bench.py --pipeline 1 --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
