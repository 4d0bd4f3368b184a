#!/bin/bash
# Round 4 (zj): K2 variant 11 = 6 chunks a side in flight at 4 waves/SIMD (123 VGPRs) vs the default 8 at 3 waves,
# alternating, on config3 10M and the N = 8 share (one pass in flight, kernel times from the timed loop).
set -o pipefail
O=gpurun_out/r04zj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "variants" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "sh_v11:0xB00" "sh_v10:0xA00" "sh_v11b:0xB00" "sh_v10b:0xA00"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python bench.py --pipeline 1 --emulate-world 8 --steps 40 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
for v in "m_v11:0xB00" "m_v10:0xA00" "m_v11b:0xB00" "m_v10b:0xA00"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 400 python bench.py --pipeline 1 --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
