#!/bin/bash
# Round 4 (o): K2 variant 10 (the default kernel with 8 chunks a side in flight, 3 waves/SIMD) vs the default
# (4 in flight, 4 waves/SIMD) on config4 (the tail's per-wave rate) and config3's byte-heaviest N = 8 share.
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "variants or largest_first" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "c4_v0:0" "c4_v10:0xA00" "c4_v0b:0" "c4_v10b:0xA00"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python bench.py --pipeline 1 --config config4 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
for v in "sh_v0:0" "sh_v10:0xA00"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python bench.py --pipeline 1 --emulate-world 8 --steps 40 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
