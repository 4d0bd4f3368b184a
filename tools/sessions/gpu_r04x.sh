#!/bin/bash
# Round 4 (x): config4 item size with the x16 kernel: 8 items per resident wave (4-pair items, the default) vs
# 16 (2-pair items, GPUDIFF_OPT_K2_ITEMS_SHIFT = 3), both with the single-pair largest-first round.
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
export TMPDIR=/tmp
for v in "c4_i8:0" "c4_i16:0x30000000" "c4_i8b:0" "c4_i16b:0x30000000"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python bench.py --pipeline 1 --config config4 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
