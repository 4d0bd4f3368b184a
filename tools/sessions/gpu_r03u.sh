#!/bin/bash
# Round 3: config4 K2 hand-out A/B -- late tickets (no tail prefetch) and item sizes
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 400 python tools/ab_k2.py --config config4 --pairs 100000 --clusters 1000 --rounds 7 \
  --variants def=0,late=0x10,ipw16=0x30000000,ipw16late=0x30000010,ipw4late=0x10000010,ipw8late=0x20000010 \
  > $O/ab_c4.json 2> $O/ab_c4.log || { tail -20 $O/ab_c4.log; exit 1; }
python -c "
import json; d=json.load(open('$O/ab_c4.json'))
for k,v in d['variants'].items(): print(k, round(v['pass_ms_median'],4), round(v['k2_span_ms'],4), round(v['join_exposed_ms'],4), round(v['emit_ms'],4))"
