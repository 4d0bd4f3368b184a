#!/bin/bash
# K2 hand-out tunings at one rank's N = 8 share (1.25M pairs) and at 10M (flags only, in-process A/B).
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 400 python tools/ab_k2.py --config config3 --pairs 1250000 --clusters 12500 --rounds 5 --passes 5 --variants "def=0,tail8=0x80,q4=0x50,q1=0x20,ipw8=0x20000000,ipw16=0x30000000" > $O/ab_share.json 2> $O/ab_share.log || { tail -20 $O/ab_share.log; exit 1; }
python -c "
import json; d=json.load(open('$O/ab_share.json'))
for k,v in d['variants'].items(): print('share', k, round(v['pass_ms_median'],4), round(v['k2_span_ms'],4))"
timeout -k 10 400 python tools/ab_k2.py --config config2 --rounds 4 --passes 5 --variants "def=0,tail8=0x80,q4=0x50,ipw8=0x20000000,ipw16=0x30000000" > $O/ab_c2.json 2> $O/ab_c2.log || { tail -20 $O/ab_c2.log; exit 1; }
python -c "
import json; d=json.load(open('$O/ab_c2.json'))
for k,v in d['variants'].items(): print('c2', k, round(v['pass_ms_median'],4), round(v['k2_span_ms'],4))"
