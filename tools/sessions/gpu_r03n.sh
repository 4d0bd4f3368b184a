#!/bin/bash
# Full -m gpu suite + smoke at HEAD, then config4 segmentation x deep-join A/B.
set -o pipefail
O=${O:-gpurun_out/r03n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python tools/ab_k2.py --config config4 --pairs 100000 --clusters 1000 --rounds 5 --passes 3 --variants "d2048=0,d2048s2=0x20000,d2048s4=0x40000,fused=0x40000000,fuseds2=0x40020000" > $O/ab_c4.json 2> $O/ab_c4.log || { tail -20 $O/ab_c4.log; exit 1; }
python -c "
import json; d=json.load(open('$O/ab_c4.json'))
for k,v in d['variants'].items(): print(k, round(v['pass_ms_median'],4), round(v['k2_span_ms'],4), round(v['join_exposed_ms'],4))"
