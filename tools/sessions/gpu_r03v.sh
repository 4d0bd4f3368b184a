#!/bin/bash
# Round 3: deep-pair K2 items largest first -- parity (deep tests, then the -m gpu suite), config4 A/B and
# the K2 wave timeline with and without the order
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "deep" > $O/pytest_deep.log 2>&1 || { tail -30 $O/pytest_deep.log; exit 1; }
tail -1 $O/pytest_deep.log
timeout -k 10 400 python tools/ab_k2.py --config config4 --pairs 100000 --clusters 1000 --rounds 7 \
  --variants def=0,nolpt=0x2 > $O/ab_c4.json 2> $O/ab_c4.log || { tail -20 $O/ab_c4.log; exit 1; }
python -c "
import json; d=json.load(open('$O/ab_c4.json'))
for k,v in d['variants'].items(): print(k, round(v['pass_ms_median'],4), round(v['k2_span_ms'],4), round(v['join_exposed_ms'],4), round(v['emit_ms'],4))"
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 > $O/wave_c4.json 2> $O/wave_c4.log || { tail -20 $O/wave_c4.log; exit 1; }
python -c "
import json; d=json.load(open('$O/wave_c4.json'))['variant14']; print('wave c4 span', d['span_us'], 'end', d['end_us'], 'busy', round(d['busy_frac_of_span'],3))"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
