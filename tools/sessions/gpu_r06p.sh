#!/bin/bash
# Round 6 (p): the BASELINE configurations' bench lines at the final sources (one box): config1 (10k Deployment pairs,
# CPU baseline on the same pairs), config2 and config4 (two passes in flight, CPU baselines), config5 watch replay
# 12 s staged and zero-copy.  (config3's line and profiles: r06o.)
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],4), 'frac', (d.get('roofline') or {}).get('frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), d.get('build_id'))"; }
timeout -k 10 300 python -u bench.py --config config1 --cpu-seconds 8 > $O/config1.json 2> $O/config1.log || { tail -30 $O/config1.log; exit 1; }
line $O/config1.json
timeout -k 10 400 python -u bench.py --config config2 --cpu-seconds 8 > $O/config2.json 2> $O/config2.log || { tail -30 $O/config2.log; exit 1; }
line $O/config2.json
timeout -k 10 400 python -u bench.py --config config4 --cpu-seconds 8 > $O/config4.json 2> $O/config4.log || { tail -30 $O/config4.log; exit 1; }
line $O/config4.json
for m in staged zc; do
  A=""; [ $m = zc ] && A="--zero-copy"
  timeout -k 10 400 python -u bench.py --config config5 --seconds 12 $A --cpu-seconds 4 > $O/config5_$m.json 2> $O/config5_$m.log || { tail -30 $O/config5_$m.log; exit 1; }
  line $O/config5_$m.json
done
echo done
