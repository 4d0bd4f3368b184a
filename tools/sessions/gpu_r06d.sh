#!/bin/bash
# Round 6 (d): config 5 (watch replay, 12 s each) with the events' JSON staged by the engine vs written into
# engine-pinned memory (store-mode zero copy), alternating on one box.
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in staged zc; do
    A=""; [ $m = zc ] && A="--zero-copy"
    timeout -k 10 400 python -u bench.py --config config5 --seconds 12 $A --cpu-seconds 4 > $O/config5_${m}_$k.json 2> $O/config5_${m}_$k.log || { tail -30 $O/config5_${m}_$k.log; exit 1; }
    python -c "
import json,sys
d=json.loads(open('$O/config5_${m}_$k.json').read().strip().splitlines()[-1])
b=d['batch_ms']
print('$m', $k, round(d['value']/1e6,3), 'M ev/s', 'h2d', round(d['h2d_gbps'],1), 'lat', {k: round(v,2) for k,v in d['latency_ms'].items() if k!='def'}, 'copy', round(b['submit_split']['submit_copy_ms'],2), 'h2d_ms', round(b['h2d'],2), 'k0', round(b['k0_encode'],2), 'zc', d['config'].get('zero_copy_batches'), d['checks'])
"
  done
done
echo done
