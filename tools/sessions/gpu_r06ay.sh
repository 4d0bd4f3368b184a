#!/bin/bash
# Round 6 (ay): config5 (zero copy; K0's key copies changed since r06an) and config4 at the final build.
set -o pipefail
O=gpurun_out/r06ay; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],4), 'frac', (d.get('roofline') or {}).get('frac'), 'h2d', d.get('h2d_gbps'), 'k0', (d.get('batch_ms') or {}).get('k0_encode'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), d.get('box'), d.get('build_id'))"; }
timeout -k 10 400 python -u bench.py --config config5 --seconds 12 --zero-copy --cpu-seconds 4 > $O/config5_zc.json 2> $O/config5_zc.log || { tail -30 $O/config5_zc.log; exit 1; }
line $O/config5_zc.json
timeout -k 10 400 python -u bench.py --config config4 --cpu-seconds 8 > $O/config4.json 2> $O/config4.log || { tail -30 $O/config4.log; exit 1; }
line $O/config4.json
echo done
