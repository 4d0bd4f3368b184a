#!/bin/bash
# Round 6 (ax): the default bench line (what the driver runs) and config2's at the final build.
set -o pipefail
O=gpurun_out/r06ax; mkdir -p $O
export TMPDIR=/tmp
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],4), 'frac', (d.get('roofline') or {}).get('frac'), 'pass', (d.get('kernels_ms') or {}).get('diff_pass'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), d.get('box'), d.get('build_id'))"; }
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -30 $O/bench_default.log; exit 1; }
line $O/bench_default.json
timeout -k 10 400 python -u bench.py --config config2 --cpu-seconds 8 > $O/config2.json 2> $O/config2.log || { tail -30 $O/config2.log; exit 1; }
line $O/config2.json
echo done
