#!/bin/bash
# Round 6 (q): the §8(f) kernels at the round-6 front end: each side bench's line (CPU baseline
# included) and a rocprofv3 kernel trace + stats of the same command (short run, no CPU legs).
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
run() {  # name, bench args...
  local N=$1; shift
  mkdir -p $O/$N
  timeout -k 10 400 python -u bench.py "$@" --cpu-seconds 6 > $O/$N/bench.json 2> $O/$N/bench.log || { tail -30 $O/$N/bench.log; return 1; }
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$O/$N/kt -o run --output-format csv -- \
      python3 $ROOT/bench.py "$@" --no-cpu-baseline --steps 5 > $ROOT/$O/$N/kt_bench.json 2> $ROOT/$O/$N/kt_bench.log ) || { tail -30 $O/$N/kt_bench.log; return 1; }
  f=$(find $O/$N/kt -name '*kernel_stats.csv' | head -n 1); cp "$f" $O/$N/kernel_stats.csv
  python -c "
import json,csv
d=json.loads(open('$O/$N/bench.json').read().strip().splitlines()[-1])
print('$N', round(d['value']/1e6,3), d['unit'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'build', d.get('build_id'))
for r in csv.DictReader(open('$O/$N/kernel_stats.csv')):
    if float(r['TotalDurationNs'])>1e6: print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,4), 'ms')
"
}
run upsert --config upsert || exit 1
run rollup --config rollup --steps 10 || exit 1
run negotiate_api --config negotiate --kind api --steps 10 || exit 1
run negotiate_crd --config negotiate --kind crd --steps 10 || exit 1
run negotiate_mixed --config negotiate --kind mixed --steps 10 || exit 1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
echo done
