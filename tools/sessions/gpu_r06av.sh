#!/bin/bash
# Round 6 (av): the final sources (K14's word compares in) -- the whole GPU suite and smoke(), then the negotiation
# benches' lines (CPU baselines included) with a rocprofv3 kernel trace + stats of each command.
set -o pipefail
O=gpurun_out/r06av; mkdir -p $O
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.txt 2>&1 || { tail -60 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
run() {  # name, bench args...
  local N=$1; shift
  mkdir -p $O/$N
  timeout -k 10 400 python -u bench.py "$@" --cpu-seconds 6 > $O/$N/bench.json 2> $O/$N/bench.log || { tail -30 $O/$N/bench.log; return 1; }
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$O/$N/kt -o run --output-format csv -- \
      python3 $ROOT/bench.py "$@" --no-cpu-baseline --steps 5 > $ROOT/$O/$N/kt_bench.json 2> $ROOT/$O/$N/kt_bench.log ) || { tail -30 $O/$N/kt_bench.log; return 1; }
  f=$(find $O/$N/kt -name '*kernel_stats.csv' | head -n 1); cp "$f" $O/$N/kernel_stats.csv; rm -rf $O/$N/kt
  python -c "
import json,csv
d=json.loads(open('$O/$N/bench.json').read().strip().splitlines()[-1])
print('$N', round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],4), d.get('kernels_ms'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'build', d.get('build_id'), json.dumps(d.get('checks')))
for r in csv.DictReader(open('$O/$N/kernel_stats.csv')):
    if float(r['TotalDurationNs'])>1e6: print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,4), 'ms')
"
}
run negotiate_api --config negotiate --kind api --steps 10 || exit 1
run negotiate_crd --config negotiate --kind crd --steps 10 || exit 1
run negotiate_mixed --config negotiate --kind mixed --steps 10 || exit 1
echo done
