#!/bin/bash
# Round 6 (as): bench.py warms the timed loop's own shape (two passes in flight) before timing, 40 steps by default:
# the world-2 rehearsal test (the collective's warm steps), then the default line twice (what the driver runs).
set -o pipefail
O=gpurun_out/r06as; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist_rehearsal.py \
  > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for k in 1 2; do
timeout -k 10 400 python -u bench.py > $O/bench_default_$k.json 2> $O/bench_default_$k.log || { tail -30 $O/bench_default_$k.log; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench_default_$k.json').read().strip().splitlines()[-1])
print('default', round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],4), 'frac', d['roofline']['frac'], 'pass', d['kernels_ms']['diff_pass'], 'cpu', d['cpu_baseline']['value'], d.get('box'), d.get('build_id'))"
done
echo done
