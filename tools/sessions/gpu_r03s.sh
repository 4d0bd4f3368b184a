#!/bin/bash
# Round 3: two-launch scans (tile sums -> apply with in-workgroup tile base) -- -m gpu suite, smoke, share and
# config3 bench lines without the CPU leg.
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_share.json 2> $O/bench_share.log || { tail -20 $O/bench_share.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_c3.json 2> $O/bench_c3.log || { tail -20 $O/bench_c3.log; exit 1; }
for f in $O/bench_share.json $O/bench_c3.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernels_ms'])"; done
