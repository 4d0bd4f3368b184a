#!/bin/bash
# Round 4 (a): exact scratch for whole deferrals -- the -m gpu suite, then the N=8 share bench
# (K3 now carries the whole-deferral join: its occupancy-sized grid must not slow the pass).
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_share.json 2> $O/bench_share.log || { tail -20 $O/bench_share.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_share.json')); print('share', d['value'], d['ms_per_step'], d['kernels_ms'])"
