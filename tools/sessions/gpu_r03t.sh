#!/bin/bash
# Round-3 final at HEAD (two-launch scans, one reset kernel per single-segment pass): -m gpu suite, smoke, then the round profile (config3 bench + rocprofv3 kernel stats +
# FETCH/WRITE passes + bench with roofline.traffic) and config4 kernel stats + PMC + bench line.
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh r03t > $O/profile_round.log 2>&1 || { tail -20 $O/profile_round.log; exit 1; }
bash tools/profile_config.sh config4 r03t || exit 1
timeout -k 10 300 python bench.py --config config4 --steps 10 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c4.json 2> $O/bench_c4.log || { tail -20 $O/bench_c4.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/prof_r03t/bench_traffic.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['format']['frac'], d['roofline']['traffic'])"
python -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms'])"
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_share.json 2> $O/bench_share.log || { tail -20 $O/bench_share.log; exit 1; }
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 --gather-world1 > $O/bench_share_gather.json 2> $O/bench_share_gather.log || { tail -20 $O/bench_share_gather.log; exit 1; }
for f in $O/bench_share.json $O/bench_share_gather.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernels_ms'])"; done
