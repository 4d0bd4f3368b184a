#!/bin/bash
# Round-3 final profile at HEAD: config3 bench + rocprofv3 kernel stats + FETCH/WRITE passes + bench with
# roofline.traffic (tools/profile_round.sh), config4 kernel stats + PMC, config2 / N=8-share bench lines.
set -o pipefail
bash tools/profile_round.sh r03o || exit 1
bash tools/profile_config.sh config4 r03o || exit 1
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 300 python bench.py --config config4 --steps 10 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c4.json 2> $O/bench_c4.log || { tail -20 $O/bench_c4.log; exit 1; }
timeout -k 10 300 python bench.py --config config2 --steps 20 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c2.json 2> $O/bench_c2.log || { tail -20 $O/bench_c2.log; exit 1; }
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_share.json 2> $O/bench_share.log || { tail -20 $O/bench_share.log; exit 1; }
for f in $O/bench_c4.json $O/bench_c2.json $O/bench_share.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms'])"; done
