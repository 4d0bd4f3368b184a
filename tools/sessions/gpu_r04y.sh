#!/bin/bash
# Round 4 (y): the round-end profile at the final kernels (config3 bench line, rocprofv3 kernel stats, FETCH /
# WRITE passes, pmc_summary, the line with traffic attached), then config4's profile and two-pass step.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 bash tools/profile_round.sh r04y || exit 1
timeout -k 10 600 bash tools/profile_config.sh config4 r04y || exit 1
timeout -k 10 200 python bench.py --config config4 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 > gpurun_out/prof_r04y/bench_c4_p2.json 2> gpurun_out/prof_r04y/bench_c4_p2.log || { tail -20 gpurun_out/prof_r04y/bench_c4_p2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/prof_r04y/bench_c4_p2.json')); print('c4 p2', d['value'], d['ms_per_step'])"
