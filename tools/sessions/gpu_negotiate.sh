#!/bin/bash
# K13/K14 (API-negotiation update classifier) on the GPU box: parity tests, bench line, kernel stats.
set -o pipefail
O=${O:-gpurun_out/r01l}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_negotiate.py -v --timeout 120 --timeout-method thread > $O/pytest_negotiate.log 2>&1 || { tail -40 $O/pytest_negotiate.log; exit 1; }
tail -2 $O/pytest_negotiate.log
timeout -k 10 400 python bench.py --config negotiate --steps 10 > $O/bench_negotiate.json 2> $O/bench_negotiate.log || { tail -30 $O/bench_negotiate.log; exit 1; }
cat $O/bench_negotiate.json
R=$(pwd)
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --config negotiate --no-cpu-baseline --steps 5 > $R/$O/kt_bench.json 2> $R/$O/kt_bench.log || { tail -20 $R/$O/kt_bench.log; exit 1; }
find $R/$O/kt -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200
