#!/bin/bash
# K11/K12 (Deployment splitter roll-up) on the GPU box: parity tests, bench line, kernel stats.
set -o pipefail
O=${O:-gpurun_out/r01i}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollup.py -v --timeout 120 --timeout-method thread > $O/pytest_rollup.log 2>&1 || { tail -40 $O/pytest_rollup.log; exit 1; }
tail -2 $O/pytest_rollup.log
timeout -k 10 500 python bench.py --config rollup --steps 10 --cpu-seconds 8 > $O/bench_rollup.json 2> $O/bench_rollup.log || { tail -30 $O/bench_rollup.log; exit 1; }
cat $O/bench_rollup.json
R=$(pwd)
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --config rollup --no-cpu-baseline --steps 5 > $R/$O/kt_bench.json 2> $R/$O/kt_bench.log || { tail -20 $R/$O/kt_bench.log; exit 1; }
find $R/$O/kt -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200
