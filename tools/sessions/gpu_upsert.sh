#!/bin/bash
# K10 (write path) on the GPU box: parity tests, bench line, kernel stats.
set -o pipefail
O=gpurun_out/k10b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_upsert.py -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --config upsert --cpu-seconds 4 > $O/bench_upsert.json 2> $O/bench_upsert.log || { tail -30 $O/bench_upsert.log; exit 1; }
cat $O/bench_upsert.json
R=$(pwd)
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --config upsert --no-cpu-baseline --sample 0 --steps 5 > $R/$O/kt_bench.json 2> $R/$O/kt_bench.log || { tail -20 $R/$O/kt_bench.log; exit 1; }
find $R/$O/kt -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200
