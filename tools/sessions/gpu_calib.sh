#!/bin/bash
# FETCH_SIZE calibration of K2's access patterns + kernel times, the 1-GPU
# strong-scaling proxy (the N = 8 shard size: 1.25M pairs / 12.5k clusters)
# and the RCCL collective test.  Every GPU step time-limited; stop at the first failure.
set -eo pipefail
R=$(pwd); O=$R/gpurun_out/calib; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $R/tools/calib_fetch > $O/calib.txt 2>&1
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $R/tools/calib_fetch >> $O/calib.txt 2>&1
cd $R
timeout -k 10 200 python bench.py --pairs 1250000 --clusters 12500 --no-cpu-baseline --steps 50 > $O/bench_1p25M.json 2> $O/bench_1p25M.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_collective.py -q --timeout 120 --timeout-method thread > $O/collective.log 2>&1
tail -1 $O/collective.log
