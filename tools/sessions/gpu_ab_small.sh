#!/bin/bash
# K2 item-size A/B at the N = 8 strong-scaling shard size and at full size, plus
# the FETCH_SIZE calibration of segmented streams.  Time-limited steps, stop at the first failure.
set -eo pipefail
R=$(pwd); O=$R/gpurun_out/ab_small; mkdir -p $O
export TMPDIR=/tmp
V="base=0,items8=0x20000000,items16=0x30000000"
timeout -k 10 300 python tools/ab_k2.py --pairs 1250000 --clusters 12500 --rounds 5 --passes 5 --variants $V > $O/ab_1p25M.json 2> $O/ab_1p25M.log
cat $O/ab_1p25M.json
timeout -k 10 300 python tools/ab_k2.py --pairs 10000000 --clusters 100000 --rounds 3 --passes 3 --variants $V > $O/ab_10M.json 2> $O/ab_10M.log
cat $O/ab_10M.json
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $R/tools/calib_fetch > $O/calib.txt 2>&1
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $R/tools/calib_fetch >> $O/calib.txt 2>&1
