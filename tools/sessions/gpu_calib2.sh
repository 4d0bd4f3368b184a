#!/bin/bash
set -eo pipefail
R=$(pwd); O=$R/gpurun_out/calib2; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $R/tools/calib_fetch > $O/calib.txt 2>&1
timeout -k 10 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $R/tools/calib_fetch >> $O/calib.txt 2>&1
