#!/bin/bash
# Round 5 (ak): the bench lines at the final sources (r05ai's kernel; tests + smoke green there): the default bench
# line and config 5's 12-s replay.
set -o pipefail
O=gpurun_out/r05ak; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -30 $O/bench_default.log; exit 1; }
cut -c1-300 $O/bench_default.json
timeout -k 10 400 python -u bench.py --config config5 --seconds 12 > $O/config5_12s.json 2> $O/config5_12s.log || { tail -30 $O/config5_12s.log; exit 1; }
cut -c1-300 $O/config5_12s.json
echo done
