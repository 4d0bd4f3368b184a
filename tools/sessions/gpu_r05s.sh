#!/bin/bash
# Round 5 (s): config 5's 12-s time-based watch replay with the round's K0 (events/s, latency, staging / K0 shares).
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config config5 --seconds 12 > $O/config5_12s.json 2> $O/config5_12s.log || { tail -30 $O/config5_12s.log; exit 1; }
cut -c1-600 $O/config5_12s.json
