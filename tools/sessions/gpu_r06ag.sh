#!/bin/bash
# Round 6 (ag): K11 / K13 phase profiles at the final front end (per-phase wall-clock ticks summed over waves).
set -o pipefail
O=gpurun_out/r06ag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k11_profile.py 250000 > $O/k11_profile.txt 2>&1 || { tail -20 $O/k11_profile.txt; exit 1; }
cat $O/k11_profile.txt
timeout -k 10 300 python -u tools/k13_profile.py > $O/k13_profile.txt 2>&1 || { tail -20 $O/k13_profile.txt; exit 1; }
cat $O/k13_profile.txt
echo done
