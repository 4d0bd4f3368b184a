#!/bin/bash
# Round 6 (ao): phase profiles of K10 / K11 / K13 at the final sources (where the per-document tree programs spend
# their time after round 6's sweeps).
set -o pipefail
O=gpurun_out/r06ao; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k10_profile.py > $O/k10_profile.txt 2>&1 || { tail -20 $O/k10_profile.txt; exit 1; }
cat $O/k10_profile.txt
timeout -k 10 300 python -u tools/k11_profile.py 250000 > $O/k11_profile.txt 2>&1 || { tail -20 $O/k11_profile.txt; exit 1; }
cat $O/k11_profile.txt
timeout -k 10 300 python -u tools/k13_profile.py > $O/k13_profile.txt 2>&1 || { tail -20 $O/k13_profile.txt; exit 1; }
cat $O/k13_profile.txt
echo done
