#!/bin/bash
# Round 5 (n): K0 blob differences after the path-table key-length fix (fx) and with phase 5's LDS path switched
# off (nt), section by section with the differing words (tools/k0_diff.py).
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k0_diff.py --lib kcp_amd/_exp/libgpudiff_fx.so --lib kcp_amd/_exp/libgpudiff_nt.so > $O/k0_diff.txt 2>&1 || { tail -30 $O/k0_diff.txt; exit 1; }
cat $O/k0_diff.txt
