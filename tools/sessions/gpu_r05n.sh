#!/bin/bash
# Round 5 (n): K0 blob differences after the path-table key-length fix (fx), with phase 5's LDS path switched off
# (nt), and with level-pipelined hashing (lv / lvnt), section by section with the differing words
# (tools/k0_diff.py); then each build's K0 rate (timing only).
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k0_diff.py --lib kcp_amd/_exp/libgpudiff_fx.so --lib kcp_amd/_exp/libgpudiff_nt.so --lib kcp_amd/_exp/libgpudiff_lv.so --lib kcp_amd/_exp/libgpudiff_lvnt.so > $O/k0_diff.txt 2>&1 || { tail -30 $O/k0_diff.txt; exit 1; }
cat $O/k0_diff.txt
for c in fx nt lv lvnt; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_$c -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --profile --lib kcp_amd/_exp/libgpudiff_$c.so > $O/k0_$c.json 2> $O/k0_$c.log || { tail -20 $O/k0_$c.log; exit 1; }
  echo "$c $(cut -c1-120 $O/k0_$c.json)"
done
echo done
