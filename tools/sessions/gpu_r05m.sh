#!/bin/bash
# Round 5 (m): bisect a K0 blob difference (kat document 0) across three builds of K0 -- fc5705a (tests green),
# 237f90e (tree-phase positions, loop-free XXH64 batches), HEAD (LDS rank order, phase 5 from LDS) -- with
# tools/k0_diff.py, then their K0 rates (timing only).
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k0_diff.py --lib kcp_amd/_exp/libgpudiff_fc5705a.so --lib kcp_amd/_exp/libgpudiff_237f90e.so --lib kcp_amd/_exp/libgpudiff_HEAD.so > $O/k0_diff.txt 2>&1 || { tail -30 $O/k0_diff.txt; exit 1; }
cat $O/k0_diff.txt
for c in fc5705a HEAD; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_$c -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --profile --lib kcp_amd/_exp/libgpudiff_$c.so > $O/k0_$c.json 2> $O/k0_$c.log || { tail -20 $O/k0_$c.log; exit 1; }
  echo "$c $(cut -c1-200 $O/k0_$c.json)"
done
echo done
