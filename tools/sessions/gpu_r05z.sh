#!/bin/bash
# Round 5 (z): interleaved A/B of K0 builds on one box: b0824b2 (r05u: 119 GB/s there), da30f27 (r05x: + branch-free
# values loop, one flattened blob copy, tree stores), HEAD (+ wave-parallel simple unescape), Yoc (HEAD with the two
# separate copy loops of b0824b2). Byte-identical check of HEAD and Yoc first (tools/k0_diff.py).
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k0_diff.py --lib kcp_amd/_exp/libgpudiff_HEAD.so --lib kcp_amd/_exp/libgpudiff_Yoc.so > $O/k0_diff.txt 2>&1 || { tail -30 $O/k0_diff.txt; exit 1; }
grep differing $O/k0_diff.txt | cut -c1-200
for r in 1 2; do
  for w in b0824b2 da30f27 HEAD Yoc; do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --profile --lib kcp_amd/_exp/libgpudiff_$w.so > $O/k0_${w}_r$r.json 2> $O/k0_${w}_r$r.log || { tail -20 $O/k0_${w}_r$r.log; exit 1; }
    echo "$w r$r done"
  done
done
echo done
