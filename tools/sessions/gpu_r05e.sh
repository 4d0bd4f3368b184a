#!/bin/bash
# Round 5 (e): K0 workgroup shape A/B (4 / 2 / 1 documents per workgroup), kernel trace of each, interleaved.
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for w in 4 2 1; do
  lib=""; [ $w != 4 ] && lib="--lib kcp_amd/_exp/libgpudiff_wpb$w.so"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_w${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py $lib --reps 4 > $O/k0_w${w}_r$r.json 2> $O/k0_w${w}_r$r.log || { tail -20 $O/k0_w${w}_r$r.log; exit 1; }
  python3 -c "
import csv,sys
r=[x for x in csv.DictReader(open('$O/kt_w${w}_r$r/k0_kernel_trace.csv')) if 'encode_docs' in x['Kernel_Name']]
print('wpb $w round $r', [round((int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e6,3) for x in r])"
done
done
