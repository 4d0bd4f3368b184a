#!/bin/bash
# Round 5 (r): what stalls K0's blob phase (41% of a wave's cycles, mostly issue stalls, profiles/r05o): timing-only
# builds with the blob space's append atomic replaced by a fixed offset (na) and the key-byte copies as dword stores
# (dw), against the unchanged kernel (b0), interleaved.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for w in b0 na dw; do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --profile --lib kcp_amd/_exp/libgpudiff_$w.so > $O/k0_${w}_r$r.json 2> $O/k0_${w}_r$r.log || { tail -20 $O/k0_${w}_r$r.log; exit 1; }
    echo "$w r$r done"
  done
done
echo done
