#!/bin/bash
# Round 5 (w): is K0's blob phase held up by its stores? Timing-only builds (outputs invalid): nc = no key / tail
# copies, ns = no blob stores at all (values kept live), against the unchanged kernel (b1); interleaved, with the
# issue-stall counter.
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for w in b1 nc ns; do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --lib kcp_amd/_exp/libgpudiff_$w.so > $O/k0_${w}_r$r.json 2> $O/k0_${w}_r$r.log || { tail -20 $O/k0_${w}_r$r.log; exit 1; }
    echo "$w r$r done"
  done
done
for w in b1 ns; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d $O/pmc_$w -o p --output-format csv -- python tools/k0_bench.py --reps 2 --lib kcp_amd/_exp/libgpudiff_$w.so > $O/pmc_$w.json 2> $O/pmc_$w.log || { tail -20 $O/pmc_$w.log; exit 1; }
done
echo done
