#!/bin/bash
# Round 5 (v): is K0 stalled on instruction fetch? SQC instruction-cache hits / misses and SQ ifetch over one
# config5-sized K0 launch (K0's code is ~11k instructions; the I-cache is shared by two CUs).
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $O/pmc_ic -o p --output-format csv -- python tools/k0_bench.py --reps 2 > $O/pmc_ic.json 2> $O/pmc_ic.log || { tail -20 $O/pmc_ic.log; exit 1; }
echo ic ok
timeout -s KILL 150 rocprofv3 --pmc SQ_IFETCH_LEVEL SQ_INSTS SQ_BUSY_CYCLES SQ_WAVES -d $O/pmc_if -o p --output-format csv -- python tools/k0_bench.py --reps 2 > $O/pmc_if.json 2> $O/pmc_if.log || { tail -20 $O/pmc_if.log; exit 1; }
echo done
