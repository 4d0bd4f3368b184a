#!/bin/bash
# Round 5 (i): K0 tree phase with token batches prefetched; K0's instruction mix and wave states (SQ counters, one
# pass each) on a config5-sized batch -- issue-bound or memory-waiting?
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
cat $O/k0_bench.json
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list failed"
grep -oE "SQ_[A-Z_0-9]+" $O/counters.txt | sort -u > $O/sq_counters.txt || true
wc -l $O/sq_counters.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU -d $O/pmc1 -o p1 --output-format csv -- python tools/k0_bench.py --reps 3 > $O/pmc1.json 2> $O/pmc1.log || { tail -20 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d $O/pmc2 -o p2 --output-format csv -- python tools/k0_bench.py --reps 3 > $O/pmc2.json 2> $O/pmc2.log || { tail -20 $O/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE -d $O/pmc3 -o p3 --output-format csv -- python tools/k0_bench.py --reps 3 > $O/pmc3.json 2> $O/pmc3.log || { tail -20 $O/pmc3.log; exit 1; }
echo done
