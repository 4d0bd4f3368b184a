#!/bin/bash
# Round 5 (k): K0 slow-atom pass (32-byte window), strings decoded into LDS, rank sort for <= 128 keys --
# byte-identical tests, then K0's rate and phase split on a config5-sized batch.
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
cat $O/k0_bench.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc1 -o p1 --output-format csv -- python tools/k0_bench.py --reps 3 > $O/pmc1.json 2> $O/pmc1.log || { tail -20 $O/pmc1.log; exit 1; }
echo done
