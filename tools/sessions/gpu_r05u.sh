#!/bin/bash
# Round 5 (u): K0 after the scalar-unit work (select-form tree, branch-free hash steps and phase-5 loads):
# byte-identical tests, K0's rate and phase split, and the per-phase SQ counts again (early-exit builds s0..s4, s9).
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_upsert.py tests/test_gpu_rollup.py tests/test_gpu_negotiate.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
cut -c1-200 $O/k0_bench.json
for v in s0 s1 s2 s3 s4 s9; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc_$v -o p --output-format csv -- python tools/k0_bench.py --reps 2 --lib kcp_amd/_exp/libgpudiff_$v.so > $O/pmc_$v.json 2> $O/pmc_$v.log || { tail -20 $O/pmc_$v.log; exit 1; }
  echo "pmc $v ok"
done
echo done
