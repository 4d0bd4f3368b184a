#!/bin/bash
# Round 5 (o): K0 at HEAD -- byte-identical tests; its instruction mix phase by phase (SQ counters of builds that
# stop after phase k, s0..s4, and the whole kernel, s9: differences are per-phase counts); 8 vs 7 waves/SIMD (w7:
# 72 VGPRs, no spills) interleaved.
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
for v in s0 s1 s2 s3 s4 s9; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc_$v -o p --output-format csv -- python tools/k0_bench.py --reps 2 --lib kcp_amd/_exp/libgpudiff_$v.so > $O/pmc_$v.json 2> $O/pmc_$v.log || { tail -20 $O/pmc_$v.log; exit 1; }
  echo "pmc $v ok"
done
for r in 1 2; do
  for w in s9 w7; do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --lib kcp_amd/_exp/libgpudiff_$w.so > $O/k0_${w}_r$r.json 2> $O/k0_${w}_r$r.log || { tail -20 $O/k0_${w}_r$r.log; exit 1; }
    echo "$w r$r done"
  done
done
echo done
