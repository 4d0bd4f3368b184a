#!/bin/bash
# Round 5 (l): K0 -- tree-phase positions, slow-atom pass, LDS rank sort, small-document phase 5 from LDS:
# byte-identical tests, then an interleaved A/B of the same K0 at 8 waves/SIMD (64 VGPRs, spills) and 7 (72, none).
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
for r in 1 2; do
  for w in 8 7; do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_w${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --profile --lib kcp_amd/_exp/libgpudiff_w$w.so > $O/k0_w${w}_r$r.json 2> $O/k0_w${w}_r$r.log || { tail -20 $O/k0_w${w}_r$r.log; exit 1; }
    echo "w$w r$r $(cut -c1-200 $O/k0_w${w}_r$r.json)"
  done
done
echo done
