#!/bin/bash
# Round 5 (af): K0's rank sort on 32-bit keys with duplicates found by reading the ids back -- byte-identical tests
# over every mode, blob diff, then K0's rate A/B on one box, interleaved: new vs dpp (r05ae's kernel).
set -o pipefail
O=gpurun_out/r05af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_upsert.py tests/test_gpu_rollup.py tests/test_gpu_negotiate.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 python -u tools/k0_diff.py > $O/k0_diff.txt 2>&1 || { tail -20 $O/k0_diff.txt; exit 1; }
grep differing $O/k0_diff.txt | cut -c1-200
for r in 1 2; do
  for v in new dpp; do
    L=""; [ $v != new ] && L="--lib kcp_amd/_exp/libgpudiff_$v.so"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt_${v}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --profile $L > $O/k0_bench_${v}_r$r.json 2> $O/k0_bench_${v}_r$r.log || { tail -20 $O/k0_bench_${v}_r$r.log; exit 1; }
  done
done
echo done
