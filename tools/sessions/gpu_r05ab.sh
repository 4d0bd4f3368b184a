#!/bin/bash
# Round 5 (ab): K0 with one XXH64 per node and LDS ranks up to 256 keys -- byte-identical tests (K0 and the modes
# sharing its front end), blob diff, K0's rate (two runs).
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_upsert.py tests/test_gpu_rollup.py tests/test_gpu_negotiate.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 python -u tools/k0_diff.py > $O/k0_diff.txt 2>&1 || { tail -20 $O/k0_diff.txt; exit 1; }
grep differing $O/k0_diff.txt | cut -c1-200
for r in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt_r$r -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench_r$r.json 2> $O/k0_bench_r$r.log || { tail -20 $O/k0_bench_r$r.log; exit 1; }
done
echo done
