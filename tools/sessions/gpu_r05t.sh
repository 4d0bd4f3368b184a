#!/bin/bash
# Round 5 (t): K0 with scalar level loops -- byte-identical tests (K0 and the modes sharing its tree phase), K0's
# rate and phase split, and the K10 / K11 / K13 benches that share the tree phase.
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py tests/test_gpu_upsert.py tests/test_gpu_rollup.py tests/test_gpu_negotiate.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
cut -c1-300 $O/k0_bench.json
echo done
