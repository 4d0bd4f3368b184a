#!/bin/bash
# Round 5 (h): K0 blob sizes from the values phase -- byte-identical to the host encoder (K0 tests, stores, JSON in, every GPU test),
# then K0's rate on a config5-sized batch (kernel trace) and its phase split.
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tokenize.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
cat $O/k0_bench.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
command -v go || echo "no go toolchain on the box"
