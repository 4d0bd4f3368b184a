#!/bin/bash
# Round 6 (x): the Go store-flush restatement through a device-encode store (zero copy) and the store tests.
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_goshim.py tests/test_gpu_store.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
echo done
