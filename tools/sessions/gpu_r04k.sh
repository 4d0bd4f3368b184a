#!/bin/bash
# Round 4 (k): JSON-in with K0 launched per uploaded chunk: the JSON-in test, rates + phases, then a kernel +
# memory-copy trace of steady-state device-encode batches (where the 26 ms of a 131k-pair batch go).
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_json_in.py tests/test_gpu_write_plan.py tests/test_gpu_tokenize.py tests/test_gpu_store.py tests/test_gpu_upsert.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/json_in_probe.py > $O/json_in.json 2> $O/json_in.log || { tail -20 $O/json_in.log; exit 1; }
cat $O/json_in.json
R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $R/tools/json_in_probe.py --device-only 4 > $R/$O/trace_probe.json 2> $R/$O/trace_probe.log || { tail -20 $R/$O/trace_probe.log; exit 1; }
cat $R/$O/trace_probe.json
