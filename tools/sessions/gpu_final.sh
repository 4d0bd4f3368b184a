#!/bin/bash
# Round-end rehearsal on the GPU box: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
O=${O:-gpurun_out/r01j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_config3.json 2> $O/bench_config3.log && cat $O/bench_config3.json
