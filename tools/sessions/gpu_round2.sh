#!/bin/bash
# Round-2 validation on the GPU box: the whole -m gpu suite, smoke(), the default bench line, the
# negotiation bench.  Each GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
O=${O:-gpurun_out/r02}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_config3.json 2> $O/bench_config3.log || { tail -30 $O/bench_config3.log; exit 1; }
cat $O/bench_config3.json
if [ -n "$NEG" ]; then
timeout -k 10 300 python bench.py --config negotiate > $O/bench_negotiate.json 2> $O/bench_negotiate.log || { tail -30 $O/bench_negotiate.log; exit 1; }
cat $O/bench_negotiate.json
fi
