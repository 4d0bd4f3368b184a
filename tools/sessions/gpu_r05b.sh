#!/bin/bash
# Round 5 (b): the whole -m gpu suite + smoke after retiring the A/B scaffolding (ABI 5), then the headline bench.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
echo bench done
