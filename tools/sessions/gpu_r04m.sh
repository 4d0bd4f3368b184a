#!/bin/bash
# Round 4 (m): the whole -m gpu suite at HEAD, smoke, then watch replay (config5, device encode) after the
# per-chunk K0 launches.
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --config config5 > $O/config5.json 2> $O/config5.log || { tail -20 $O/config5.log; exit 1; }
cat $O/config5.json
