#!/bin/bash
# Round 5 (y): round-end checks at the final sources -- the whole -m gpu suite and smoke, K0's final rate on the
# config5 batch (kernel trace + stats), and config 5's 12-s replay with that K0.
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 --output-format csv -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
cut -c1-200 $O/k0_bench.json
timeout -k 10 400 python -u bench.py --config config5 --seconds 12 > $O/config5_12s.json 2> $O/config5_12s.log || { tail -30 $O/config5_12s.log; exit 1; }
cut -c1-300 $O/config5_12s.json
echo done
