#!/bin/bash
# Round 4 (g): the default bench line at HEAD (two passes in flight, isolated-pass kernel times, JSON-in phase
# split), the gloo two-rank rehearsal test, and the 10M encoder-independent tree-walk check with K0.
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_rehearsal.py tests/test_gpu_collective.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -40 $O/pytest_dist.log; exit 1; }
tail -1 $O/pytest_dist.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['format']['frac'], d['kernels_ms']); print(d['json_in'])"
timeout -k 10 900 python tools/full_tree_check.py --k0 > $O/full_tree_check.json 2> $O/full_tree_check.log || { tail -30 $O/full_tree_check.log; exit 1; }
cat $O/full_tree_check.json
