#!/bin/bash
# Round 5 (aj): the tree phase's parent info and base gathered by one cross-lane read instead of two -- the whole
# -m gpu suite and smoke at these sources, blob diff, then K0's rate A/B on one box, interleaved: new vs r05ai.
set -o pipefail
O=gpurun_out/r05aj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u tools/k0_diff.py > $O/k0_diff.txt 2>&1 || { tail -20 $O/k0_diff.txt; exit 1; }
grep differing $O/k0_diff.txt | cut -c1-200
for r in 1 2; do
  for v in new r05ai; do
    L=""; [ $v != new ] && L="--lib kcp_amd/_exp/libgpudiff_$v.so"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt_${v}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --profile $L > $O/k0_bench_${v}_r$r.json 2> $O/k0_bench_${v}_r$r.log || { tail -20 $O/k0_bench_${v}_r$r.log; exit 1; }
  done
done
echo done
