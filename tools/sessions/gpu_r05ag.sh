#!/bin/bash
# Round 5 (ag): round-end checks at the final sources -- the whole -m gpu suite and smoke, K0's final rate on the
# config5 batch (kernel trace + stats; A/B against r05ae's kernel, which also stored small documents' hashes to the
# scratch), config 5's 12-s replay with that K0, and the default bench line.
set -o pipefail
O=gpurun_out/r05ag; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for r in 1 2; do
  for v in new dpp; do
    L=""; [ $v != new ] && L="--lib kcp_amd/_exp/libgpudiff_$v.so"
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt_${v}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --profile $L > $O/k0_bench_${v}_r$r.json 2> $O/k0_bench_${v}_r$r.log || { tail -20 $O/k0_bench_${v}_r$r.log; exit 1; }
  done
done
timeout -k 10 400 python -u bench.py --config config5 --seconds 12 > $O/config5_12s.json 2> $O/config5_12s.log || { tail -30 $O/config5_12s.log; exit 1; }
cut -c1-300 $O/config5_12s.json
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -30 $O/bench_default.log; exit 1; }
cut -c1-400 $O/bench_default.json
echo done
