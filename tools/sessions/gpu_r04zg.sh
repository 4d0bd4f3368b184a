#!/bin/bash
# Round 4 (zg): interleaved A/B of streaming JSON-in: decoupled K0 stage (default) vs coupled vs one K0 stream,
# staged and zero copy; watch replay twice each with two / one K0 streams.
set -o pipefail
O=gpurun_out/r04zg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/json_in_ab.py > $O/ab_staged.json 2> $O/ab_staged.log || { tail -20 $O/ab_staged.log; exit 1; }
cat $O/ab_staged.json
timeout -k 10 400 python tools/json_in_ab.py --zero-copy > $O/ab_zc.json 2> $O/ab_zc.log || { tail -20 $O/ab_zc.log; exit 1; }
cat $O/ab_zc.json
for v in "c5_two:" "c5_one:GPUDIFF_K0_ONE_STREAM=1" "c5_two_b:" "c5_one_b:GPUDIFF_K0_ONE_STREAM=1"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 300 python bench.py --config config5 --no-cpu-baseline > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); b=d['batch_ms']; print('$n', d['value'], b['host_submit'], b['h2d'], b['k0_encode'])"
done
