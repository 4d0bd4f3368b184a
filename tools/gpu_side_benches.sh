#!/bin/bash
# The §8(f) side benches on the GPU box (write path, roll-up, negotiation of
# the three kinds), bench lines only; every step time-limited, stop at the
# first failure.
set -o pipefail
O=${O:-gpurun_out/side}; mkdir -p $O
timeout -k 10 300 python bench.py --config upsert --cpu-seconds 4 > $O/bench_upsert.json 2> $O/bench_upsert.log || { tail -30 $O/bench_upsert.log; exit 1; }
timeout -k 10 400 python bench.py --config rollup --steps 10 --cpu-seconds 6 > $O/bench_rollup.json 2> $O/bench_rollup.log || { tail -30 $O/bench_rollup.log; exit 1; }
for K in api crd mixed; do
  timeout -k 10 400 python bench.py --config negotiate --kind $K --steps 10 --cpu-seconds 6 > $O/neg_$K.json 2> $O/neg_$K.log || { tail -30 $O/neg_$K.log; exit 1; }
done
timeout -k 10 400 python bench.py --config config5 --cpu-seconds 6 > $O/bench_config5.json 2> $O/bench_config5.log || { tail -30 $O/bench_config5.log; exit 1; }
for f in $O/*.json; do echo "$f"; python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['unit'], d.get('kernels_ms'), (d.get('cpu_baseline') or {}).get('value'))"; done
