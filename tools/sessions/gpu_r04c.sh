#!/bin/bash
# Round 4 (c): debug the gloo two-rank rehearsal (node sets vs truth)
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 2 --pairs 100000 --clusters 1000 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --threads 8 > $O/n2.json 2> $O/n2.log; echo rc=$?
cat $O/n2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['checks'], indent=1)); print(d['config']['shard'])"
grep -v "^\[W\|Gloo" $O/n2.log | tail -30
