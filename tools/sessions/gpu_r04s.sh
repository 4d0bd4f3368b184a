#!/bin/bash
# Round 4 (s): final K2 -- a 10M pass (two in flight), the byte-heaviest N = 8 share with the world-1 collective
# (two passes / one), and the two-rank gloo rehearsal of the N > 1 bench path, in one session.
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
W="--weights-cache $R/$O/w8.npy"
timeout -k 10 400 python bench.py --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_10m.json 2> $O/bench_10m.log || { tail -30 $O/bench_10m.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_10m.json')); print('10M', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'])"
for v in "p2_gather:--pipeline 2 --gather-world1" "p1_gather:--pipeline 1 --gather-world1"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 python bench.py --emulate-world 8 $W --steps 100 $a --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share_$n.json 2> $O/share_$n.log || { tail -30 $O/share_$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/share_$n.json')); print('$n', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'], d['checks']['gather'])"
done
timeout -k 10 400 python bench.py --gpus 2 --pairs 2000000 --clusters 20000 --dist-backend gloo --steps 10 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_n2_onegpu.json 2> $O/bench_n2_onegpu.log || { tail -30 $O/bench_n2_onegpu.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_onegpu.json')); print('n2', d['n_gpus'], d['value'], d['checks']['gather'])"
