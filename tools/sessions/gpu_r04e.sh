#!/bin/bash
# Round 4 (e): two passes in flight (dbatch view on a second context) at the byte-heaviest N = 8 share
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
W="--weights-cache $R/$O/w8.npy"
timeout -k 10 400 python -u -m pytest tests/test_gpu_collective.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -40 $O/pytest_dist.log; exit 1; }
tail -1 $O/pytest_dist.log
timeout -k 10 400 python bench.py --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_10m.json 2> $O/bench_10m.log || { tail -30 $O/bench_10m.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_10m.json')); print('10M', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'])"
for v in "p2_gather:--pipeline 2 --gather-world1" "p1_gather:--gather-world1" "p2:--pipeline 2"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 python bench.py --emulate-world 8 $W --steps 100 $a --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share_$n.json 2> $O/share_$n.log || { tail -30 $O/share_$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/share_$n.json')); print('$n', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'], d['checks']['gather'], d['checks']['full_size'].get('pipeline_view_flags_eq'))"
done
timeout -k 10 400 python bench.py --pipeline 2 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_10m_p2.json 2> $O/bench_10m_p2.log || { tail -30 $O/bench_10m_p2.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_10m_p2.json')); print('10M p2', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'])"
