#!/bin/bash
# Round 4 (f): the -m gpu suite at HEAD (range tail, gather binding, views), config4 range-tail A/B, the
# byte-heaviest N = 8 share with two passes in flight vs one, and a 10M pass, in one session.
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
W="--weights-cache $R/$O/w8.npy"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in "c4_auto:" "c4_off:--engine-flags 0x2" "c4_k8:--engine-flags 0x6"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py --config config4 --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 $a > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms'])"
done
timeout -k 10 400 python bench.py --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_10m.json 2> $O/bench_10m.log || { tail -30 $O/bench_10m.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_10m.json')); print('10M', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'])"
for v in "p2_gather:--pipeline 2 --gather-world1" "p1_gather:--gather-world1" "p2:--pipeline 2"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 python bench.py --emulate-world 8 $W --steps 100 $a --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share_$n.json 2> $O/share_$n.log || { tail -30 $O/share_$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/share_$n.json')); print('$n', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'], d['checks']['gather'], d['checks']['full_size'].get('pipeline_view_flags_eq'))"
done
