#!/bin/bash
# Round 4 (d): gather binding (K3 writes the send buffer) + lookahead count check; the byte-heaviest N = 8
# share with the world-1 collective vs a 10M pass in the same session; kernel-trace timeline.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
W="--weights-cache $R/$O/w8.npy"
timeout -k 10 400 python -u -m pytest tests/test_gpu_collective.py tests/test_gpu_dist_rehearsal.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -40 $O/pytest_dist.log; exit 1; }
tail -2 $O/pytest_dist.log
timeout -k 10 400 python bench.py --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_10m.json 2> $O/bench_10m.log || { tail -30 $O/bench_10m.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_10m.json')); print('10M', d['value'], d['ms_per_step'], d['kernels_ms'])"
for v in "gather:--gather-world1" "gather_nolook:--gather-world1 --no-gather-lookahead" "nogather:"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 python bench.py --emulate-world 8 $W --steps 100 $a --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share_$n.json 2> $O/share_$n.log || { tail -30 $O/share_$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/share_$n.json')); print('$n', d['value'], d['ms_per_step'], d['kernels_ms']['diff_pass'], d['checks']['gather'])"
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/tl -o run --output-format csv -- \
    python3 $R/bench.py --emulate-world 8 $W --steps 20 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $R/$O/tl_bench.json 2> $R/$O/tl_bench.log || { tail -30 $R/$O/tl_bench.log; exit 1; }
cd $R
python tools/timeline_split.py $O/tl --last 15 > $O/timeline_split.json && cat $O/timeline_split.json
