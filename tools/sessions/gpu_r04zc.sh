#!/bin/bash
# Round 4 (zc): kernel + copy trace of the byte-heaviest N = 8 share with two passes in flight and the world-1
# collective: GPU busy fraction and idle gaps over the last 30 steps.
set -o pipefail
O=gpurun_out/r04zc; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/tr -o run --output-format csv -- python3 $R/bench.py --emulate-world 8 --steps 40 --pipeline 2 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $R/$O/share.json 2> $R/$O/share.log || { tail -20 $R/$O/share.log; exit 1; }
cd $R
f=$(find $O/tr -name 'run_kernel_trace.csv' | head -n 1); d=$(dirname $f)
python tools/busy_union.py $d --steps 30 | tee $O/busy.json
python -c "import json; d=json.load(open('$O/share.json')); print(d['ms_per_step'])"
