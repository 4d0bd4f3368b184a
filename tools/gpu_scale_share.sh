#!/bin/bash
# One rank's share of the N = 8 strong-scaling run (10M/8 pairs, 100k/8 clusters) on one GPU:
# the diff pass alone, then with the per-step RCCL collective (world size 1) serial and pipelined.
set -e
O=gpurun_out/${TAG:-scale}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_collective.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
C="--pairs 1250000 --clusters 12500 --steps 50 --warmup 5 --no-cpu-baseline --json-in-pairs 0 --sample 50"
timeout -k 10 240 python bench.py $C > $O/share_nogather.json 2> $O/share_nogather.err
timeout -k 10 240 python bench.py $C --gather-world1 --gather-depth 1 > $O/share_d1.json 2> $O/share_d1.err
timeout -k 10 240 python bench.py $C --gather-world1 --gather-depth 2 > $O/share_d2.json 2> $O/share_d2.err
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o share -- python3 bench.py $C --steps 20 > $O/prof_share.json 2> $O/prof_share.err
