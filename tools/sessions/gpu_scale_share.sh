#!/bin/bash
# One rank's share of the N = 8 strong-scaling run (10M/8 pairs, 100k/8 clusters) on one GPU:
# the diff pass alone (chained single-pass K3/K5 vs the three-launch scans), then with the
# per-step RCCL collective (world size 1) serial and pipelined; then config3 at full size, A/B.
set -e
O=gpurun_out/${TAG:-scale}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_collective.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
C="--pairs 1250000 --clusters 12500 --steps 50 --warmup 5 --no-cpu-baseline --json-in-pairs 0 --sample 50"
timeout -k 10 240 python bench.py $C > $O/share_chained.json 2> $O/share_chained.err
timeout -k 10 240 python bench.py $C --engine-flags 0x40000000 > $O/share_scan3.json 2> $O/share_scan3.err
timeout -k 10 240 python bench.py $C --gather-world1 --gather-depth 1 > $O/share_d1.json 2> $O/share_d1.err
timeout -k 10 240 python bench.py $C --gather-world1 --gather-depth 2 > $O/share_d2.json 2> $O/share_d2.err
F="--steps 20 --warmup 3 --no-cpu-baseline --json-in-pairs 0 --sample 50"
timeout -k 10 300 python bench.py $F > $O/c3_chained.json 2> $O/c3_chained.err
timeout -k 10 300 python bench.py $F --engine-flags 0x40000000 > $O/c3_scan3.json 2> $O/c3_scan3.err
