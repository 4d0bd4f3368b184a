#!/bin/bash
# A/B of the chained single-pass K3 / K5+K6 against the three-launch scans, at one rank's N = 8
# share (1.25M pairs) and at config3's full size; plus the per-step collective at world size 1.
set -e
O=gpurun_out/${TAG:-abscan}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "chained or segmented or deferred or overflow or mixed" tests/test_gpu_collective.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
C="--pairs 1250000 --clusters 12500 --steps 50 --warmup 5 --no-cpu-baseline --json-in-pairs 0 --sample 50"
for r in 1 2; do
timeout -k 10 240 python bench.py $C > $O/share_chained_$r.json 2> $O/share_chained_$r.err
timeout -k 10 240 python bench.py $C --engine-flags 0x40000000 > $O/share_scan3_$r.json 2> $O/share_scan3_$r.err
done
timeout -k 10 240 python bench.py $C --gather-world1 --gather-depth 1 > $O/share_d1.json 2> $O/share_d1.err; echo "d1 rc=$?" >> $O/rc.txt
timeout -k 10 240 python bench.py $C --gather-world1 --gather-depth 2 > $O/share_d2.json 2> $O/share_d2.err; echo "d2 rc=$?" >> $O/rc.txt
F="--steps 20 --warmup 3 --no-cpu-baseline --json-in-pairs 0 --sample 50"
timeout -k 10 300 python bench.py $F > $O/c3_chained.json 2> $O/c3_chained.err
timeout -k 10 300 python bench.py $F --engine-flags 0x40000000 > $O/c3_scan3.json 2> $O/c3_scan3.err
