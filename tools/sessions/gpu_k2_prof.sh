#!/bin/bash
set -e
O=gpurun_out/${TAG:-k2prof}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
timeout -k 10 200 python tools/k2_wave_profile.py --pairs 1250000 > $O/wave_share.json 2> $O/wave_share.err
timeout -k 10 300 python tools/k2_wave_profile.py --pairs 10000000 > $O/wave_10M.json 2> $O/wave_10M.err
B="--steps 30 --warmup 3 --no-cpu-baseline --json-in-pairs 0 --sample 20"
timeout -k 10 240 python bench.py $B --pairs 1250000 --clusters 12500 > $O/share.json 2> $O/share.err
timeout -k 10 300 python bench.py $B > $O/c3.json 2> $O/c3.err
