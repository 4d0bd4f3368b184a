#!/bin/bash
# In-process A/B of K2's tail (GPUDIFF_OPT_K2_TAIL_SHIFT / GPUDIFF_OPT_K2_TAIL8), after the parity tests.
set -e
O=gpurun_out/${TAG:-abtail}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_store.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
V="dflt=0x0,notail_late=0x10,tail8=0x80,h4=0x50"
timeout -k 10 200 python tools/ab_k2.py --pairs 1250000 --clusters 12500 --rounds 6 --passes 5 --variants $V > $O/ab_share.json 2> $O/ab_share.err
timeout -k 10 300 python tools/ab_k2.py --pairs 10000000 --clusters 100000 --rounds 4 --passes 3 --variants $V > $O/ab_10M.json 2> $O/ab_10M.err
