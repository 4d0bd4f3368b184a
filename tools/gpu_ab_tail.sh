#!/bin/bash
# In-process A/B of K2's 8-pair tail size (GPUDIFF_OPT_K2_TAIL_SHIFT, quarters of the wave count).
set -e
O=gpurun_out/${TAG:-abtail}
mkdir -p $O
V="t1=0x10,t2=0x20,t4=0x40,t7=0x70"
timeout -k 10 200 python tools/ab_k2.py --pairs 1250000 --clusters 12500 --rounds 6 --passes 5 --variants $V > $O/ab_share.json 2> $O/ab_share.err
timeout -k 10 300 python tools/ab_k2.py --pairs 10000000 --clusters 100000 --rounds 4 --passes 3 --variants $V > $O/ab_10M.json 2> $O/ab_10M.err
