#!/bin/bash
set -eo pipefail
R=$(pwd); O=$R/gpurun_out/ab_k2v; mkdir -p $O
V="base=0,dynx2=0xF00,b5=0x5000,b6=0x6000,x2b6=0x6F00,x2b8=0x8F00"
timeout -k 10 400 python tools/ab_k2.py --pairs 10000000 --clusters 100000 --rounds 3 --passes 3 --variants $V > $O/ab_10M.json 2> $O/ab_10M.log
