#!/bin/bash
# JSON front-end phase profiles on the GPU box (K0, K10, K13), one process each, time-limited.
set -eo pipefail
O=gpurun_out/fe_prof; mkdir -p $O
timeout -k 10 200 python tools/k0_profile.py > $O/k0.txt 2>&1
timeout -k 10 200 python tools/k10_profile.py > $O/k10.txt 2>&1
timeout -k 10 200 python tools/k13_profile.py > $O/k13.txt 2>&1
timeout -k 10 200 python tools/k11_profile.py > $O/k11.txt 2>&1
cat $O/k0.txt $O/k10.txt $O/k13.txt $O/k11.txt | grep -v amdgpu.ids
