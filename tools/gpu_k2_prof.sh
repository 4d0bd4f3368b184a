#!/bin/bash
set -e
O=gpurun_out/${TAG:-k2prof}
mkdir -p $O
timeout -k 10 200 python tools/k2_wave_profile.py --pairs 1250000 > $O/wave_share.json 2> $O/wave_share.err
timeout -k 10 300 python tools/k2_wave_profile.py --pairs 10000000 > $O/wave_10M.json 2> $O/wave_10M.err
