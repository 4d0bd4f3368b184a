#!/bin/bash
# Round 4 (u): K2 per-wave timeline on config4 with the default deep-pair kernel (16 a side in flight; the
# profiled variant follows the default's shape choice), and on the config3 N = 8 share size (8 a side).
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 > $O/wave_c4.json 2> $O/wave_c4.log || { tail -20 $O/wave_c4.log; exit 1; }
python -c "import json; d=json.load(open('$O/wave_c4.json')); v=d['variant14']; print('c4', d['variant0']['k2_ms'], v['k2_ms'], v['span_us'], v['end_us'], v['busy_frac_of_span'], v['running_at'], v['per_item_us'], v['items_per_wave'])"
timeout -k 10 300 python tools/k2_wave_profile.py --pairs 1250000 > $O/wave_share.json 2> $O/wave_share.log || { tail -20 $O/wave_share.log; exit 1; }
python -c "import json; d=json.load(open('$O/wave_share.json')); v=d['variant14']; print('share', d['variant0']['k2_ms'], v['k2_ms'], v['span_us'], v['end_us'], v['busy_frac_of_span'], v['running_at'], v['per_item_us'], v['items_per_wave'])"
