#!/bin/bash
# Round 6 (a): config 2 (BASELINE configs[1]: 1M ConfigMaps/Secrets, 10k clusters) at the round-start sources --
# the bench line (two passes in flight, CPU baseline), rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes, and
# K2's per-wave timeline.
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O/config2
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config config2 --cpu-seconds 8 > $O/config2/bench.json 2> $O/config2/bench.log || { tail -30 $O/config2/bench.log; exit 1; }
cut -c1-400 $O/config2/bench.json
timeout -k 10 600 bash tools/profile_config.sh config2 r06a || exit 1
timeout -k 10 300 python -u tools/k2_wave_profile.py --config config2 --pairs 1000000 > $O/config2/wave_c2.json 2> $O/config2/wave.log || { tail -30 $O/config2/wave.log; exit 1; }
cut -c1-600 $O/config2/wave_c2.json
echo done
