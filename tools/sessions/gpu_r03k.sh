#!/bin/bash
# Round-3 profile on MI355X at the K2 default: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes
# and the bench line with roofline.traffic (tools/profile_round.sh), then the §8(f) side benches.
set -o pipefail
bash tools/profile_round.sh r03k || exit 1
O=gpurun_out/r03k_side bash tools/gpu_side_benches.sh || exit 1
