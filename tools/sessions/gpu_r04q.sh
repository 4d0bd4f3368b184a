#!/bin/bash
# Round 4 (q): K2 default by batch shape (x8 at 3 waves/SIMD; x16 at 2 for deep pairs): parity, golden,
# collective and rehearsal tests, then config4's rocprof + PMC profile.
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_collective.py tests/test_gpu_dist_rehearsal.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 bash tools/profile_config.sh config4 r04q
