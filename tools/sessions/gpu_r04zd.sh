#!/bin/bash
# Round 4 (zd): the collective test with two passes in flight (PipelinedGather, regrow), JSON-in and store tests
# after gpudiff_close's host-buffer release, then the round-end profile at the final sources.
set -o pipefail
O=gpurun_out/r04zd; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_collective.py tests/test_gpu_json_in.py tests/test_gpu_store.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 1000 bash tools/profile_round.sh r04zd || exit 1
timeout -k 10 600 bash tools/profile_config.sh config4 r04zd || exit 1
