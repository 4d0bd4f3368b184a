#!/bin/bash
# Round 4 (z): zero-copy JSON-in (gpudiff_host_alloc buffers): the JSON-in tests, then rates (staged vs zero copy,
# sequential and streaming).
set -o pipefail
O=gpurun_out/r04z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_json_in.py tests/test_gpu_write_plan.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/json_in_probe.py > $O/json_in.json 2> $O/json_in.log || { tail -20 $O/json_in.log; exit 1; }
python -c "import json; d=json.load(open('$O/json_in.json')); print({k: (v.get('pairs_per_s') if isinstance(v, dict) else v) for k, v in d.items()}); print(d['device_encode_zero_copy'])"
