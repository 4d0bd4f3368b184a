#!/bin/bash
# K10 (write path) parity + profile + bench on the GPU box; time-limited steps, stop at the first failure.
set -o pipefail
O=${O:-gpurun_out/k10}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_upsert.py tests/test_gpu_write_plan.py -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/k10_profile.py > $O/k10_profile.txt 2>&1 || { tail -20 $O/k10_profile.txt; exit 1; }
grep -v amdgpu.ids $O/k10_profile.txt
timeout -k 10 300 python bench.py --config upsert --cpu-seconds 4 > $O/bench_upsert.json 2> $O/bench_upsert.log || { tail -30 $O/bench_upsert.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_upsert.json')); print(d['value'], d['ms_per_step'], d['checks'])"
