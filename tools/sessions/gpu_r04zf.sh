#!/bin/bash
# Round 4 (zf): pair-mode K0 stage decoupled from the kernel stream: device-encode tests, JSON-in rates (A/B against one K0
# stream), watch replay A/B, and a kernel + copy trace of JSON-in batches.
set -o pipefail
O=gpurun_out/r04zf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_json_in.py tests/test_gpu_write_plan.py tests/test_gpu_tokenize.py tests/test_gpu_store.py tests/test_gpu_upsert.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/json_in_probe.py > $O/json_in.json 2> $O/json_in.log || { tail -20 $O/json_in.log; exit 1; }
python -c "import json; d=json.load(open('$O/json_in.json')); print({k: (v.get('pairs_per_s') if isinstance(v, dict) else v) for k, v in d.items()}); print(d['device_encode']['phases_ms']); print(d['device_encode_zero_copy'])"
timeout -k 10 300 python bench.py --config config5 --no-cpu-baseline > $O/config5.json 2> $O/config5.log || { tail -20 $O/config5.log; exit 1; }
python -c "import json; d=json.load(open('$O/config5.json')); print('c5', d['value'], d['batch_ms'])"
GPUDIFF_K0_ONE_STREAM=1 timeout -k 10 300 python bench.py --config config5 --no-cpu-baseline > $O/config5_one.json 2> $O/config5_one.log || { tail -20 $O/config5_one.log; exit 1; }
python -c "import json; d=json.load(open('$O/config5_one.json')); print('c5 one K0 stream', d['value'], d['batch_ms'])"
R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/trace -o run --output-format csv -- python3 $R/tools/json_in_probe.py --device-only 4 > $R/$O/trace_probe.json 2> $R/$O/trace_probe.log || { tail -20 $R/$O/trace_probe.log; exit 1; }
cat $R/$O/trace_probe.json
