#!/bin/bash
# Round 4 (n): watch replay (config5) with upload chunks of >= 16k documents, A/B against one chunk; JSON-in.
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config config5 --no-cpu-baseline > $O/config5.json 2> $O/config5.log || { tail -20 $O/config5.log; exit 1; }
python -c "import json; d=json.load(open('$O/config5.json')); print('c5', d['value'], d['batch_ms'])"
GPUDIFF_H2D_MAX_CHUNKS=1 timeout -k 10 300 python bench.py --config config5 --no-cpu-baseline > $O/config5_1chunk.json 2> $O/config5_1chunk.log || { tail -20 $O/config5_1chunk.log; exit 1; }
python -c "import json; d=json.load(open('$O/config5_1chunk.json')); print('c5 1 chunk', d['value'], d['batch_ms'])"
timeout -k 10 200 python tools/json_in_probe.py > $O/json_in.json 2> $O/json_in.log || { tail -20 $O/json_in.log; exit 1; }
cat $O/json_in.json
