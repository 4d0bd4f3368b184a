#!/bin/bash
# Round 4 (zs): opt-in store-mode K0 stage on its own stream (GPUDIFF_K0_DECOUPLE_STORE=1): the store tests in
# both settings, then watch replay A/B, interleaved.
set -o pipefail
O=gpurun_out/r04zs; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_store.py tests/test_gpu_json_in.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GPUDIFF_K0_DECOUPLE_STORE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_store.py tests/test_gpu_json_in.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dec.log 2>&1 || { tail -40 $O/pytest_dec.log; exit 1; }
tail -1 $O/pytest_dec.log
for v in "c5_dec:GPUDIFF_K0_DECOUPLE_STORE=1" "c5_def:X=1" "c5_dec_b:GPUDIFF_K0_DECOUPLE_STORE=1" "c5_def_b:X=1"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 300 python bench.py --config config5 --no-cpu-baseline > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); b=d['batch_ms']; print('$n', round(d['value']/1e6,2), b['host_submit'], b['h2d'], b['k0_encode'], d['checks'])"
done
