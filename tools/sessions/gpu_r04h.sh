#!/bin/bash
# Round 4 (h): parity + collective + rehearsal tests at HEAD; config4 largest-first final round A/B; the
# default bench line (two passes in flight, JSON-in phases); (the 10M tree-walk check is r04i).
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_collective.py tests/test_gpu_dist_rehearsal.py tests/test_gpu_json_in.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "c4_lpt:--engine-flags 0" "c4_idx:--engine-flags 0x4" "c4_lpt2:--engine-flags 0" "c4_idx2:--engine-flags 0x4"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py --pipeline 1 --config config4 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 $a > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['format']['frac'], d['kernels_ms']); print(json.dumps(d['json_in']))"
