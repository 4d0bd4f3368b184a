#!/bin/bash
# Round 4 (zn): the largest-first rounds defer joins over 256 keys to K4 (deep batches): parity
# (incl. the hand-out order agreement test), config4 A/B against the joins kept in K2 (0x80) and index order (0x4),
# and config4's per-wave timeline.
set -o pipefail
O=gpurun_out/r04zn; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "c4_defer:0" "c4_k2join:0x80" "c4_defer_b:0" "c4_k2join_b:0x80"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python bench.py --pipeline 1 --config config4 --steps 30 --no-cpu-baseline --sample 0 --json-in-pairs 0 --engine-flags $f > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms']['compare_all_launches'])"
done
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 > $O/wave_c4.json 2> $O/wave_c4.log || { tail -20 $O/wave_c4.log; exit 1; }
python -c "import json; d=json.load(open('$O/wave_c4.json')); v=d['variant14']; print('c4', d['variant0']['k2_ms'], v['k2_ms'], v['span_us'], v['end_us'], v['busy_frac_of_span'], v['running_at'])"
