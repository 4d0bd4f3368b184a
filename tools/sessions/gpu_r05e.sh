#!/bin/bash
# Round 5 (e): K0 workgroup shape A/B (4 / 2 / 1 documents per workgroup), kernel trace of each, interleaved.
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for w in 4 2 1; do
  lib=""; [ $w != 4 ] && lib="--lib kcp_amd/_exp/libgpudiff_wpb$w.so"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_w${w}_r$r -o k0 --output-format csv -- python tools/k0_bench.py $lib --reps 4 > $O/k0_w${w}_r$r.json 2> $O/k0_w${w}_r$r.log || { tail -20 $O/k0_w${w}_r$r.log; exit 1; }
  python3 -c "
import csv,sys
r=[x for x in csv.DictReader(open('$O/kt_w${w}_r$r/k0_kernel_trace.csv')) if 'encode_docs' in x['Kernel_Name']]
print('wpb $w round $r', [round((int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e6,3) for x in r])"
done
done
# the deep-pair K2 with in-workgroup helpers: parity on deep batches, then config4 (isolated K2, wave timeline)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 --passes 5 > $O/wave_c4.json 2> $O/wave_c4.log || { tail -20 $O/wave_c4.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/wave_c4.json')); v=d['variant0']; w=d['variant14']
print('config4 K2 ms', v['k2_ms'], 'frac', v['format_bytes']/v['k2_ms']/1e6/8000, 'timeline', w['k2_ms'], w['end_us'], w['running_at'])"
