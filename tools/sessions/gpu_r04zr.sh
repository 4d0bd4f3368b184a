#!/bin/bash
# Round 4 (zr): K2 writes status-absent-only paths lane-parallel: parity, then an interleaved A/B of the whole
# library against the previous build (kcp_amd/libgpudiff_before.so, swapped in between runs) on config3 10M and
# the N = 8 share.
set -o pipefail
O=gpurun_out/r04zr; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp kcp_amd/libgpudiff.so $O/new.so
for v in new before new before; do
  cp $O/new.so kcp_amd/libgpudiff.so
  [ $v = before ] && cp kcp_amd/libgpudiff_before.so kcp_amd/libgpudiff.so
  timeout -k 10 400 python bench.py --pipeline 1 --steps 20 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/m_$v.json 2> $O/m_$v.log || { cp $O/new.so kcp_amd/libgpudiff.so; tail -20 $O/m_$v.log; exit 1; }
  python -c "import json; d=json.load(open('$O/m_$v.json')); print('10M $v', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['roofline']['format']['frac'],4), round(d['kernels_ms']['compare_all_launches'],4))"
  timeout -k 10 400 python bench.py --pipeline 1 --emulate-world 8 --steps 40 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/sh_$v.json 2> $O/sh_$v.log || { cp $O/new.so kcp_amd/libgpudiff.so; tail -20 $O/sh_$v.log; exit 1; }
  python -c "import json; d=json.load(open('$O/sh_$v.json')); print('share $v', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['kernels_ms']['compare_all_launches'],4))"
done
cp $O/new.so kcp_amd/libgpudiff.so
rm -f $O/new.so
