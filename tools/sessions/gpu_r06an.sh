#!/bin/bash
# Round 6 (an): final sources, part 2 -- the final measurement -- smoke + K2 parity; config3 round-end profile (bench line,
# config3's bench line, rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes and the line with traffic attached;
# then config2's and config4's kernel stats + counters.
set -o pipefail
O=gpurun_out/r06an; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py::test_k2_kernels_bit_exact tests/test_gpu_golden.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 900 bash tools/profile_round.sh r06an || exit 1
timeout -k 10 500 bash tools/profile_config.sh config2 r06an || exit 1
timeout -k 10 500 bash tools/profile_config.sh config4 r06an || exit 1
line() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],4), 'frac', (d.get('roofline') or {}).get('frac'), 'cpu', (d.get('cpu_baseline') or {}).get('value'), d.get('build_id'))"; }
timeout -k 10 300 python -u bench.py --config config1 --cpu-seconds 8 > $O/config1.json 2> $O/config1.log || { tail -30 $O/config1.log; exit 1; }
line $O/config1.json
timeout -k 10 400 python -u bench.py --config config2 --cpu-seconds 8 > $O/config2.json 2> $O/config2.log || { tail -30 $O/config2.log; exit 1; }
line $O/config2.json
timeout -k 10 400 python -u bench.py --config config4 --cpu-seconds 8 > $O/config4.json 2> $O/config4.log || { tail -30 $O/config4.log; exit 1; }
line $O/config4.json
for m in staged zc; do
  A=""; [ $m = zc ] && A="--zero-copy"
  timeout -k 10 400 python -u bench.py --config config5 --seconds 12 $A --cpu-seconds 4 > $O/config5_$m.json 2> $O/config5_$m.log || { tail -30 $O/config5_$m.log; exit 1; }
  line $O/config5_$m.json
done
R=$(pwd)
timeout -k 10 400 python -u bench.py --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 100 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/share_gather.json 2> $O/share_gather.log || { tail -30 $O/share_gather.log; exit 1; }
line $O/share_gather.json
echo done
