#!/bin/bash
# Round-3 check on MI355X: -m gpu suite, smoke, default bench line, config4 / config2 / N=8-share K2 state, config4 K2 A/B
# N=8-share K2 state (wave timeline + benches).
set -o pipefail
O=${O:-gpurun_out/r03g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_config3.json 2> $O/bench_config3.log || { tail -20 $O/bench_config3.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_config3.json'));print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['format']['frac'])"
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 > $O/wave_c4.json 2> $O/wave_c4.log || exit 1
python -c "import json;d=json.load(open('$O/wave_c4.json'));v=d['variant0'];w=d['variant14'];print(json.dumps(w.get('per_item_us')));print('wave c4 k2', round(v['k2_ms'],3), 'pass', round(v['pass_ms'],3), 'busy', round(w['busy_frac_of_span'],3), 'join', round(w['join_frac_of_busy'],3), 'items', w['items_per_wave']['50'], 'end', w['end_us'])"
timeout -k 10 300 python bench.py --config config4 --steps 10 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c4.json 2> $O/bench_c4.log || { tail -20 $O/bench_c4.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms'])"
timeout -k 10 300 python bench.py --config config2 --steps 20 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c2.json 2> $O/bench_c2.log || { tail -20 $O/bench_c2.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['kernels_ms'])"
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_share.json 2> $O/bench_share.log || { tail -20 $O/bench_share.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_share.json'));print('share', d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 400 python tools/ab_k2.py --config config4 --pairs 100000 --clusters 1000 --rounds 4 --passes 3 --variants "def=0,fused=0x40000000,v13=0xD00" > $O/ab_c4.json 2> $O/ab_c4.log || { tail -20 $O/ab_c4.log; exit 1; }
tail -c 1500 $O/ab_c4.json
timeout -k 10 400 python tools/ab_k2.py --config config3 --rounds 3 --passes 3 --variants "def=0,fused=0x40000000" > $O/ab_c3.json 2> $O/ab_c3.log || { tail -20 $O/ab_c3.log; exit 1; }
tail -c 800 $O/ab_c3.json
timeout -k 10 400 python tools/ab_k2.py --config config3 --pairs 1250000 --clusters 12500 --rounds 4 --passes 5 --variants "def=0,fused=0x40000000" > $O/ab_share.json 2> $O/ab_share.log || { tail -20 $O/ab_share.log; exit 1; }
tail -c 800 $O/ab_share.json
