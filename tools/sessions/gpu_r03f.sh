set -o pipefail
O=${O:-gpurun_out/r03f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_store.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for it in 0 1 2; do
  timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 --flags $((it << 28)) > $O/wave_c4_it$it.json 2> $O/wave_c4_it$it.log || exit 1
  python -c "import json;d=json.load(open('$O/wave_c4_it$it.json'));v=d['variant0'];w=d['variant14'];print('it$it', 'k2', round(v['k2_ms'],3), 'pass', round(v['pass_ms'],3), 'busy', round(w['busy_frac_of_span'],3), 'join', round(w['join_frac_of_busy'],3), 'items', w['items_per_wave']['50'])"
done
timeout -k 10 300 python bench.py --config config4 --steps 10 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c4.json 2> $O/bench_c4.log && python -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4', d['value'], d['ms_per_step'], d['roofline']['format']['frac'], d['checks']['full_size'])" &&
timeout -k 10 300 python bench.py --config config2 --steps 20 --cpu-seconds 2 --json-in-pairs 0 > $O/bench_c2.json 2> $O/bench_c2.log && python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2', d['value'], d['ms_per_step'], d['roofline']['format']['frac'])" &&
timeout -k 10 300 python bench.py --pairs 1250000 --clusters 12500 --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_share.json 2> $O/bench_share.log && python -c "import json;d=json.load(open('$O/bench_share.json'));print('share', d['value'], d['ms_per_step'], d['kernels_ms'])"
