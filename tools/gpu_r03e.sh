set -o pipefail
O=${O:-gpurun_out/r03e}; mkdir -p $O
for v in 0 1 3; do timeout -k 10 120 python tools/dbg_k1.py $v > $O/dbg$v.txt 2>&1 || exit 1; grep "bad slots" $O/dbg$v.txt; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_store.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/k1_ab.py --pairs 2500000 > $O/k1_ab.json 2> $O/k1_ab.log && cat $O/k1_ab.json &&
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 > $O/wave_c4.json 2> $O/wave_c4.log && cat $O/wave_c4.json &&
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 --flags 0xF00000 > $O/wave_c4_k4.json 2> $O/wave_c4_k4.log && cat $O/wave_c4_k4.json
