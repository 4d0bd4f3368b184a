set -o pipefail
O=${O:-gpurun_out/r03b}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_store.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python tools/k1_ab.py --pairs 2500000 > $O/k1_ab.json 2> $O/k1_ab.log && cat $O/k1_ab.json &&
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 > $O/wave_c4.json 2> $O/wave_c4.log && cat $O/wave_c4.json &&
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 --flags 0xF00000 > $O/wave_c4_k4.json 2> $O/wave_c4_k4.log && cat $O/wave_c4_k4.json
