set -o pipefail
O=${O:-gpurun_out/r01h}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_config3.json 2> $O/bench_config3.log && cat $O/bench_config3.json &&
timeout -k 10 200 python bench.py --config config2 --cpu-seconds 4 > $O/bench_config2.json 2> $O/bench_config2.log && cat $O/bench_config2.json &&
timeout -k 10 200 python bench.py --config config4 --cpu-seconds 4 > $O/bench_config4.json 2> $O/bench_config4.log && cat $O/bench_config4.json
