set -o pipefail
O=${O:-gpurun_out/r03a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_store.py tests/test_gpu_write_plan.py tests/test_gpu_goshim.py tests/test_gpu_rollup.py tests/test_gpu_collective.py -x -v --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1 || { tail -40 $O/pytest_new.log; exit 1; }
tail -5 $O/pytest_new.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 3 > $O/bench.json 2> $O/bench.log && cat $O/bench.json
