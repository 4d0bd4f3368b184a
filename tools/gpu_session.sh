#!/bin/bash
# One GPU-box verification pass (run through gpurun from the repo root):
#   the -m gpu suite, smoke(), the default bench line (config3), the watch replay (config5) and a
#   rocprofv3 --kernel-trace --stats pass over a short config5 run.
# Every GPU step has its own limit; the chain stops at the first failure.
# usage: O=gpurun_out/r02n [SKIP_TESTS=1] [SKIP_C3=1] bash tools/gpu_session.sh
set -o pipefail
O=${O:?output dir}; mkdir -p $O
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
if [ -z "$SKIP_C3" ]; then
timeout -k 10 400 python bench.py > $O/bench_config3.json 2> $O/bench_config3.log || { tail -30 $O/bench_config3.log; exit 1; }
cat $O/bench_config3.json
fi
if [ -z "$SKIP_C5" ]; then
timeout -k 10 300 python bench.py --config config5 > $O/bench_config5.json 2> $O/bench_config5.log || { tail -30 $O/bench_config5.log; exit 1; }
cat $O/bench_config5.json
R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt5 -o run --output-format csv -- \
    python3 $R/bench.py --config config5 --no-cpu-baseline --batches 20 > $R/$O/kt5_bench.json 2> $R/$O/kt5_bench.log || { tail -30 $R/$O/kt5_bench.log; exit 1; }
cd $R
f=$(find $O/kt5 -name 'run_kernel_stats.csv' | head -n 1 || true); [ -n "$f" ] && head -12 "$f"
fi
