#!/bin/bash
# Round 6 (i): K10 tests at the no-promotion build; the world-2 rehearsal (two ranks on one GPU over gloo, two passes
# in flight, forced regrow) with each rank's isolated passes run alone, its rocprofv3 kernel trace, and the world-1
# share of the same population.
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O/rehearsal_p2
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_upsert.py tests/test_gpu_write_plan.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
R="--pipeline 2 --pairs 2000000 --clusters 20000 --steps 6 --warmup 2 --json-in-pairs 0 --sample 0"
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --gather-cap-frac 0.5 $R > $O/rehearsal_p2/bench_n2.json 2> $O/rehearsal_p2/bench_n2.log || { tail -30 $O/rehearsal_p2/bench_n2.log; exit 1; }
timeout -k 10 400 python -u bench.py --emulate-world 2 --no-cpu-baseline $R > $O/rehearsal_p2/world1_share.json 2> $O/rehearsal_p2/world1_share.log || { tail -30 $O/rehearsal_p2/world1_share.log; exit 1; }
( cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $ROOT/$O/rehearsal_p2/kt -o run --output-format csv -- \
    python3 $ROOT/bench.py --gpus 2 --dist-backend gloo $R > $ROOT/$O/rehearsal_p2/kt_bench.json 2> $ROOT/$O/rehearsal_p2/kt_bench.log ) || { tail -30 $O/rehearsal_p2/kt_bench.log; exit 1; }
python - <<'PY'
import json
O = "gpurun_out/r06i/rehearsal_p2"
for f in ("bench_n2", "world1_share"):
    d = json.loads(open("%s/%s.json" % (O, f)).read().strip().splitlines()[-1])
    print(f, d["n_gpus"], round(d["value"] / 1e6, 1), "M pairs/s", round(d["ms_per_step"], 3), json.dumps(d["kernels_ms"])[:600])
    print("   gather", json.dumps((d.get("checks") or {}).get("gather"))[:400])
PY
find $O/rehearsal_p2/kt -name '*kernel_stats.csv' | head -3
echo done
