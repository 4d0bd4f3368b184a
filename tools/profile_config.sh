#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes (separate runs) of bench.py on one config, and the
# per-kernel summary (tools/pmc_summary.py).  usage: tools/profile_config.sh CONFIG TAG
set -eo pipefail
CFG=${1:?config}; TAG=${2:?tag}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_${TAG}_${CFG}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$ROOT/bench.py"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python3 "$B" --pipeline 1 --config "$CFG" --no-cpu-baseline --sample 0 --json-in-pairs 0 --steps 10 > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.log"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$B" --pipeline 1 --config "$CFG" --no-cpu-baseline --sample 0 --json-in-pairs 0 --steps 2 --warmup 1 > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.log"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$B" --pipeline 1 --config "$CFG" --no-cpu-baseline --sample 0 --json-in-pairs 0 --steps 2 --warmup 1 > "$OUT/write_bench.json" 2> "$OUT/write_bench.log"
cd "$ROOT"
for d in kt fetch write; do
    f=$(find "$OUT/$d" -name 'run_*.csv' | head -n 1 || true)
    if [ -n "$f" ] && [ "$(dirname "$f")" != "$OUT/$d" ]; then mv "$(dirname "$f")"/run_*.csv "$OUT/$d/"; fi
done
python3 tools/pmc_summary.py "$OUT/kt" "$OUT/fetch" "$OUT/write" "$OUT/kt_bench.json" "$OUT/pmc_summary.json"
python3 -c "import json; d=json.load(open('$OUT/pmc_summary.json')); print('$CFG', {k: (v['avg_ms'], v['hbm_bytes']) for k, v in d['kernels'].items() if v['avg_ms'] > 0.01})"
