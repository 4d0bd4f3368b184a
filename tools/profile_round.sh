#!/bin/bash
# Round profile on the GPU box (run through gpurun from the repo root):
#   1. bench.py at defaults (the judged line, with cpu_baseline)
#   2. rocprofv3 --kernel-trace --stats over a short bench run
#   3. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) -- counters never share
#      a run with traces
#   4. tools/pmc_summary.py -> per-kernel avg duration + corrected HBM bytes per
#      launch, then bench.py again with --traffic-json so roofline.traffic is set
# Every GPU step has its own time limit and the chain stops at the first failure.
# usage: tools/profile_round.sh ROUND_TAG   (e.g. r01)
set -eo pipefail
TAG=${1:?round tag}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$ROOT/bench.py"

timeout -k 10 600 python3 "$B" > "$OUT/bench.json" 2> "$OUT/bench.log"
cat "$OUT/bench.json"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
    python3 "$B" --pipeline 1 --no-cpu-baseline --sample 0 --steps 10 > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.log"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$B" --pipeline 1 --no-cpu-baseline --sample 0 --steps 2 --warmup 1 > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.log"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$B" --pipeline 1 --no-cpu-baseline --sample 0 --steps 2 --warmup 1 > "$OUT/write_bench.json" 2> "$OUT/write_bench.log"
cd "$ROOT"
# rocprofv3 may nest its files under host/pid directories: flatten
for d in kt fetch write; do
    f=$(find "$OUT/$d" -name 'run_*.csv' | head -n 1 || true)
    if [ -n "$f" ] && [ "$(dirname "$f")" != "$OUT/$d" ]; then mv "$(dirname "$f")"/run_*.csv "$OUT/$d/"; fi
done
python3 tools/pmc_summary.py "$OUT/kt" "$OUT/fetch" "$OUT/write" "$OUT/kt_bench.json" "$OUT/pmc_summary.json"
timeout -k 10 600 python3 "$B" --traffic-json "$OUT/pmc_summary.json" --cpu-seconds 4 > "$OUT/bench_traffic.json" 2> "$OUT/bench_traffic.log"
cat "$OUT/bench_traffic.json"
