#!/bin/bash
# Round 4 (b): the N > 1 bench path on one GPU (gloo rehearsal), byte-weighted LPT, the byte-heaviest
# rank's N = 8 share vs a 10M pass in the same session, and a kernel-trace timeline of 20 share steps.
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_rehearsal.py tests/test_gpu_collective.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1 || { tail -40 $O/pytest_dist.log; exit 1; }
tail -2 $O/pytest_dist.log
timeout -k 10 400 python bench.py --gpus 2 --pairs 2000000 --clusters 20000 --dist-backend gloo --steps 10 --no-cpu-baseline --sample 0 --json-in-pairs 0 > $O/bench_n2_onegpu.json 2> $O/bench_n2_onegpu.log || { tail -30 $O/bench_n2_onegpu.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_n2_onegpu.json')); print('n2', d['n_gpus'], d['value'], d['checks']['gather'], d['config']['shard'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_10m.json 2> $O/bench_10m.log || { tail -30 $O/bench_10m.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_10m.json')); print('10M', d['value'], d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 400 python bench.py --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 50 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_share_heavy_gather.json 2> $O/bench_share_heavy_gather.log || { tail -30 $O/bench_share_heavy_gather.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_share_heavy_gather.json')); print('heavy+gather', d['value'], d['ms_per_step'], d['kernels_ms'], d['config']['shard'])"
timeout -k 10 400 python bench.py --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 50 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $O/bench_share_heavy.json 2> $O/bench_share_heavy.log || { tail -30 $O/bench_share_heavy.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench_share_heavy.json')); print('heavy', d['value'], d['ms_per_step'], d['kernels_ms'])"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/tl -o run --output-format csv -- \
    python3 $R/bench.py --emulate-world 8 --weights-cache $R/$O/w8.npy --steps 20 --gather-world1 --no-cpu-baseline --sample 0 --json-in-pairs 0 --no-full-paths > $R/$O/tl_bench.json 2> $R/$O/tl_bench.log || { tail -30 $R/$O/tl_bench.log; exit 1; }
cd $R
python tools/timeline_split.py $O/tl --last 15 > $O/timeline_split.json && cat $O/timeline_split.json
timeout -k 10 300 python tools/k2_wave_profile.py --pairs 1250000 --passes 5 > $O/wave_share.json 2> $O/wave_share.log || { tail -20 $O/wave_share.log; exit 1; }
python -c "import json; d=json.load(open('$O/wave_share.json')); print({k: d[k] for k in list(d)[:12]})"
