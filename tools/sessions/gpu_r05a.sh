#!/bin/bash
# Round 5 (a): the two-pass N > 1 path at world 2 (gloo rehearsal, forced regrow), the lookahead regrow with
# changing counts, zero-copy write plans; config1 and the 10-s config5 lines.
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_collective.py tests/test_gpu_write_plan.py tests/test_gpu_dist_rehearsal.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --pipeline 2 --gather-cap-frac 0.5 --pairs 2000000 --clusters 20000 --steps 6 --warmup 2 --json-in-pairs 0 --sample 0 > $O/bench_n2_onegpu_p2.json 2> $O/bench_n2_onegpu_p2.log || { tail -30 $O/bench_n2_onegpu_p2.log; exit 1; }
timeout -k 10 300 python bench.py --config config1 --sample 10000 --cpu-seconds 6 > $O/config1.json 2> $O/config1.log || { tail -30 $O/config1.log; exit 1; }
timeout -k 10 400 python bench.py --config config5 --seconds 12 --cpu-seconds 6 > $O/config5_10s.json 2> $O/config5_10s.log || { tail -30 $O/config5_10s.log; exit 1; }
echo benches done
# K0 on a config5-sized batch: kernel stats, phase split, SQ counters; config4's K2 per-wave timeline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k0kt -o k0 -- python tools/k0_bench.py --profile > $O/k0_bench.json 2> $O/k0_bench.log || { tail -20 $O/k0_bench.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/k0pmc -o k0 -- python tools/k0_bench.py --reps 2 > $O/k0_pmc_run.json 2> $O/k0_pmc.log || { tail -20 $O/k0_pmc.log; exit 1; }
timeout -k 10 300 python tools/k2_wave_profile.py --config config4 --pairs 100000 --passes 5 > $O/wave_c4.json 2> $O/wave_c4.log || { tail -20 $O/wave_c4.log; exit 1; }
echo profiled
