#!/bin/bash
# Round 6 (o): the round-end profile at the final K2 sources (compressed code objects): smoke + K2 parity first, then
# config3's bench line, rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes and the line with traffic attached;
# then config2's and config4's kernel stats + counters.
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py::test_k2_kernels_bit_exact tests/test_gpu_golden.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 900 bash tools/profile_round.sh r06o || exit 1
timeout -k 10 500 bash tools/profile_config.sh config2 r06o || exit 1
timeout -k 10 500 bash tools/profile_config.sh config4 r06o || exit 1
echo done
