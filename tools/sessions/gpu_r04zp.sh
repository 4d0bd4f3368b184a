#!/bin/bash
# Round 4 (zl): final -- the whole -m gpu suite and smoke, then the round-end profile at the final sources
# (config3 line + rocprofv3 + PMC passes + pmc_summary + the line with traffic) and config4's profile.
set -o pipefail
O=gpurun_out/r04zp; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 bash tools/profile_round.sh r04zp || exit 1
timeout -k 10 600 bash tools/profile_config.sh config4 r04zp || exit 1
