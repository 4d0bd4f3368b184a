#!/bin/bash
# Round 5 (p): the round-end profile at the final K2 sources -- config3 bench line, rocprofv3 kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes (separate runs), pmc_summary and the line with traffic attached; then config4's.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 bash tools/profile_round.sh r05p || exit 1
timeout -k 10 500 bash tools/profile_config.sh config4 r05p || exit 1
echo done
