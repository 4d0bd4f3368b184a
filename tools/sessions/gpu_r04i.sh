#!/bin/bash
# Round 4 (i): JSON-in rates and phases alone (warm ring slots), the H2D probe, then the 10M
# encoder-independent tree-walk check (flags + changed paths of every pair, device-encode path on the same chunks).
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/json_in_probe.py > $O/json_in.json 2> $O/json_in.log || { tail -20 $O/json_in.log; exit 1; }
cat $O/json_in.json
timeout -k 10 150 python tools/h2d_probe.py > $O/h2d_probe.txt 2>&1 || { cat $O/h2d_probe.txt; exit 1; }
cat $O/h2d_probe.txt
timeout -k 10 900 python -u tools/full_tree_check.py --k0 > $O/full_tree_check.json 2> $O/full_tree_check.log || { tail -30 $O/full_tree_check.log; exit 1; }
cat $O/full_tree_check.json
