#!/bin/bash
# Round 5 (j): K0 small-document hash phase (tokenize tests), then an ablation A/B of K0 on a config5-sized batch:
# kcp_amd/_exp/libgpudiff_abl<bits>.so built from the same K0 with parts switched off (1 decoded strings, 2 atom
# parsing, 4 the sort, 8 the XXH64 path hashes; 15 all four; 0 none) -- timing only, their outputs are not valid.
set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_json_in.py tests/test_gpu_store.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tok.log 2>&1 || { tail -40 $O/pytest_tok.log; exit 1; }
tail -1 $O/pytest_tok.log
for r in 1 2; do
  for a in 0 1 2 4 8 15; do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_a${a}_r$r -o k0 --output-format csv -- python tools/k0_bench.py --reps 4 --profile --lib kcp_amd/_exp/libgpudiff_abl$a.so > $O/k0_a${a}_r$r.json 2> $O/k0_a${a}_r$r.log || { tail -20 $O/k0_a${a}_r$r.log; exit 1; }
    echo "a$a r$r $(cut -c1-160 $O/k0_a${a}_r$r.json)"
  done
done
echo done
