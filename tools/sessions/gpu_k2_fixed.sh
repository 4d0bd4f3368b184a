#!/bin/bash
# K2's fixed cost per launch: config3 mix at several sizes (K2(n) = a + b n), and at the N = 8
# share size with every join deferred to K4 and with other item counts per wave.
set -e
O=gpurun_out/${TAG:-k2fixed}
mkdir -p $O
B="--steps 30 --warmup 3 --no-cpu-baseline --json-in-pairs 0 --sample 20"
for n in 625000 1250000 2500000 5000000; do
  timeout -k 10 240 python bench.py $B --pairs $n --clusters $((n / 100)) > $O/n$n.json 2> $O/n$n.err
done
timeout -k 10 240 python bench.py $B --pairs 1250000 --clusters 12500 --engine-flags $((14 << 21)) > $O/share_nojoin.json 2> $O/share_nojoin.err
timeout -k 10 240 python bench.py $B --pairs 1250000 --clusters 12500 --engine-flags $((1 << 28)) > $O/share_ipw4.json 2> $O/share_ipw4.err
timeout -k 10 240 python bench.py $B --pairs 1250000 --clusters 12500 --engine-flags $((3 << 28)) > $O/share_ipw16.json 2> $O/share_ipw16.err
