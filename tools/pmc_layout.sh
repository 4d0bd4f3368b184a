#!/bin/bash
# K2 traffic experiment on the GPU box: FETCH_SIZE and HIP-event K2 time of the
# config3 pass for blob alignments 16 / 128, with joins in K2 and with every
# join deferred to K4 (arena shrunk), each in its own short run.
set -eo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_layout; mkdir -p $OUT
export TMPDIR=/tmp
B="$ROOT/bench.py"
cd /tmp
for AL in 16 128; do
  for FL in 0 0x1E00000; do
    T=al${AL}_fl${FL}
    GPUDIFF_BLOB_ALIGN=$AL timeout -k 10 300 python3 "$B" --no-cpu-baseline --sample 0 --steps 10 --engine-flags $FL > $OUT/$T.json 2> $OUT/$T.log
    GPUDIFF_BLOB_ALIGN=$AL timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/f_$T -o run --output-format csv -- \
      python3 "$B" --no-cpu-baseline --sample 0 --steps 2 --warmup 1 --engine-flags $FL > $OUT/f_$T.json 2> $OUT/f_$T.log
    echo "$T done"
  done
done
