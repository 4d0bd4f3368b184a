set -o pipefail
O=${O:-gpurun_out/r03d}; mkdir -p $O
timeout -k 10 120 python tools/dbg_k1_trace.py > $O/trace.json 2> $O/trace.log; tail -3 $O/trace.log; head -c 3000 $O/trace.json
