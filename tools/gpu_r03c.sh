set -o pipefail
O=${O:-gpurun_out/r03c}; mkdir -p $O
timeout -k 10 120 python tools/dbg_k1.py 0 > $O/dbg0.txt 2>&1; tail -30 $O/dbg0.txt
timeout -k 10 120 python tools/dbg_k1.py 3 > $O/dbg3.txt 2>&1; tail -16 $O/dbg3.txt
timeout -k 10 120 python tools/dbg_k1.py 2 > $O/dbg2.txt 2>&1; tail -4 $O/dbg2.txt
