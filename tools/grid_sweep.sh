#!/bin/bash
# Default grid vs one tile per wave (max_blocks uncapped) for the uniform kernel
# across the bench configs and a few mid sizes (tools/sweep.py, interleaved rounds).
set -e
O=gpurun_out/grid_sweep
mkdir -p $O
timeout -k 10 200 python3 tools/sweep.py --config 64 --blocks 0,4096,16384,65536,262144 --unrolls 0 --rounds 5 --steps 30 > $O/c64.jsonl 2>>$O/err
timeout -k 10 200 python3 tools/sweep.py --config 64k --blocks 0,1024,4096,65536 --unrolls 0 --rounds 5 --steps 10 > $O/c64k.jsonl 2>>$O/err
for L in 256 576 4096 8192; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,16384,65536,262144 --unrolls 0 --rounds 5 --steps 20 > $O/len$L.jsonl 2>>$O/err
done
timeout -k 10 200 python3 tools/sweep.py --config 1500 --blocks 0,16384 --unrolls 0 --rounds 7 --steps 30 --probe > $O/c1500.jsonl 2>>$O/err
