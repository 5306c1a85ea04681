#!/bin/bash
# One-wave-per-segment uniform batches (shape 9): default grid against larger ones.
set -e
O=gpurun_out/grid_long
mkdir -p $O
for L in 9000 12300 20004 65536; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,4096,16384,16777216 --unrolls 0 --rounds 5 --steps 10 > $O/len$L.jsonl 2>>$O/err
done
