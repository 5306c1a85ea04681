#!/bin/bash
# Byte-granular (M1) uniform batches: the 4096-workgroup default against larger grids.
set -e
O=gpurun_out/grid_m1
mkdir -p $O
for L in 99 577 1499 3001; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --blocks 0,16384,65536,16777216 --unrolls 0,2 --rounds 5 --steps 20 > $O/len$L.jsonl 2>>$O/err
done
