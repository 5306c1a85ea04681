#!/bin/bash
# Uniform batches across sizes: the auto plan against every shape that covers the size.
set -e
O=gpurun_out/usz
mkdir -p $O
for L in 40 200 576 1024 2048 3000 4096 6000 8192; do
  timeout -k 10 200 python3 tools/sweep.py --len $L --shapes=-1,2,3,4,5,6,7,8,9,12,13 --blocks 0 --unrolls 0 --rounds 3 --steps 10 > $O/len$L.jsonl 2>>$O/err
done
